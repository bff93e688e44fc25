"""proxylib memcached (proxylib/memcached/) through the
proxylib C ABI: the reference's TestMemcache cases (proxylib/
proxylib_memcached_test.go:120-732, transcribed as data in
tests/golden/memcache_kat.json) and random text/binary streams against
oracle/memcache_ref.py.  The framing runs on the host (proxylib_memcache.cc);
every request frame's PolicyMatches verdict comes from the GPU batch of its
OnData call (no CPU evaluation path), so the ABI tests are GPU tests.  The
oracle itself is pinned on the CPU against the same fixtures."""
import json

import numpy as np
import pytest

from cilium_amd import _native as N
from kat_util import load
from oracle import memcache_ref as MR
from test_proxylib_abi import F_OK, Conn, _lib, open_module

KAT = load("memcache_kat.json")


def _policy(name, rules, remotes=(1, 3, 4), port=80):
    return {"name": name, "policy": 2, "ingress_per_port_policies": [{"port": port, "rules": [
        {"remote_policies": list(remotes), "l7_proto": "memcache",
         "l7_rules": {"l7_rules": [{"rule": dict(r)} for r in rules]}}]}]}


def _oracle_matches(rules, remotes=(1, 3, 4), remote=1):
    """PolicyMatches for a port with one rule: no L7 rules on the port →
    allowed from anyone (PortNetworkPolicyRules.Matches, policymap.go:150-158);
    else the remote set, then an OR over the L7 rules (:91-111)."""
    rs = [MR.Rule(dict(r)) for r in rules]
    return lambda m: not rs or (remote in remotes and any(r.matches(m) for r in rs))


def _check_buf(got: bytes, want: bytes):
    """checkBuf (helpers_test.go:101-110): the expected bytes truncated to
    the buffer's length."""
    if len(got) < len(want):
        want = want[:len(got)]
    return got == want


def test_oracle_pinned_on_reference_cases():
    for case in KAT["cases"]:
        conn = MR.Connection(_oracle_matches(case["rules"]), KAT["buf_cap"])
        for c in case["calls"]:
            rc, ops = conn.on_data(c["reply"], [bytes.fromhex(x) for x in c["chunks"]], 1 + 2 * len(c["ops"]))
            assert rc == MR.F_OK and [list(o) for o in ops] == c["ops"], case["name"]
            assert _check_buf(bytes(conn.reply_buf), bytes.fromhex(c["inject"])), case["name"]
            conn.reply_buf.clear()


def test_oracle_go_helpers():
    assert MR.go_fields(b" a\tb\x0bc\xc2\xa0d\xe2\x80\x83e\xc2") == [b"a", b"b", b"c", b"d", b"e\xc2"]
    assert MR.go_fields(b"a\xc0\xa0b") == [b"a\xc0\xa0b"]  # overlong NBSP is not a space
    assert [MR.go_atoi(x) for x in (b"5", b"+5", b"-5", b"", b"-", b"5x", b"9223372036854775808")] == \
        [5, 5, -5, None, None, None, None]


def test_translation_rules():
    """L7RuleParser's ParseError cases (parser.go:114-148) through
    cg_proxylib_policy_update."""
    inst = open_module([(b"node-id", b"cpu-memcache")], "-1")
    assert inst != 0

    def upd(rules):
        t = json.dumps([_policy("m", rules)]).encode()
        return N.lib.cg_proxylib_policy_update(inst, t, len(t))

    assert upd([{"command": "get", "keyExact": "a"}]) == N.CG_OK
    assert upd([{"command": "storage", "keyPrefix": "a"}, {"command": "writeGroup", "keyRegex": "^b+$"}]) == N.CG_OK
    assert upd([{"command": "tap-flush"}, {}]) == N.CG_OK
    assert upd([{"command": "no-such-command"}]) == N.CG_OK  # unknown command, no key: empty rule
    for bad in ([{"keyExact": "a"}], [{"command": "nope", "keyPrefix": "a"}], [{"command": "get", "key": "a"}],
                [{"keyRegex": ""}]):
        assert upd(bad) == N.CG_POLICY_REJECTED, bad
    _lib.CloseModule(inst)


@pytest.mark.gpu
def test_gpu_memcache_reference_cases():
    inst = open_module([(b"node-id", b"gpu-memcache")], "0")
    assert inst != 0
    for case in KAT["cases"]:
        t = json.dumps([_policy("bm1", case["rules"])]).encode()
        assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK, case["name"]
        c = Conn(inst, proto=b"memcache", src=1, dst=2, policy=b"bm1", buf_cap=KAT["buf_cap"])
        assert c.rc == F_OK
        for call in case["calls"]:
            rc, ops = c.on_data([bytes.fromhex(x) for x in call["chunks"]], reply=call["reply"],
                                cap=1 + 2 * len(call["ops"]))
            assert rc == F_OK and [list(o) for o in ops] == call["ops"], case["name"]
            assert _check_buf(c.take_reply(), bytes.fromhex(call["inject"])), case["name"]
        c.close()
    _lib.CloseModule(inst)


# ---- random streams
KEYS = [b"key1", b"key2", b"Hello", b"user:1", b"user:22", b"x", b"a:b:c"]
BIN_KEYS = KEYS + [b"k\x00y", b"\x01\x02", b"k\x03\x14", b"", b"\x03"]
TEXT_CMDS = ["get", "gets", "gat", "gats", "set", "add", "cas", "append", "delete", "incr", "decr", "touch",
             "slabs", "stats", "version", "flush_all", "watch", "quit", "lru_crawler"]


def _rand_rules(rng):
    names = ["get", "gat", "set", "storage", "writeGroup", "delete", "touch", "incr", "stats", "flush_all",
             "version", "slabs", "noop", "quit", "rget", "lru_crawler", "watch"]
    rules = []
    for _ in range(int(rng.integers(0, 4))):
        r = {"command": names[int(rng.integers(len(names)))]}
        k = int(rng.integers(0, 5))
        if k == 1:
            r["keyExact"] = KEYS[int(rng.integers(len(KEYS)))].decode()
        elif k == 2:
            r["keyPrefix"] = ["user:", "key", "H", "a:b"][int(rng.integers(4))]
        elif k == 3:
            r["keyRegex"] = ["^user:[0-9]+$", "ey", "^.el.o$", "[0-9]$", ":"][int(rng.integers(5))]
        rules.append(r)
    return rules


def _text_request(rng):
    cmd = TEXT_CMDS[int(rng.integers(len(TEXT_CMDS)))]
    key = lambda: KEYS[int(rng.integers(len(KEYS)))]
    nr = [b" noreply"] if rng.random() < 0.3 else []
    c = cmd.encode()
    if cmd.startswith("get"):
        return b" ".join([c] + [key() for _ in range(int(rng.integers(0, 4)))]) + b"\r\n"
    if cmd.startswith("gat"):
        return b" ".join([c, b"5"] + [key() for _ in range(int(rng.integers(1, 3)))]) + b"\r\n"
    if cmd in ("set", "add", "cas", "append"):
        val = bytes(rng.integers(97, 123, int(rng.integers(0, 12))).astype(np.uint8))
        head = [c, key(), b"0", b"0", str(len(val)).encode()] + ([b"77"] if cmd == "cas" else [])
        return b" ".join(head + nr) + b"\r\n" + val + b"\r\n"
    if cmd == "delete":
        return b" ".join([c, key()] + nr) + b"\r\n"
    if cmd in ("incr", "decr", "touch"):
        return b" ".join([c, key(), b"5"] + nr) + b"\r\n"
    if cmd == "flush_all":
        return b" ".join([c] + nr) + b"\r\n"
    if cmd == "slabs":
        return b"slabs automove 1\r\n"
    if cmd == "lru_crawler":
        return b"lru_crawler metadump all\r\n"
    if cmd in ("stats", "version", "quit"):
        return c + b"\r\n"
    if cmd == "watch":
        return b"watch mutations\r\n"
    raise AssertionError(cmd)


TEXT_REPLIES = [b"STORED\r\n", b"NOT_FOUND\r\n", b"END\r\n", b"VALUE key1 0 1\r\nx\r\nEND\r\n", b"ERROR\r\n",
                b"OK\r\n", b"DELETED\r\n", b"VERSION 1.6\r\n", b"STAT pid 1\r\nEND\r\n"]


def _bin_frame(rng, request=True):
    key = BIN_KEYS[int(rng.integers(len(BIN_KEYS)))] if request else b""
    extras = bytes(int(rng.integers(0, 8)) * [7])
    val = bytes(rng.integers(0, 256, int(rng.integers(0, 6))).astype(np.uint8))
    op = int(rng.choice([0, 1, 2, 4, 5, 9, 10, 12, 16, 17, 28, 29, 48, 71, 99]))
    magic = 0x80 if request else 0x81
    body = len(extras) + len(key) + len(val)
    hdr = bytes([magic, op]) + len(key).to_bytes(2, "big") + bytes([len(extras), 0, 0, 0]) + \
        body.to_bytes(4, "big") + bytes(12)
    return hdr + extras + key + val


def _chunks(rng, data: bytes):
    cuts = sorted(set(int(x) for x in rng.integers(0, len(data) + 1, int(rng.integers(0, 3)))))
    parts, prev = [], 0
    for c in cuts + [len(data)]:
        parts.append(data[prev:c])
        prev = c
    return [p for p in parts if p] if rng.random() < 0.9 else parts


def _stream(rng, binary: bool, n_calls: int):
    """(reply, bytes appended to that direction) per call."""
    out = []
    for _ in range(n_calls):
        reply = rng.random() < 0.35
        k = int(rng.integers(0, 4))
        if binary:
            data = b"".join(_bin_frame(rng, not reply) for _ in range(k))
            if rng.random() < 0.15:
                data += _bin_frame(rng, not reply)[:int(rng.integers(1, 26))]
        else:
            data = b"".join((TEXT_REPLIES[int(rng.integers(len(TEXT_REPLIES)))] if reply else _text_request(rng))
                            for _ in range(k))
            if rng.random() < 0.1:
                data += (b"bogus cmd\r\n" if rng.random() < 0.5 else b"\r\n")
        out.append((reply, data))
    return out


def _run_streams(inst, rng, binary, rules, remotes, policy=b"rp", n_conns=8):
    """Random streams on fresh connections, each call checked against the
    oracle (ops, result, injected reply bytes).  Returns (request frames,
    denied frames)."""
    n_frames = n_denied = 0
    for _ in range(n_conns):
        remote = int(rng.choice([1, 3, 5]))
        cap_buf = int(rng.choice([30, 40, 1024]))
        c = Conn(inst, proto=b"memcache", src=remote, dst=2, policy=policy, buf_cap=cap_buf)
        assert c.rc == F_OK
        o = MR.Connection(_oracle_matches(rules, remotes, remote) if rules is not None else (lambda m: False),
                          cap_buf)
        pend = {False: b"", True: b""}
        for reply, data in _stream(rng, binary, 12):
            pend[reply] += data
            cap = int(rng.integers(1, 10))
            chunks = _chunks(rng, pend[reply])
            want_rc, want_ops = o.on_data(reply, chunks, cap)
            rc, ops = c.on_data(chunks, reply=reply, cap=cap)
            ctx = (rules, remote, reply, chunks, cap)
            assert (rc, ops) == (want_rc, [tuple(x) for x in want_ops]), ctx
            assert c.take_reply() == bytes(o.reply_buf), ctx
            o.reply_buf.clear()
            if rc != F_OK:
                break
            used = sum(n for op, n in ops if op in (MR.PASS, MR.DROP) and n > 0)
            n_frames += sum(1 for op, _ in ops if op in (MR.PASS, MR.DROP) and not reply)
            n_denied += sum(1 for op, _ in ops if op == MR.DROP)
            pend[reply] = pend[reply][used:]
        c.close()
    return n_frames, n_denied


@pytest.mark.parametrize("binary", [False, True])
def test_framing_random_streams_no_policy(binary):
    """The host framing alone: a connection whose policy name is not
    installed is denied every request without a GPU batch (PolicyMatches
    false), so text and binary framing, reply tracking, denial injection and
    the op loop are checked against the oracle on the CPU."""
    inst = open_module([(b"node-id", b"cpu-memcache-frames")], "-1")
    assert inst != 0
    rng = np.random.default_rng(5 + binary)
    n_frames, n_denied = _run_streams(inst, rng, binary, None, (), policy=b"not-installed", n_conns=120)
    assert n_frames > 150 and n_denied == n_frames
    _lib.CloseModule(inst)


@pytest.mark.gpu
@pytest.mark.parametrize("binary", [False, True])
def test_gpu_memcache_random_streams_vs_oracle(binary):
    inst = open_module([(b"node-id", b"gpu-memcache-rand")], "0")
    assert inst != 0
    rng = np.random.default_rng(71 + binary)
    n_frames = n_denied = 0
    for pol_i in range(6):
        rules = _rand_rules(rng)
        remotes = (1, 3, 4) if pol_i % 3 else (5,)
        t = json.dumps([_policy("rp", rules, remotes)]).encode()
        assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK, rules
        f, d = _run_streams(inst, rng, binary, rules, remotes)
        n_frames += f
        n_denied += d
    assert n_frames > 100 and 0 < n_denied < n_frames
    _lib.CloseModule(inst)


# ---- Rule.Matches in bulk: the compiled list matchers against the oracle
KEY_ALPHA = np.frombuffer(b"keyHlo:user0123ab\x00\x01\x02\x03\x14 ", np.uint8)


def _rand_meta(rng):
    if rng.random() < 0.5:
        cmd = bytes(rng.choice([b"get", b"gets", b"gat", b"set", b"cas", b"incr", b"delete", b"touch", b"stats",
                                b"flush_all", b"watch", b"getx", b"lru_crawler", b"slabs", b"version"]))
        op = 0
    else:
        cmd, op = b"", int(rng.integers(0, 80))
    keys = []
    for _ in range(int(rng.integers(0, 4))):
        if rng.random() < 0.5:
            keys.append(KEYS[int(rng.integers(len(KEYS)))])
        else:
            keys.append(KEY_ALPHA[rng.integers(0, len(KEY_ALPHA), int(rng.integers(0, 9)))].tobytes())
    return cmd, op, keys


def _check_metas(cl, seed, n, gpu):
    from cilium_amd import proxylib as P
    rng = np.random.default_rng(seed)
    pols, oracles = [], []
    for i in range(4):
        rules = _rand_rules(rng) + _rand_rules(rng)
        remotes = (1, 3, 4) if i % 2 else (2,)
        pols.append(_policy(f"m{i}", rules, remotes))
        oracles.append((rules, remotes))
    pl = P.ProxylibPolicy(cl)
    pl.update(pols)
    metas = [_rand_meta(rng) for _ in range(n)]
    pi = rng.integers(0, 4, n)
    rem = rng.choice([1, 2, 3, 7], n)
    fields = [P.memcache_request(*m) for m in metas]
    got = pl.matches_fields([pl.index(f"m{i}") for i in pi], [1] * n, [80] * n, rem.tolist(), fields,
                            host_diag=not gpu)
    ms = {}
    exp = []
    for (cmd, op, keys), i, r in zip(metas, pi, rem):
        key = (int(i), int(r))
        if key not in ms:
            ms[key] = _oracle_matches(oracles[i][0], oracles[i][1], int(r))
        exp.append(int(ms[key](MR.Meta(cmd, op, keys))))
    assert got.tolist() == exp
    assert 0 < sum(exp) < n


@pytest.mark.parametrize("seed", range(3))
def test_rule_matches_tables_vs_oracle(host, seed):
    _check_metas(host, seed, 3000, gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(2))
def test_gpu_rule_matches_vs_oracle(gpu, seed):
    _check_metas(gpu, 50 + seed, 20000, gpu=True)
