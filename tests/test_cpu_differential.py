"""Randomized differential tests on the CPU: the engine's compilers (regex →
DFA, NPDS → union DFAs, Kafka rule compiler, L4/LPM table builders), walked
by the host diagnostic walkers, against the oracle on seeded random inputs.
The GPU kernels are checked against the same oracle in test_gpu_parity.py."""
import ctypes as C
import random

import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import synth

# ------------------------------------------------------------------ regex ---
ATOMS = ["a", "b", "c", "x", "/", ".", "[a-c]", "[^ab]", "[^]", "[]", "\\d", "\\w", "\\s", "\\W", "\\D", "\\S",
         "(a|b)", "(?:ab|c|)", "[0-9x-z]", "\\.", "\\/", "\\x41", "[\\d\\s]", "()", "(a*)", "\\t", "\\-", "[-a]",
         "[a-]", "\\r", "\\n", "]", "}", "\\u0062"]
QUANTS = ["", "", "", "*", "+", "?", "{0,1}", "{1,3}", "{2}", "{2,}", "*?", "+?", "??", "{1,2}?"]
ALPHA = ["a", "b", "c", "x", "y", "/", ".", "1", "9", " ", "\t", "\n", "\r", "-", "_", "A", "B", "]", "}", "\x80",
         "\xff", "\x00", "\x01"]


def _rand_regex(rng, depth=0):
    k = rng.randint(1, 4)
    parts = []
    for _ in range(k):
        if depth < 2 and rng.random() < 0.15:
            parts.append("(" + _rand_regex(rng, depth + 1) + ")" + rng.choice(QUANTS))
        else:
            parts.append(rng.choice(ATOMS) + rng.choice(QUANTS))
    r = "".join(parts)
    if rng.random() < 0.2:
        r = r + "|" + _rand_regex(rng, depth + 1) if depth < 2 else r
    if rng.random() < 0.1:
        r = "^" + r
    if rng.random() < 0.1:
        r = r + "$"
    return r


def _engine_match(p: bytes, s: bytes, search: bool):
    res = C.c_uint8()
    buf = np.frombuffer(s, np.uint8) if s else np.zeros(1, np.uint8)
    rc = N.lib.cg_diag_regex_match(p, len(p), buf.ctypes.data, len(s), 1 if search else 0, C.byref(res))
    return -1 if rc != 0 else res.value


def test_regex_random_vs_std_regex():
    """Full match vs std::regex_match (Envoy's engine).  Search mode is Go's
    regexp (tests/test_regex_flavours.py)."""
    rng = random.Random(1234)
    checked = 0
    for _ in range(400):
        p = _rand_regex(rng).encode("latin-1")
        valid = oracle.regex_match(p, b"") != -1
        e = _engine_match(p, b"", False)
        assert (e != -1) == valid, p
        if not valid:
            continue
        for _ in range(30):
            s = "".join(rng.choice(ALPHA) for _ in range(rng.randint(0, 8))).encode("latin-1")
            assert _engine_match(p, s, False) == oracle.regex_match(p, s), (p, s)
            checked += 1
    assert checked > 4000


GO_ATOMS = [a for a in ATOMS if a not in ("[^]", "[]", "\\u0062", "[\\d\\s]")] + ["\\v", "[\\r\\n]"]


def test_regex_search_vs_go_flavour():
    """Search mode against the Go regexp restatement (oracle/go_regexp_ref.py)
    on the ASCII syntax subset and strings with CR, VT, NUL and high bytes
    (each high byte an invalid rune: U+FFFD)."""
    from oracle.go_regexp_ref import GoRegexp, GoSyntaxError
    rng = random.Random(77)
    alpha = ALPHA + ["\v", "\f"]
    checked = 0
    for _ in range(400):
        r = "".join(rng.choice(GO_ATOMS) + rng.choice(QUANTS) for _ in range(rng.randint(1, 4)))
        p = r.encode("latin-1")
        try:
            g = GoRegexp(p)
        except GoSyntaxError:
            assert _engine_match(p, b"", True) == -1, r
            continue
        for _ in range(30):
            s = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 8))).encode("latin-1")
            assert _engine_match(p, s, True) == int(g.match_string(s)), (r, s)
            checked += 1
    assert checked > 5000


# ------------------------------------------------------------------- HTTP ---
HDR_NAMES = [":path", ":method", ":authority", "x-a", "X-B", "x-c"]
VALUES = ["/", "/a", "/ab", "/public", "/x/y", "GET", "PUT", "POST", "h1", "h2.example.com", "true", "True", "", "zz"]


def _rand_matcher(rng):
    name = rng.choice(HDR_NAMES)
    kind = rng.random()
    if kind < 0.4:
        return {"name": name, "exact_match": rng.choice(VALUES)}
    if kind < 0.8:
        return {"name": name, "regex_match": rng.choice(["/a.*", ".*b", "G.T", "P(UT|OST)", "[a-z]+", "h[0-9]",
                                                         "/[a-z]*/?y?", ".*", "", "x|/", "T?r.e"])}
    if kind < 0.9:
        return {"name": name, "present_match": True}
    return {"name": name, "value": rng.choice(VALUES), "regex": rng.random() < 0.5}


# remote identity universes: a dense span (the kernel's direct identity → row
# array) and one spread past kRdirMaxSpan (the 2-choice bucket table)
ID_SETS = {"dense": [1, 2, 3, 4], "spread": [1, 2, 70000, 16777300]}


def _rand_policy(rng, n_pol=3, ids=(1, 2, 3, 4)):
    pols = []
    for pi in range(n_pol):
        p = {"name": f"p{pi}", "policy": pi}
        for key in ("ingress_per_port_policies", "egress_per_port_policies"):
            if rng.random() < 0.2:
                continue
            ports = rng.sample([0, 80, 81, 8080], rng.randint(0, 3))
            lst = []
            for port in ports:
                rules = []
                for _ in range(rng.randint(0, 3)):
                    r = {"remote_policies": sorted(rng.sample(list(ids), rng.randint(0, 2)))}
                    if rng.random() < 0.85:
                        r["http_rules"] = {"http_rules": [
                            {"headers": [_rand_matcher(rng) for _ in range(rng.randint(0, 3))]}
                            for _ in range(rng.randint(0, 3))]}
                    rules.append(r)
                lst.append({"port": port, "protocol": "UDP" if rng.random() < 0.1 else "TCP", "rules": rules})
            p[key] = lst
        pols.append(p)
    return pols


def _rand_requests(rng, n, n_pol, ids=(1, 2, 3, 4)):
    reqs = []
    for _ in range(n):
        hs = []
        for name in HDR_NAMES:
            if rng.random() < 0.7:
                hs.append((name.upper() if rng.random() < 0.2 else name, rng.choice(VALUES)))
        if rng.random() < 0.1 and hs:
            hs.append((hs[0][0], "dup"))  # repeated header: the first value wins
        if rng.random() < 0.2:  # a header no rule references
            hs.append(("x-unref", rng.choice(VALUES)))
        if rng.random() < 0.05 and hs:
            # a control byte the codec rejects (any header) → denied; HTAB is fine
            k = rng.randrange(len(hs))
            c = rng.choice(["\x01", "\x02", "\x07", "\x1f", "\x7f", "\t", "\r"])
            hs[k] = (hs[k][0], hs[k][1] + c)
        reqs.append(hs)
    parts, off = [], [0]
    for hs in reqs:
        b = b"".join(k.encode() + b"\0" + v.encode() + b"\0" for k, v in hs)
        parts.append(b)
        off.append(off[-1] + len(b))
    return dict(policy=np.array([rng.randint(0, n_pol) for _ in range(n)], np.uint32),  # n_pol = unknown
                ingress=np.array([rng.randint(0, 1) for _ in range(n)], np.uint8),
                port=np.array([rng.choice([80, 81, 8080, 9]) for _ in range(n)], np.uint16),
                remote=np.array([rng.choice([0, 5] + list(ids)) for _ in range(n)], np.uint32),
                hdr_blob=np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy(),
                hdr_off=np.array(off, np.uint64))


@pytest.mark.parametrize("ids", sorted(ID_SETS))
@pytest.mark.parametrize("seed", range(12))
def test_http_random_policies(host, seed, ids):
    rng = random.Random(seed)
    pols = _rand_policy(rng, ids=ID_SETS[ids])
    rq = _rand_requests(rng, 600, len(pols), ids=ID_SETS[ids])
    try:
        orc = oracle.HttpOracle(pols)
    except ValueError:
        with pytest.raises(N.CiliumGPUError):
            host.update_http_policy(pols)
        return
    host.update_http_policy(pols)
    b = host.pack_http(**rq)
    assert np.array_equal(host.http_eval_host_diag(b), orc.eval(**rq))


NUM_VALUES = ["0", "5", "-5", "+12", "007", "-0", "12a", "", " 5", "\t7", "+", "-", "99",
              "9223372036854775807", "9223372036854775808", "-9223372036854775808", "-9223372036854775809",
              "000000000000000000000000000042", "1e3"]
RANGES = [(0, 10), (-10, 0), (5, 6), (-9223372036854775808, 9223372036854775807), (100, 50), (-3, 13), (10, 100),
          (-9223372036854775808, -1), (9223372036854775806, 9223372036854775807), (0, 0)]


def _rand_matcher_ext(rng):
    """Every HeaderMatcher form of route.pb.go:3185-3198 Envoy evaluates:
    exact (empty = presence), regex, present, prefix, suffix, range, each
    optionally inverted."""
    name = rng.choice(HDR_NAMES)
    k = rng.random()
    vals = VALUES + NUM_VALUES
    if k < 0.15:
        m = {"name": name, "exact_match": rng.choice(vals)}
    elif k < 0.3:
        m = {"name": name, "regex_match": rng.choice(["/a.*", ".*b", "[0-9]+", "-?[0-9]", ".*", ""])}
    elif k < 0.4:
        m = {"name": name, "present_match": True}
    elif k < 0.55:
        m = {"name": name, "prefix_match": rng.choice(["", "/", "/a", "G", "9", "-", "h2"])}
    elif k < 0.7:
        m = {"name": name, "suffix_match": rng.choice(["", "b", "com", "ue", "7", "5", "/"])}
    else:
        a, b = rng.choice(RANGES)
        m = {"name": name, "range_match": {"start": a, "end": b}}
    if rng.random() < 0.3:
        m["invert_match"] = True
    return m


def all_matcher_case(seed: int, n: int = 1500):
    """Random policies over every matcher form and requests with numeric
    and textual values: (policies, request arrays, request header lists)."""
    rng = random.Random(900 + seed)
    pols = []
    for pi in range(3):
        p = {"name": f"p{pi}", "policy": pi, "ingress_per_port_policies": [], "egress_per_port_policies": []}
        for key in ("ingress_per_port_policies", "egress_per_port_policies"):
            for port in rng.sample([0, 80, 81], rng.randint(1, 3)):
                rules = []
                for _ in range(rng.randint(1, 3)):
                    r = {"remote_policies": sorted(rng.sample([1, 2, 3, 4], rng.randint(0, 2))),
                         "http_rules": {"http_rules": [{"headers": [_rand_matcher_ext(rng)
                                                                    for _ in range(rng.randint(1, 3))]}
                                                       for _ in range(rng.randint(1, 3))]}}
                    rules.append(r)
                p[key].append({"port": port, "protocol": "TCP", "rules": rules})
        pols.append(p)
    reqs = []
    for _ in range(n):
        reqs.append([(nm, rng.choice(VALUES + NUM_VALUES)) for nm in HDR_NAMES if rng.random() < 0.75])
    parts, off = [], [0]
    for hs in reqs:
        b = b"".join(k.encode() + b"\0" + v.encode() + b"\0" for k, v in hs)
        parts.append(b)
        off.append(off[-1] + len(b))
    rq = dict(policy=np.array([rng.randint(0, 3) for _ in range(n)], np.uint32),
              ingress=np.array([rng.randint(0, 1) for _ in range(n)], np.uint8),
              port=np.array([rng.choice([80, 81, 9]) for _ in range(n)], np.uint16),
              remote=np.array([rng.choice([0, 1, 2, 3, 4]) for _ in range(n)], np.uint32),
              hdr_blob=np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy(),
              hdr_off=np.array(off, np.uint64))
    return pols, rq, reqs


@pytest.mark.parametrize("seed", range(10))
def test_http_random_policies_all_matchers(host, seed):
    """prefix / suffix / range / invert / empty-exact matchers compiled into
    the union DFAs (http.cc, regex.cc dfa_suffix / dfa_int_range /
    dfa_complement) against the oracle's restatement of Envoy's matchHeaders
    (oracle.cc match_header; strtol for ranges)."""
    pols, rq, reqs = all_matcher_case(seed)
    host.update_http_policy(pols)
    b = host.pack_http(**rq)
    want = oracle.HttpOracle(pols).eval(**rq)
    got = host.http_eval_host_diag(b)
    bad = np.nonzero(got != want)[0]
    assert not len(bad), [(i, reqs[i], int(got[i]), int(want[i])) for i in bad[:5]]
    assert 0.05 < want.mean() < 0.95


def test_http_10k_compile_and_overflow(host):
    pols, info = synth.http10k_rules()
    rq = synth.http10k_requests(20_000, info)
    host.update_http_policy(pols)
    st = host.http_policy_stats()
    assert st["rules"] == 10_000 and st["programs"] == 64
    b = host.pack_http(**rq)
    assert np.array_equal(host.http_eval_host_diag(b), oracle.HttpOracle(pols).eval(**rq, nthreads=4))


def test_http_long_fields_overflow(host):
    pols = synth.starwars_policy()
    host.update_http_policy(pols)
    rq = synth.starwars_requests(500, seed=3)
    blob, off = rq["hdr_blob"].tobytes(), rq["hdr_off"]
    parts = []
    for i in range(len(off) - 1):
        b = blob[off[i]:off[i + 1]]
        if i % 2:
            b = b.replace(b"/v1/", b"/v1/" + b"q" * (100 + i), 1)
        parts.append(b)
    rq["hdr_blob"] = np.frombuffer(b"".join(parts), np.uint8).copy()
    rq["hdr_off"] = np.concatenate([[0], np.cumsum([len(p) for p in parts])]).astype(np.uint64)
    b = host.pack_http(**rq)
    assert b.arena.nbytes > 16
    assert np.array_equal(host.http_eval_host_diag(b), oracle.HttpOracle(pols).eval(**rq))


# ------------------------------------------------------------------ Kafka ---
@pytest.mark.parametrize("seed", range(4))
def test_kafka_random(host, seed):
    pols, info = synth.kafka_policy(n_rules=300, n_topics=50, n_clients=10, seed=seed)
    rq = synth.kafka_requests(20_000, info, seed=seed)
    host.update_kafka_policy(pols)
    reqs, arena = host.pack_kafka(**rq)
    assert np.array_equal(host.kafka_eval_host_diag(reqs, arena), oracle.KafkaOracle(pols).eval(**rq))


def test_kafka_many_topics_overflow(host):
    pols, info = synth.kafka_policy(n_rules=200, n_topics=20, n_clients=4)
    host.update_kafka_policy(pols)
    rng = random.Random(5)
    n = 300
    rq = dict(redirect=[0] * n, remote=[rng.choice(info["ids"] + [0]) for _ in range(n)],
              api_key=[rng.choice([0, 1, 3]) for _ in range(n)], api_version=[0] * n, kind=[1] * n,
              client_id=[b"client-1"] * n,
              topics=[[info["topics"][rng.randrange(20)].encode() for _ in range(rng.randint(0, 30))]
                      for _ in range(n)])
    reqs, arena = host.pack_kafka(**rq)
    assert np.array_equal(host.kafka_eval_host_diag(reqs, arena), oracle.KafkaOracle(pols).eval(**rq))


def _kafka_edge_policy(rng):
    from cilium_amd.policy import KAFKA_API_KEY_MAP, PortRuleKafka
    keys = list(KAFKA_API_KEY_MAP)
    topics = [f"t{i}" for i in range(6)]
    clients = ["c0", "c1", "c2"]

    def rule():
        r = PortRuleKafka()
        pick = rng.random()
        if pick < 0.3:
            r.APIKey = rng.choice(keys)
        elif pick < 0.5:
            r.Role = rng.choice(["produce", "consume"])
        # else apiKey wildcard
        if rng.random() < 0.4:
            r.APIVersion = str(rng.choice([0, 1, 5, 63, 64, 100, -1, 32767, -32768]))
        if rng.random() < 0.3:
            r.ClientID = rng.choice(clients)
        if rng.random() < 0.4:
            r.Topic = rng.choice(topics)
        return r

    sels = [{"identities": [7, 8], "rules": [rule() for _ in range(rng.randint(0, 6))]},
            {"identities": [8, 9], "rules": [rule() for _ in range(rng.randint(1, 6))]},
            {"identities": [10], "rules": []},
            {"identities": None, "rules": [rule() for _ in range(rng.randint(0, 2))]}]
    return [{"name": "r0", "selectors": sels}, {"name": "r1", "selectors": sels[1:3]}], topics, clients


@pytest.mark.parametrize("seed", range(12))
def test_kafka_edge_rules(host, seed):
    """Versions outside 0..63 and negative, apiKey-wildcard rules with topics
    and clientIDs, unknown apiKeys (negative, > 63) and request kinds: the
    summary bits, exception rules and topic lists against the oracle."""
    rng = random.Random(seed)
    pols, topics, clients = _kafka_edge_policy(rng)
    host.update_kafka_policy(pols)
    n = 3000
    rq = dict(redirect=[rng.choice([0, 0, 1, 2]) for _ in range(n)],
              remote=[rng.choice([0, 7, 8, 9, 10, 11]) for _ in range(n)],
              api_key=[rng.choice([0, 1, 3, 10, 12, 18, 37, -1, 40, 63, 64, 1000]) for _ in range(n)],
              api_version=[rng.choice([0, 1, 5, 63, 64, 100, -1, 32767, -32768]) for _ in range(n)],
              kind=[rng.choice([0, 1, 2, 3]) for _ in range(n)],
              client_id=[rng.choice(clients + ["zz"]).encode() for _ in range(n)],
              topics=[[rng.choice(topics + ["nope"]).encode() for _ in range(rng.choice([0, 0, 1, 2, 3]))]
                      for _ in range(n)])
    reqs, arena = host.pack_kafka(**rq)
    assert np.array_equal(host.kafka_eval_host_diag(reqs, arena), oracle.KafkaOracle(pols).eval(**rq))


# ---------------------------------------------------------------- L4, LPM ---
def test_l4_table_builder(host):
    keys, ports = synth.l4_table(n_entries=16384)
    pm = host.policy_map()
    pm.allow_keys(keys, ports)
    t = synth.l4_tuples(200_000, keys)
    assert np.array_equal(pm.eval_host_diag(t), oracle.l4(keys, ports, t)[0])


@pytest.mark.parametrize("cfg", [(True, True), (False, False), (True, False)])
def test_prefilter_table_builder(host, cfg):
    dyn4, dyn6 = cfg
    pfx = synth.lpm_prefixes(40_000, 20_000, seed=11)
    keep = ((pfx["family"] == 4) & ((pfx["prefixlen"] == 32) | dyn4)) | \
           ((pfx["family"] == 6) & ((pfx["prefixlen"] == 128) | dyn6))
    pfx = pfx[keep]
    pf = host.prefilter(dyn4=dyn4, dyn6=dyn6, max_lpm=1 << 20)
    pf.insert(0, pfx)
    v4, v6, ep4, ep6 = synth.lpm_addresses(100_000, synth.lpm_prefixes(40_000, 20_000, seed=11), seed=5)
    pf.set_endpoints(ep4, ep6)
    g4, g6 = pf.eval_host_diag(v4, v6)
    o4, o6 = oracle.prefilter(pf.config, pfx, ep4, ep6, v4, v6)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6)


def dense_prefilter_case(seed: int, n: int = 50_000):
    """Dense partial /24 blocks (so group ranks add up over many partial
    blocks), v6 buckets with many intervals (binary-search fallback), and the
    all-zero addresses as endpoints (the probe tables' empty-slot flags)."""
    from cilium_amd.classifier import CIDR_DTYPE
    rng = np.random.default_rng(seed)
    m4, m6 = 6000, 3000
    pfx = np.zeros(m4 + m6, CIDR_DTYPE)
    plen4 = rng.integers(25, 33, m4)
    a4 = (0x0A000000 | rng.integers(0, 1 << 18, m4)).astype(np.uint32)  # 10.0.0.0/14
    a4 &= ((0xFFFFFFFF << (32 - plen4)) & 0xFFFFFFFF).astype(np.uint32)
    pfx["family"][:m4] = 4
    pfx["prefixlen"][:m4] = plen4
    pfx["addr"][:m4, :4] = a4.astype(">u4").view(np.uint8).reshape(-1, 4)
    plen6 = rng.integers(40, 129, m6)
    a6 = np.zeros((m6, 16), np.uint8)
    a6[:, 0], a6[:, 1] = 0x20, 0x01  # everything under 2001::/16: one crowded top-bits bucket range
    a6[:, 2:] = rng.integers(0, 256, (m6, 14), dtype=np.uint8)
    a6[:, 2] &= 0x03
    for i in range(16):
        keep = np.clip(plen6 - 8 * i, 0, 8)
        a6[:, i] &= ((0xFF << (8 - keep)) & 0xFF).astype(np.uint8)
    pfx["family"][m4:] = 6
    pfx["prefixlen"][m4:] = plen6
    pfx["addr"][m4:] = a6
    v4 = np.zeros((n, 2), np.uint32)
    s4 = np.where(rng.random(n) < 0.8, 0x0A000000 | rng.integers(0, 1 << 18, n),
                  rng.integers(0, 1 << 32, n, dtype=np.uint64)).astype(np.uint32)
    v4[:, 0] = s4.astype(">u4").view("<u4")
    ep4 = np.concatenate([[0], rng.integers(1, 1 << 32, 500, dtype=np.uint64)]).astype(np.uint32)
    v4[:, 1] = np.where(rng.random(n) < 0.5, ep4[rng.integers(0, len(ep4), n)], 0)
    v6 = np.zeros((n, 32), np.uint8)
    v6[:, :16] = a6[rng.integers(0, m6, n)]
    v6[:, 15] ^= rng.integers(0, 256, n, dtype=np.uint8)
    v6[:, 8] ^= np.where(rng.random(n) < 0.3, rng.integers(0, 256, n), 0).astype(np.uint8)
    ep6 = np.concatenate([np.zeros((1, 16), np.uint8), rng.integers(0, 256, (300, 16), dtype=np.uint8)])
    pick = rng.integers(0, len(ep6), n)
    v6[:, 16:] = np.where((rng.random(n) < 0.5)[:, None], ep6[pick], 0)
    return pfx, v4, v6, ep4, ep6


@pytest.mark.parametrize("seed", range(3))
def test_prefilter_dense_partials(host, seed):
    pfx, v4, v6, ep4, ep6 = dense_prefilter_case(seed)
    pf = host.prefilter(dyn4=True, dyn6=True, max_lpm=1 << 20)
    pf.insert(0, pfx)
    pf.set_endpoints(ep4, ep6)
    g4, g6 = pf.eval_host_diag(v4, v6)
    o4, o6 = oracle.prefilter(pf.config, pfx, ep4, ep6, v4, v6)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6)
    assert 0.05 < (o4 == 1).mean() < 0.95 and 0.05 < (o6 == 1).mean() < 0.95


def v6_bucket_case(seed: int):
    """IPv6 bucket classes: short prefixes covering whole top-bits buckets
    (code 1), prefixes ending on bucket edges, the last bucket (ffff::/16),
    ::/0-adjacent ranges and adjacent prefixes that merge, with addresses
    at and beside every interval edge."""
    from cilium_amd.classifier import CIDR_DTYPE
    rng = np.random.default_rng(100 + seed)
    m = 2000
    pfx = np.zeros(m, CIDR_DTYPE)
    plen = np.where(rng.random(m) < 0.05, rng.integers(6, 24, m), rng.integers(24, 129, m))
    a6 = rng.integers(0, 256, (m, 16), dtype=np.uint8)
    a6[:50, :2] = 0xFF  # the last buckets
    a6[50:100, :2] = 0x00  # the first ones
    for i in range(16):
        keep = np.clip(plen - 8 * i, 0, 8)
        a6[:, i] &= ((0xFF << (8 - keep)) & 0xFF).astype(np.uint8)
    pfx["family"] = 6
    pfx["prefixlen"] = plen
    pfx["addr"] = a6
    # addresses: each prefix's first and last address, one past/before them
    lo = a6.copy()
    hi = a6.copy()
    for i in range(16):
        host_bits = np.clip(8 * (i + 1) - plen, 0, 8)
        hi[:, i] |= ((1 << host_bits) - 1).astype(np.uint8)

    def step(x, d):
        v = int.from_bytes(bytes(x), "big") + d
        return list((v % (1 << 128)).to_bytes(16, "big"))
    edges = [lo, hi, np.array([step(x, -1) for x in lo], np.uint8), np.array([step(x, 1) for x in hi], np.uint8)]
    src = np.concatenate(edges + [rng.integers(0, 256, (4 * m, 16), dtype=np.uint8)])
    v6 = np.zeros((len(src), 32), np.uint8)
    v6[:, :16] = src
    v4 = np.zeros((1, 2), np.uint32)
    ep4 = np.zeros(0, np.uint32)
    ep6 = rng.integers(0, 256, (16, 16), dtype=np.uint8)
    v6[:, 16:] = ep6[rng.integers(0, 16, len(src))]  # local destinations: drops come from the CIDRs
    return pfx, v4, v6, ep4, ep6


@pytest.mark.parametrize("seed", range(2))
def test_prefilter_v6_bucket_codes(host, seed):
    pfx, v4, v6, ep4, ep6 = v6_bucket_case(seed)
    pf = host.prefilter(dyn4=True, dyn6=True, max_lpm=1 << 20)
    pf.insert(0, pfx)
    pf.set_endpoints(ep4, ep6)
    g4, g6 = pf.eval_host_diag(v4, v6)
    o4, o6 = oracle.prefilter(pf.config, pfx, ep4, ep6, v4, v6)
    assert np.array_equal(g6, o6)
    assert 0.05 < (o6 == 1).mean() < 0.95
