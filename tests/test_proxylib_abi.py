"""The proxylib C ABI of libciliumgpu.so (include/cilium_proxylib.h): the
symbols Envoy's proxylib filter dlopens (proxylib/libcilium.h:77-115), driven
the way the reference's r2d2 tests drive them (proxylib/r2d2/
r2d2parser_test.go:70-190: CheckInsertPolicyText → CheckNewConnectionOK →
CheckOnDataOK with expected ops and injected reply bytes)."""
import ctypes as C
import json
import os
import re

import pytest

from cilium_amd import _native as N

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "cilium_proxylib.h")
MORE, PASS, DROP = 0, 1, 2
F_OK, F_UNKNOWN_PARSER, F_UNKNOWN_CONNECTION, F_INVALID_ADDRESS, F_INVALID_INSTANCE = 0, 3, 4, 5, 6
F_UNKNOWN_ERROR = 7


class GoString(C.Structure):
    _fields_ = [("p", C.c_char_p), ("n", C.c_ssize_t)]


class GoSlice(C.Structure):
    _fields_ = [("data", C.c_void_p), ("len", C.c_int64), ("cap", C.c_int64)]


class FilterOp(C.Structure):
    _fields_ = [("op", C.c_uint64), ("n_bytes", C.c_int64)]


def gs(b: bytes) -> GoString:
    return GoString(b, len(b))


_lib = C.CDLL(str(N.LIB_PATH))
_lib.OpenModule.restype = C.c_uint64
_lib.OpenModule.argtypes = [GoSlice, C.c_uint8]
_lib.CloseModule.argtypes = [C.c_uint64]
_lib.OnNewConnection.restype = C.c_int
_lib.OnNewConnection.argtypes = [C.c_uint64, GoString, C.c_uint64, C.c_uint8, C.c_uint32, C.c_uint32, GoString,
                                 GoString, GoString, C.POINTER(GoSlice), C.POINTER(GoSlice)]
_lib.OnData.restype = C.c_int
_lib.OnData.argtypes = [C.c_uint64, C.c_uint8, C.c_uint8, C.POINTER(GoSlice), C.POINTER(GoSlice)]
_lib.Close.argtypes = [C.c_uint64]


def open_module(params, device: str):
    os.environ["CILIUM_GPU_DEVICE"] = device
    arr = (GoString * (2 * max(len(params), 1)))()
    for i, (k, v) in enumerate(params):
        arr[2 * i], arr[2 * i + 1] = gs(k), gs(v)
    return _lib.OpenModule(GoSlice(C.cast(arr, C.c_void_p), len(params), len(params)), 0)


class Conn:
    """A connection with caller-owned inject buffers (cap 1024 each)."""
    _next = [1000]

    def __init__(self, inst, proto=b"r2d2", ingress=True, src=1, dst=2, dst_addr=b"2.2.2.2:80", policy=b"cp1",
                 buf_cap=1024):
        self.orig_mem = C.create_string_buffer(buf_cap)
        self.reply_mem = C.create_string_buffer(buf_cap)
        self.orig = GoSlice(C.cast(self.orig_mem, C.c_void_p), 0, buf_cap)
        self.reply = GoSlice(C.cast(self.reply_mem, C.c_void_p), 0, buf_cap)
        Conn._next[0] += 1
        self.id = Conn._next[0]
        self.rc = _lib.OnNewConnection(inst, gs(proto), self.id, ingress, src, dst, gs(b"1.1.1.1:34567"),
                                       gs(dst_addr), gs(policy), C.byref(self.orig), C.byref(self.reply))

    def on_data(self, chunks, reply=False, cap=16):
        bufs = [C.create_string_buffer(c, len(c)) for c in chunks]
        arr = (GoSlice * max(len(chunks), 1))()
        for i, (b, c) in enumerate(zip(bufs, chunks)):
            arr[i] = GoSlice(C.cast(b, C.c_void_p), len(c), len(c))
        data = GoSlice(C.cast(arr, C.c_void_p), len(chunks), len(chunks))
        ops_mem = (FilterOp * cap)()
        ops = GoSlice(C.cast(ops_mem, C.c_void_p), 0, cap)
        rc = _lib.OnData(self.id, reply, 0, C.byref(data), C.byref(ops))
        return rc, [(int(ops_mem[i].op), int(ops_mem[i].n_bytes)) for i in range(ops.len)]

    def injected_reply(self) -> bytes:
        return self.reply_mem.raw[:self.reply.len]

    def take_reply(self) -> bytes:
        """The reply inject buffer's contents, then empty it (CheckOnData)."""
        b = self.injected_reply()
        self.reply.len = 0
        return b

    def close(self):
        _lib.Close(self.id)


def test_symbols_exported():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    names = set(re.findall(r"\b(OnNewConnection|OnData|Close|OpenModule|CloseModule)\s*\(", text))
    assert names == {"OnNewConnection", "OnData", "Close", "OpenModule", "CloseModule"}
    for n in names:
        assert hasattr(_lib, n)


def test_module_and_connection_errors():
    assert open_module([(b"bogus", b"x")], "-1") == 0  # unknown key → 0 (proxylib.go:129-131)
    inst = open_module([(b"node-id", b"cpu-test"), (b"xds-path", b"/tmp/xds")], "-1")
    assert inst != 0
    assert open_module([(b"node-id", b"cpu-test"), (b"xds-path", b"/tmp/xds")], "-1") == inst  # same params
    assert Conn(inst + 999).rc == F_INVALID_INSTANCE
    assert Conn(inst, proto=b"nosuchparser").rc == F_UNKNOWN_PARSER
    assert Conn(inst, dst_addr=b"2.2.2.2").rc == F_INVALID_ADDRESS
    assert Conn(inst, dst_addr=b"2.2.2.2:0").rc == F_INVALID_ADDRESS
    assert Conn(inst, dst_addr=b"2.2.2.2:http").rc == F_INVALID_ADDRESS
    c = Conn(inst)
    assert c.rc == F_OK
    # reply direction: frames pass without a verdict (r2d2parser.go:160-162)
    assert c.on_data([b"OK abc\r\nERR", b"OR\r\n"], reply=True) == (F_OK, [(PASS, 8), (PASS, 7), (MORE, 1)])
    # partial request: MORE 1, no verdict needed
    assert c.on_data([b"REA"]) == (F_OK, [(MORE, 1)])
    # ops capacity bounds the frames handled in one call (connection.go:141)
    assert c.on_data([b"OK\r\n" * 5], reply=True, cap=3) == (F_OK, [(PASS, 4)] * 3)
    c.close()
    rc, _ = c.on_data([b"READ x\r\n"])
    assert rc == F_UNKNOWN_CONNECTION
    bad = json.dumps([{"name": "e", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"cmd": "JUMP"}}]}}]}]}]).encode()
    assert N.lib.cg_proxylib_policy_update(inst, bad, len(bad)) == N.CG_POLICY_REJECTED
    assert N.lib.cg_proxylib_policy_update(inst + 999, bad, len(bad)) == N.CG_INVALID_INSTANCE
    _lib.CloseModule(inst)


# the reference's r2d2 tests, end to end through the ABI
R2D2_POLICIES = [
    {"name": "cp1", "policy": 2, "ingress_per_port_policies": [{"port": 80, "rules": [{"l7_proto": "r2d2"}]}]},
    {"name": "cp2", "policy": 2, "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"cmd": "READ"}}]}}]}]},
    {"name": "cp3", "policy": 2, "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"file": "s.*"}}]}}]}]},
]


@pytest.mark.gpu
def test_gpu_r2d2_reference_sequences():
    inst = open_module([(b"node-id", b"gpu-test")], "0")
    assert inst != 0
    txt = json.dumps(R2D2_POLICIES).encode()
    assert N.lib.cg_proxylib_policy_update(inst, txt, len(txt)) == N.CG_OK
    # TestR2d2OnDataBasicPass (:70-95)
    c = Conn(inst, policy=b"cp1")
    msgs = [b"READ sssss\r\n", b"WRITE sssss\r\n", b"HALT\r\n", b"RESET\r\n"]
    assert c.on_data([b"".join(msgs)]) == (F_OK, [(PASS, len(m)) for m in msgs] + [(MORE, 1)])
    assert c.injected_reply() == b""
    # TestR2d2OnDataMultipleReq (:97-117)
    c = Conn(inst, policy=b"cp1")
    assert c.on_data([b"RE", b"SET\r\n"]) == (F_OK, [(PASS, 7), (MORE, 1)])
    # TestR2d2OnDataAllowDenyCmd (:119-146)
    c = Conn(inst, policy=b"cp2")
    m1, m2 = b"READ xssss\r\n", b"WRITE xssss\r\n"
    assert c.on_data([m1 + m2]) == (F_OK, [(PASS, len(m1)), (DROP, len(m2)), (MORE, 1)])
    assert c.injected_reply() == b"ERROR\r\n"
    # TestR2d2OnDataAllowDenyRegex (:148-176)
    c = Conn(inst, policy=b"cp3")
    m1, m2 = b"READ ssss\r\n", b"WRITE yyyyy\r\n"
    assert c.on_data([m1 + m2]) == (F_OK, [(PASS, len(m1)), (DROP, len(m2)), (MORE, 1)])
    assert c.injected_reply() == b"ERROR\r\n"
    # no policy for the port (81) and an unknown policy name: DROP
    c = Conn(inst, policy=b"cp1", dst_addr=b"2.2.2.2:81")
    assert c.on_data([b"READ a\r\n"]) == (F_OK, [(DROP, 8), (MORE, 1)])
    c = Conn(inst, policy=b"nosuch")
    assert c.on_data([b"READ a\r\n"]) == (F_OK, [(DROP, 8), (MORE, 1)])
    _lib.CloseModule(inst)


def test_policy_update_translation_rules():
    """cg_proxylib_policy_update applies the ParseError rules of both rule
    parsers (r2d2parser.go:91-123, cassandraparser.go:97-131) and the port
    rules of newPortNetworkPolicies (policymap.go:177-206)."""
    inst = open_module([(b"node-id", b"cpu-translate")], "-1")
    assert inst != 0

    def upd(pols):
        t = json.dumps(pols).encode()
        return N.lib.cg_proxylib_policy_update(inst, t, len(t))

    def pol(rules, port=80, proto="TCP"):
        return [{"name": "p", "ingress_per_port_policies": [{"port": port, "protocol": proto, "rules": rules}]}]

    def l7(parser, *rs):
        return {"l7_proto": parser, "l7_rules": {"l7_rules": [{"rule": r} for r in rs]}}

    assert upd(pol([l7("r2d2", {"cmd": "READ", "file": "^/a"})])) == N.CG_OK
    assert upd(pol([l7("cassandra", {"query_action": "select", "query_table": "t$"})])) == N.CG_OK
    assert upd(pol([l7("cassandra", {"query_action": "drop-role"})])) == N.CG_OK
    assert upd(pol([l7("unknown-parser", {"x": "y"})])) == N.CG_OK  # the port is dropped, not an error
    assert upd(pol([l7("r2d2"), {"l7_proto": "other"}])) == N.CG_OK  # unknown parser drops the port first
    assert upd(pol([], proto="UDP")) == N.CG_OK
    for bad in (pol([l7("cassandra", {"query_action": "explode"})]),
                pol([l7("cassandra", {"query_action": "create-role", "query_table": "x"})]),
                pol([l7("cassandra", {"table": "x"})]),
                pol([l7("r2d2", {"cmd": "JUMP"})]),
                pol([l7("r2d2", {"cmd": "RESET", "file": "x"})]),
                pol([l7("r2d2"), l7("cassandra")]),
                [{"name": "p", "ingress_per_port_policies": [{"port": 80}, {"port": 80}]}]):
        assert upd(bad) == N.CG_POLICY_REJECTED, bad
    _lib.CloseModule(inst)


@pytest.mark.gpu
def test_gpu_shim_random_vs_oracle():
    """Random r2d2 policies through the C++ translation and OnData framing,
    one request frame per call, against oracle/proxylib_ref.py."""
    import numpy as np

    from oracle.proxylib_ref import ProxylibOracle
    from test_proxylib import _rand_policies, _rand_requests
    from cilium_amd import proxylib as P
    inst = open_module([(b"node-id", b"gpu-random")], "0")
    assert inst != 0
    for seed in range(2):
        rng = np.random.default_rng(300 + seed)
        pols = _rand_policies(rng)
        reqs = _rand_requests(rng, 1500, len(pols))
        t = json.dumps(pols).encode()
        assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK
        o = ProxylibOracle(pols)
        conns = {}
        for name, ingress, port, remote, line in reqs:
            key = (name, ingress, port, remote)
            if key not in conns:
                conns[key] = Conn(inst, ingress=ingress, src=remote, dst=9, dst_addr=b"10.0.0.1:%d" % port,
                                  policy=name.encode())
                assert conns[key].rc == F_OK
            rc, ops = conns[key].on_data([line + b"\r\n"])
            exp = o.matches(name, ingress, port, remote, *P.r2d2_request(line))
            assert rc == F_OK and ops == [(PASS if exp else DROP, len(line) + 2), (MORE, 1)], (key, line)
        for c in conns.values():
            c.close()
    _lib.CloseModule(inst)


@pytest.mark.gpu
def test_gpu_r2d2_control_bytes_through_ondata():
    """NUL and control bytes inside r2d2 frames, through OnData, against the
    oracle (r2d2parser.go:148-199 frames on "\\r\\n" only)."""
    from oracle.proxylib_ref import ProxylibOracle
    from test_proxylib import CTRL_LINES, CTRL_POLS
    from cilium_amd import proxylib as P
    inst = open_module([(b"node-id", b"gpu-ctrl")], "0")
    assert inst != 0
    t = json.dumps(CTRL_POLS).encode()
    assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK
    o = ProxylibOracle(CTRL_POLS)
    for name in ("c1", "c2"):
        c = Conn(inst, policy=name.encode())
        frames = [line + b"\r\n" for line in CTRL_LINES]
        rc, ops = c.on_data([b"".join(frames)], cap=len(frames) + 1)
        exp = [o.matches(name, True, 80, 1, *P.r2d2_request(line)) for line in CTRL_LINES]
        assert rc == F_OK
        assert ops == [(PASS if e else DROP, len(f)) for e, f in zip(exp, frames)] + [(MORE, 1)], name
        assert c.injected_reply() == b"ERROR\r\n" * sum(1 for e in exp if not e)
        c.close()
    _lib.CloseModule(inst)


@pytest.mark.gpu
def test_gpu_ondata_concurrent_connections_share_batches():
    """16 threads, one connection each (different remote identities and
    policies), OnData concurrently: every call's ops match the oracle, and
    the instance's accounting adds up (cg_proxylib_stats: every call counted,
    1 <= batches <= calls). Whether calls combine depends on Python threads
    overlapping inside OnData under the GIL, so it is reported, not asserted;
    tests/test_ondata_combine_gpu.py holds the flusher to make combining
    deterministic, and tools/ondata_bench.cc measures it from C threads."""
    import threading

    import numpy as np

    from oracle.proxylib_ref import ProxylibOracle
    from test_proxylib import _rand_policies
    from cilium_amd import proxylib as P
    inst = open_module([(b"node-id", b"gpu-concurrent")], "0")
    assert inst != 0
    rng = np.random.default_rng(404)
    pols = _rand_policies(rng)
    t = json.dumps(pols).encode()
    assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK
    o = ProxylibOracle(pols)
    files = [b"/public/a", b"a.txt", b"secret", b"aaa", b"foo7", b"ssss", b"", b"x/y", b"sx"]
    errors = []

    def worker(k):
        try:
            r = np.random.default_rng(k)
            name = f"p{k % 3}"
            port = [80, 8080, 443][k % 3]
            remote = int(k % 8)
            c = Conn(inst, ingress=True, src=remote, dst=9, dst_addr=b"10.0.0.1:%d" % port, policy=name.encode())
            assert c.rc == F_OK
            for _ in range(60):
                lines = [bytes(r.choice([b"READ", b"WRITE", b"HALT"])) + b" " + bytes(r.choice(files))
                         for _ in range(int(r.integers(1, 17)))]
                # room for every frame and the MORE op (connection.go:141: a
                # full ops slice ends the call without MORE)
                rc, ops = c.on_data([b"".join(x + b"\r\n" for x in lines)], cap=len(lines) + 1)
                exp = [(PASS if o.matches(name, True, port, remote, *P.r2d2_request(x)) else DROP, len(x) + 2)
                       for x in lines]
                assert rc == F_OK and ops == exp + [(MORE, 1)], (k, lines, ops)
                c.take_reply()
        except Exception as e:  # noqa: BLE001 — surfaced below
            errors.append(repr(e))

    b0, c0 = C.c_uint64(), C.c_uint64()
    N.lib.cg_proxylib_stats(inst, C.byref(b0), C.byref(c0))
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    b1, c1 = C.c_uint64(), C.c_uint64()
    N.lib.cg_proxylib_stats(inst, C.byref(b1), C.byref(c1))
    _lib.CloseModule(inst)
    assert not errors, errors[:3]
    calls, batches = c1.value - c0.value, b1.value - b0.value
    print(f"ondata concurrent: calls={calls} batches={batches}")
    assert calls == 16 * 60 and 1 <= batches <= calls, (calls, batches)


def test_ondata_combiner_concurrency_without_device():
    """The flat-combining batcher under 16 concurrent connections on a
    handle without a GPU: every call with request frames reaches the shared
    queue, each flush fails (no device) and releases all the calls it took —
    every OnData returns the engine error, none waits forever, and the
    instance's counts add up (cg_proxylib_stats: calls = calls made, batches
    <= calls)."""
    import threading

    inst = open_module([(b"node-id", b"cpu-combiner")], "-1")
    assert inst != 0
    t = json.dumps(R2D2_POLICIES).encode()
    assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK
    rcs, per = [], 40

    def worker(k):
        c = Conn(inst, policy=b"cp2", src=k)
        assert c.rc == F_OK
        for j in range(per):
            rc, ops = c.on_data([b"READ f%d\r\nWRITE g%d\r\n" % (j, j)], cap=3)
            rcs.append((rc, ops))
        c.close()

    b0, c0 = C.c_uint64(), C.c_uint64()
    N.lib.cg_proxylib_stats(inst, C.byref(b0), C.byref(c0))
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(timeout=120)
        assert not x.is_alive(), "an OnData call never returned"
    b1, c1 = C.c_uint64(), C.c_uint64()
    N.lib.cg_proxylib_stats(inst, C.byref(b1), C.byref(c1))
    _lib.CloseModule(inst)
    assert len(rcs) == 16 * per
    assert all(rc == F_UNKNOWN_ERROR and ops == [] for rc, ops in rcs), rcs[:3]
    calls, batches = c1.value - c0.value, b1.value - b0.value
    assert calls == 16 * per and 1 <= batches <= calls, (calls, batches)


def test_ondata_batching_window_without_device():
    """cg_proxylib_set_batching on a handle without a GPU: 16 connections
    released from one barrier per round, window of 16 calls — each round's
    calls are taken as ONE batch (whose flush fails: no device), every call
    returns the engine error, none waits past the window."""
    import threading

    inst = open_module([(b"node-id", b"cpu-window")], "-1")
    assert inst != 0
    assert N.lib.cg_proxylib_set_batching(inst + 999, 16, 1000) == N.CG_INVALID_INSTANCE
    t = json.dumps(R2D2_POLICIES).encode()
    assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK
    assert N.lib.cg_proxylib_set_batching(inst, 16, 5_000_000) == N.CG_OK
    rounds, bar, rcs = 3, threading.Barrier(16), []

    def worker(k):
        c = Conn(inst, policy=b"cp2", src=k)
        assert c.rc == F_OK
        for j in range(rounds):
            bar.wait()
            rcs.append(c.on_data([b"READ f%d\r\n" % j], cap=2))
            bar.wait()
        c.close()

    b0, c0 = C.c_uint64(), C.c_uint64()
    N.lib.cg_proxylib_stats(inst, C.byref(b0), C.byref(c0))
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(timeout=120)
        assert not x.is_alive(), "an OnData call never returned"
    b1, c1 = C.c_uint64(), C.c_uint64()
    N.lib.cg_proxylib_stats(inst, C.byref(b1), C.byref(c1))
    _lib.CloseModule(inst)
    assert all(rc == F_UNKNOWN_ERROR and ops == [] for rc, ops in rcs), rcs[:3]
    assert (c1.value - c0.value, b1.value - b0.value) == (16 * rounds, rounds)
