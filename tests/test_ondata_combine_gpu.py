"""The OnData combiner on the GPU, made deterministic.

Envoy calls OnData on many connections at once (one thread per connection at
a time, proxylib/libcilium.h:79-80); the instance decides the request frames
of the calls queued together as one GPU batch (csrc/proxylib_shim.cc decide).
Python threads rarely overlap inside OnData under the GIL, so these tests
open a batching window (cg_proxylib_set_batching: the flusher waits for k
queued calls) and release all threads from one barrier: the calls must then
share batches, and every call's ops must equal the oracle's.

The policy-swap test pins the advisor's round-4 finding: a queued call's
policy is resolved by name under the instance lock, from the snapshot its
batch is decided with (the Go proxylib looks it up at match time,
proxylib/proxylib/policymap.go:208-236), so a policy update that shifts the
policy list's indices never evaluates a request under another policy."""
import ctypes as C
import json
import threading

import numpy as np
import pytest

from cilium_amd import _native as N
from test_proxylib_abi import DROP, F_OK, MORE, PASS, Conn, _lib, open_module

pytestmark = [pytest.mark.gpu, pytest.mark.run_last]


def _stats(inst):
    b, c = C.c_uint64(), C.c_uint64()
    assert N.lib.cg_proxylib_stats(inst, C.byref(b), C.byref(c)) == N.CG_OK
    return b.value, c.value


def test_gpu_ondata_batching_window_combines_calls():
    """16 connections, 4 rounds of one OnData call each, released together:
    with a window of 16 calls each round is decided as one GPU batch, and
    every call's ops match the oracle."""
    from oracle.proxylib_ref import ProxylibOracle
    from test_proxylib import _rand_policies
    from cilium_amd import proxylib as P
    inst = open_module([(b"node-id", b"gpu-window")], "0")
    assert inst != 0
    pols = _rand_policies(np.random.default_rng(505))
    t = json.dumps(pols).encode()
    assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK
    assert N.lib.cg_proxylib_set_batching(inst, 16, 5_000_000) == N.CG_OK
    o = ProxylibOracle(pols)
    files = [b"/public/a", b"a.txt", b"secret", b"aaa", b"foo7", b"", b"x/y"]
    nthreads, rounds = 16, 4
    bar = threading.Barrier(nthreads)
    errors, per_round = [], []

    def worker(k):
        try:
            r = np.random.default_rng(k)
            name, port, remote = f"p{k % 3}", [80, 8080, 443][k % 3], k % 8
            c = Conn(inst, ingress=True, src=remote, dst=9, dst_addr=b"10.0.0.1:%d" % port, policy=name.encode())
            assert c.rc == F_OK
            for _ in range(rounds):
                lines = [bytes(r.choice([b"READ", b"WRITE", b"HALT"])) + b" " + bytes(r.choice(files))
                         for _ in range(int(r.integers(1, 9)))]
                bar.wait()
                rc, ops = c.on_data([b"".join(x + b"\r\n" for x in lines)], cap=len(lines) + 1)
                exp = [(PASS if o.matches(name, True, port, remote, *P.r2d2_request(x)) else DROP, len(x) + 2)
                       for x in lines]
                assert rc == F_OK and ops == exp + [(MORE, 1)], (k, lines, ops)
                c.take_reply()
                if bar.wait() == 0:
                    per_round.append(_stats(inst))
            c.close()
        except Exception as e:  # noqa: BLE001 — surfaced below
            errors.append(repr(e))
            bar.abort()

    b0, c0 = _stats(inst)
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(timeout=120)
        assert not x.is_alive(), "an OnData call never returned"
    b1, c1 = _stats(inst)
    _lib.CloseModule(inst)
    assert not errors, errors[:3]
    calls, batches = c1 - c0, b1 - b0
    print(f"ondata window: calls={calls} batches={batches} per round={per_round}")
    assert calls == nthreads * rounds
    assert batches == rounds, (calls, batches)


def test_gpu_ondata_policy_indices_shift_under_updates():
    """OnData on policy "pb" from 8 threads while another thread alternates
    the installed list between [pa, pb] and [pb] (pb's index 1 <-> 0); pa
    allows only HALT, pb only READ.  Every READ must PASS and every HALT DROP
    whichever list a batch meets."""
    pa = {"name": "pa", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"cmd": "HALT"}}]}}]}]}
    pb = {"name": "pb", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"cmd": "READ"}}]}}]}]}
    texts = [json.dumps([pa, pb]).encode(), json.dumps([pb]).encode()]
    inst = open_module([(b"node-id", b"gpu-shift")], "0")
    assert inst != 0
    assert N.lib.cg_proxylib_policy_update(inst, texts[0], len(texts[0])) == N.CG_OK
    assert N.lib.cg_proxylib_set_batching(inst, 4, 2_000)  == N.CG_OK
    stop = threading.Event()
    errors = []

    def updater():
        k = 0
        while not stop.is_set():
            k ^= 1
            if N.lib.cg_proxylib_policy_update(inst, texts[k], len(texts[k])) != N.CG_OK:
                errors.append("update failed")

    def worker(k):
        try:
            c = Conn(inst, ingress=True, src=k, dst=9, dst_addr=b"10.0.0.1:80", policy=b"pb")
            assert c.rc == F_OK
            for j in range(40):
                rc, ops = c.on_data([b"READ a%d\r\nHALT b%d\r\n" % (j, j)], cap=3)
                assert rc == F_OK and ops == [(PASS, len(b"READ a%d\r\n" % j)), (DROP, len(b"HALT b%d\r\n" % j)),
                                              (MORE, 1)], (k, j, ops)
                c.take_reply()
            c.close()
        except Exception as e:  # noqa: BLE001 — surfaced below
            errors.append(repr(e))

    u = threading.Thread(target=updater)
    u.start()
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(timeout=120)
        assert not x.is_alive(), "an OnData call never returned"
    stop.set()
    u.join(timeout=60)
    _lib.CloseModule(inst)
    assert not errors, errors[:3]
