"""The persistent verdict ring (cg_http_ring_*, csrc/ring.cc + kernels_http_raw.hip
http_ring_kernel): Envoy-sized calls (AccessFilter::decodeHeaders decides one
request, envoy/cilium_l7policy.cc:127-182) decided by a resident kernel that
polls request slots in fine-grained device memory the host writes through its
mapping (or, CILIUM_GPU_RING_SLOTS=host, in pinned host memory).  Verdicts against the oracle and
the staged entry; calls from many threads; a policy update between calls;
the kernel's idle exit and relaunch; calls past a slot; open / close.  The
test prints throughput and asserts no timing."""
import threading
import time

import numpy as np
import pytest

from cilium_amd import _native as N
from cilium_amd import synth
from cilium_amd.classifier import Classifier
from test_http_fields_gpu import _host_path, _join, _oracle, _split, _vary


def test_ring_needs_a_gpu(host):
    with pytest.raises(N.CiliumGPUError):
        host.http_ring_open(2, 4)


def _pool(n, seed):
    pols, info = synth.http10k_rules()
    rq = synth.http10k_requests(n, info, seed=seed)
    lists = _split(rq["hdr_blob"], rq["hdr_off"])
    args = (np.asarray(rq["policy"], np.uint32), np.asarray(rq["ingress"], np.uint8),
            np.asarray(rq["port"], np.uint16), np.asarray(rq["remote"], np.uint32))
    return pols, lists, args


@pytest.mark.gpu
@pytest.mark.parametrize("slots", ["device", "host"])
def test_gpu_ring_calls(slots, monkeypatch):
    if slots == "host":
        monkeypatch.setenv("CILIUM_GPU_RING_SLOTS", "host")
    else:
        monkeypatch.delenv("CILIUM_GPU_RING_SLOTS", raising=False)
    cl = Classifier(device=0)
    try:
        pols, lists, args = _pool(4096, 71)
        cl.update_http_policy(pols)
        blob, off = _join(lists)
        want = _oracle(pols, *args, blob, off)
        assert np.array_equal(want, cl.http_verdicts_fields(*args, blob, off))
        cl.http_ring_open(8, 16)
        # single-request calls, the Envoy shape
        t0 = time.perf_counter()
        for i in range(1000):
            b, o = _join(lists[i:i + 1])
            got = cl.http_ring_verdicts(*(a[i:i + 1] for a in args), b, o)
            assert got[0] == want[i], i
        dt = time.perf_counter() - t0
        print(f"ring, 1 thread, batch 1 (Python ctypes): {1000 / dt:.0f} calls/s, {dt / 1000 * 1e6:.1f} us per call")
        # one launch serves a steady stream of calls (it leaves only when idle
        # 50 ms or 2 s old)
        if dt < 1.5:  # (a pause of the test process past 50 ms may cost one relaunch)
            assert cl.http_ring_stats()["launches"] <= 3, cl.http_ring_stats()
        # batches of 16 and 256 (a slot's limit), and 300 (past it: the staged entry)
        for B in (16, 256, 300):
            for a in range(0, 1200, B):
                b, o = _join(lists[a:a + B])
                got = cl.http_ring_verdicts(*(x[a:a + B] for x in args), b, o)
                assert np.array_equal(got, want[a:a + B]), (B, a)
        # an empty call
        assert len(cl.http_ring_verdicts([], [], [], [], np.zeros(1, np.uint8), np.zeros(1, np.uint64))) == 0
        # 16 threads at once, each with its own calls
        errs = []

        def worker(t):
            try:
                for k in range(150):
                    i = (t * 257 + k * 13) % len(lists)
                    b, o = _join(lists[i:i + 1])
                    if cl.http_ring_verdicts(*(x[i:i + 1] for x in args), b, o)[0] != want[i]:
                        errs.append((t, i))
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t0
        assert not errs, errs[:5]
        print(f"ring, 16 threads, batch 1 (Python ctypes): {16 * 150 / dt:.0f} calls/s")
        st = cl.http_ring_stats()
        assert st["served"] >= 1000 + 16 * 150 and st["launches"] >= 1, st
        # the kernel leaves after 50 ms without a call; the next call starts it again
        time.sleep(0.3)
        b, o = _join(lists[:64])
        assert np.array_equal(cl.http_ring_verdicts(*(x[:64] for x in args), b, o), want[:64])
        assert cl.http_ring_stats()["launches"] > st["launches"]
        cl.http_ring_close()
        with pytest.raises(N.CiliumGPUError):
            cl.http_ring_verdicts(*(x[:1] for x in args), *_join(lists[:1]))
    finally:
        cl.close()


@pytest.mark.gpu
def test_gpu_ring_policy_update_and_fallbacks():
    """A policy update between calls: the next call is decided by the new
    tables (the ring restarts its kernel).  A snapshot walking more than 32
    fields takes the staged entry.  cg_close stops a running ring."""
    cl = Classifier(device=0)
    try:
        pols = synth.starwars_policy()
        cl.update_http_policy(pols)
        rq = synth.starwars_requests(2000, seed=72)
        lists = _split(rq["hdr_blob"], rq["hdr_off"])
        args = tuple(np.asarray(rq[k], dt) for k, dt in (("policy", np.uint32), ("ingress", np.uint8),
                                                          ("port", np.uint16), ("remote", np.uint32)))
        blob, off = _join(lists)
        cl.http_ring_open(4, 8)
        want = _oracle(pols, *args, blob, off)
        got = np.concatenate([cl.http_ring_verdicts(*(x[a:a + 100] for x in args), *_join(lists[a:a + 100]))
                              for a in range(0, 2000, 100)])
        assert np.array_equal(got, want) and 0.05 < want.mean() < 0.95
        # allow everything on the same policy names: every request is allowed now
        open_pols = [{"name": p["name"], "policy": p.get("policy", 0),
                      "egress_per_port_policies": [{"port": 80, "rules": [{"remote_policies": []}]}],
                      "ingress_per_port_policies": [{"port": 80, "rules": [{"remote_policies": []}]}]}
                     for p in pols]
        cl.update_http_policy(open_pols)
        want2 = _oracle(open_pols, *args, blob, off)
        got2 = np.concatenate([cl.http_ring_verdicts(*(x[a:a + 100] for x in args), *_join(lists[a:a + 100]))
                               for a in range(0, 2000, 100)])
        assert np.array_equal(got2, want2) and not np.array_equal(want, want2)
        # 40 walked fields: past the device list parser, decided by the staged entry
        names = ["x-f%02d" % i for i in range(40)]
        many = [{"name": "m", "policy": 0, "ingress_per_port_policies": [{"port": 80, "rules": [
            {"remote_policies": [], "http_rules": {"http_rules": [
                {"headers": [{"name": nm, "exact_match": "v"}]} for nm in names]}}]}]}]
        cl.update_http_policy(many)
        ml = [b":method\0GET\0x-f%02d\0%s\0" % (i % 40, b"v" if i % 3 else b"w") for i in range(200)]
        mb, mo = _join(ml)
        margs = (np.zeros(200, np.uint32), np.ones(200, np.uint8), np.full(200, 80, np.uint16), np.zeros(200, np.uint32))
        assert np.array_equal(cl.http_ring_verdicts(*margs, mb, mo), _oracle(many, *margs, mb, mo))
        cl.update_http_policy(pols)
        assert cl.http_ring_verdicts(*(x[:1] for x in args), *_join(lists[:1]))[0] == want[0]
    finally:
        cl.close()  # stops the ring


def _ring_batches(cl, args, lists, sizes):
    """Verdicts of lists through the ring in calls of the given sizes (cycled)."""
    out, a, k = [], 0, 0
    while a < len(lists):
        B = sizes[k % len(sizes)]
        out.append(cl.http_ring_verdicts(*(x[a:a + B] for x in args), *_join(lists[a:a + B])))
        a += B
        k += 1
    return np.concatenate(out)


@pytest.mark.gpu
def test_gpu_ring_varied_lists():
    """Lists as a proxy hands them over (test_http_fields_gpu._vary: name case,
    repeated names, unknown headers, values past the ring's 256-byte string
    buffer, multi-KiB lists, control bytes, empty names, cut-short pairs,
    empty lists), the hand-made edge cases, and a proxylib snapshot's escaped
    values, through the ring at batch sizes 1, 3, 16 and 64 — against the
    oracle and the host packer path."""
    cl = Classifier(device=0)
    try:
        pols, info = synth.http10k_rules()
        cl.update_http_policy(pols)
        rq = synth.http10k_requests(3000, info, seed=73)
        lists = _vary(_split(rq["hdr_blob"], rq["hdr_off"]), np.random.default_rng(74), frac=0.5)
        args = tuple(np.asarray(rq[k], dt) for k, dt in (("policy", np.uint32), ("ingress", np.uint8),
                                                          ("port", np.uint16), ("remote", np.uint32)))
        blob, off = _join(lists)
        want = _oracle(pols, *args, blob, off)
        assert np.array_equal(want, _host_path(cl, *args, blob, off))
        cl.http_ring_open(8, 32)
        got = _ring_batches(cl, args, lists, (1, 3, 16, 64))
        bad = np.nonzero(got != want)[0]
        assert not len(bad), [(int(i), lists[i][:160], int(got[i]), int(want[i])) for i in bad[:4]]
        assert 0.1 < want.mean() < 0.9
        # the hand-made edge cases (test_gpu_fields_edge_cases, without the 20 KiB list)
        sw_pols = synth.starwars_policy()
        cl.update_http_policy(sw_pols)
        sw = cl.http_policy_index(sw_pols[0]["name"])
        ok = b":method\0POST\0:path\0/v1/request-landing/\0:authority\0deathstar\0"
        upper = b":METHOD\0POST\0:Path\0/v1/request-landing/\0:AUTHORITY\0deathstar\0"
        el = [b"", b"\0", ok[:-1], ok, upper, ok + b":method\0GET\0", b":method\0GET\0" + ok,
              ok + b"x-a\0bad\x7fbyte\0", ok + b"x-a\0bad\nbyte\0", ok + b"x-a\0tab\there\0", ok + b"x-a\0\x80\xff\0",
              b"\0v\0" + ok, ok + b"x-big\0" + b"z" * 9_000 + b"\0", ok.replace(b"POST", b"PO\x01ST"),
              ok.replace(b"/v1/request-landing/", b"/v1/request-landing/" + b"q" * 400),
              # pair counts about the wave-cooperative parse's limit of 127 NULs
              # (batch 1): 62 / 63 / 64 / 70 / 200 pairs, with the real fields
              # last, a repeated name and a rejected byte late in the list
              *[b"".join(b"x-p%d\0v%d\0" % (q, q) for q in range(m)) + ok for m in (59, 60, 61, 67, 197)],
              b"".join(b"x-p%d\0v\0" % q for q in range(61)) + b":method\0GET\0" + ok,
              b"".join(b"x-p%d\0v\0" % q for q in range(100)) + ok + b"x-late\0b\x01d\0",
              ok, ok]
        n = len(el)
        eargs = (np.array([sw] * (n - 2) + [sw, 0xFFFFFFFF], np.uint32), np.zeros(n, np.uint8),
                 np.array([80] * (n - 2) + [8080, 80], np.uint16), np.full(n, synth.SPACESHIP_ID, np.uint32))
        eb, eo = _join(el)
        ew = _oracle(sw_pols, *eargs, eb, eo)
        for sizes in ((1,), (n,), (5,)):
            assert np.array_equal(_ring_batches(cl, eargs, el, sizes), ew), sizes
        # a proxylib snapshot (escaped values, raw_values lists)
        rules = [{"headers": [{"name": "cmd", "exact_match": "READ"}, {"name": "file", "regex_match": "/pub/.*"}]},
                 {"headers": [{"name": "cmd", "exact_match": "WR\x01TE"}]}]
        ppol = [{"name": "p", "proxylib": True, "policy": 0, "ingress_per_port_policies": [
            {"port": 80, "rules": [{"remote_policies": [1], "http_rules": {"http_rules": rules}}]}]}]
        cl.update_http_policy(ppol)
        rng = np.random.default_rng(75)
        vals = [b"READ", b"WRITE", b"WR\x03\x11TE", b"WR\x01TE", b"RE\x03AD", b"READ\x03", b"\x03\x14x", b"/pub/a",
                b"/pub/\x03\x10", b"/priv/x", b"\x02", b"\x03\x15"]
        pl = []
        for _ in range(600):
            ps = [(b"cmd", vals[int(rng.integers(0, len(vals)))])]
            if rng.random() < 0.7:
                ps.append((b"File" if rng.random() < 0.3 else b"file", vals[int(rng.integers(0, len(vals)))]))
            if rng.random() < 0.2:
                ps.reverse()
            pl.append(b"".join(nm + b"\0" + v + b"\0" for nm, v in ps))
        m = len(pl)
        pargs = (np.zeros(m, np.uint32), np.ones(m, np.uint8), np.full(m, 80, np.uint16),
                 rng.integers(0, 3, m).astype(np.uint32))
        pb, po = _join(pl)
        pw = _host_path(cl, *pargs, pb, po)
        assert np.array_equal(_ring_batches(cl, pargs, pl, (1, 7, 64)), pw)
        assert 0.02 < pw.mean() < 0.9
    finally:
        cl.close()
