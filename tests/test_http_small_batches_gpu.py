"""cg_http_verdicts_fields_host at Envoy batch sizes (capi.cc
small_lists_combined): a call of at most 1024 header lists is decided with
the small calls other threads have queued on the handle — one host-packed
batch, one http_kernel launch — and every call's verdicts equal the
reference path's (cg_http_pack + http_kernel over the same lists, itself
checked against the oracle in test_http_fields_gpu.py).  The window test
holds the flusher until 16 calls are queued (cg_http_set_batching), so the
combining is deterministic: one batch per round of 16 threads."""
import ctypes as C
import threading

import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import synth
from cilium_amd.classifier import Classifier

pytestmark = [pytest.mark.gpu, pytest.mark.run_last]


def _split(rq, a, b):
    off = rq["hdr_off"]
    return (rq["policy"][a:b], rq["ingress"][a:b], rq["port"][a:b], rq["remote"][a:b], rq["hdr_blob"],
            np.ascontiguousarray(off[a:b + 1]))


def _stats(cl):
    b, c = C.c_uint64(), C.c_uint64()
    assert N.lib.cg_http_batching_stats(cl.h, C.byref(b), C.byref(c)) == N.CG_OK
    return b.value, c.value


@pytest.fixture(scope="module")
def http10k():
    cl = Classifier(device=0)
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    rq = synth.http10k_requests(40_000, info, seed=150)
    want = cl.http_verdicts(cl.pack_http(**rq))
    k = 6_000
    sub = {kk: (v[:k] if kk not in ("hdr_blob", "hdr_off") else v) for kk, v in rq.items()}
    sub["hdr_off"] = rq["hdr_off"][:k + 1]
    assert np.array_equal(want[:k], oracle.HttpOracle(pols).eval(**sub, nthreads=8))
    yield cl, rq, want
    cl.close()


def test_gpu_small_calls_equal_the_pack_path(http10k):
    """Lone calls of 1 .. 1025 lists (1025: the GPU packing path) at offsets
    that do not start at 0 in the blob."""
    cl, rq, want = http10k
    a = 0
    for n in (1, 2, 3, 16, 63, 64, 65, 255, 1000, 1024, 1025, 1):
        got = cl.http_verdicts_fields(*_split(rq, a, a + n))
        assert np.array_equal(got, want[a:a + n]), n
        a += n


def test_gpu_small_calls_combined_across_threads(http10k):
    cl, rq, want = http10k
    assert N.lib.cg_http_set_batching(cl.h, 16, 5_000_000) == N.CG_OK
    nthreads, rounds = 16, 5
    bar = threading.Barrier(nthreads)
    errors = []

    def worker(t):
        try:
            r = np.random.default_rng(t)
            for j in range(rounds):
                n = int(r.integers(1, 9))
                a = int(r.integers(0, len(want) - n))
                bar.wait()
                got = cl.http_verdicts_fields(*_split(rq, a, a + n))
                assert np.array_equal(got, want[a:a + n]), (t, j, a, n)
                bar.wait()
        except Exception as e:  # noqa: BLE001 — surfaced below
            errors.append(repr(e))
            bar.abort()

    b0, c0 = _stats(cl)
    ts = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(timeout=120)
        assert not x.is_alive(), "a call never returned"
    b1, c1 = _stats(cl)
    assert N.lib.cg_http_set_batching(cl.h, 1, 0) == N.CG_OK
    assert not errors, errors[:3]
    print(f"small calls: {c1 - c0} calls in {b1 - b0} batches")
    assert (c1 - c0, b1 - b0) == (nthreads * rounds, rounds)


def test_gpu_small_calls_concurrent_default_window(http10k):
    """16 threads x 40 calls with the default window: parity for every call,
    and the accounting adds up (batches <= calls)."""
    cl, rq, want = http10k
    errors = []

    def worker(t):
        try:
            r = np.random.default_rng(100 + t)
            for _ in range(40):
                n = int(r.integers(1, 65))
                a = int(r.integers(0, len(want) - n))
                got = cl.http_verdicts_fields(*_split(rq, a, a + n))
                assert np.array_equal(got, want[a:a + n]), (t, a, n)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    b0, c0 = _stats(cl)
    ts = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(timeout=120)
    b1, c1 = _stats(cl)
    assert not errors, errors[:3]
    assert c1 - c0 == 16 * 40 and 1 <= b1 - b0 <= c1 - c0
