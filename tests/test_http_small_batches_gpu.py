"""cg_http_verdicts_fields_host at Envoy batch sizes (capi.cc
small_lists_host): a call of at most 1024 header lists is packed on the
calling thread and decided with one staged copy, one http_kernel launch and
one copy out; every call's verdicts equal the reference path's (cg_http_pack
+ http_kernel over the same lists, checked against the oracle here), alone
and from 16 concurrent threads."""
import threading

import numpy as np
import pytest

import oracle
from cilium_amd import synth
from cilium_amd.classifier import Classifier

pytestmark = [pytest.mark.gpu, pytest.mark.run_last]


def _split(rq, a, b):
    off = rq["hdr_off"]
    return (rq["policy"][a:b], rq["ingress"][a:b], rq["port"][a:b], rq["remote"][a:b], rq["hdr_blob"],
            np.ascontiguousarray(off[a:b + 1]))


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


def test_gpu_small_calls_concurrent(http10k):
    """16 threads x 40 calls of 1..64 lists: parity for every call."""
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

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(timeout=120)
        assert not x.is_alive(), "a call never returned"
    assert not errors, errors[:3]
