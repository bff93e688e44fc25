"""The pieces the multi-GPU bench relies on, on one device:

- ranks >= 1 import the image rank 0 compiled (bench.py: cg_http_policy_export
  → broadcast → cg_http_policy_import) and run http_kernel on it: an imported
  snapshot on its own handle decides a config-5 sample exactly as the
  compiling handle and the oracle do;
- the per-step all-reduce sums each rank's counter vector
  (cg_counters_copy_dev of CG_CTR_HTTP_ALLREDUCE, then RCCL sum): two handles'
  vectors copied on the device and summed there equal the oracle's
  first-match totals over both shards.

These are the same calls bench.py makes; only the RCCL transport itself (one
process per GPU over xGMI) needs an 8-GPU node."""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import synth
from cilium_amd.classifier import Classifier
from test_rule_counters import _oracle_counts

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.fixture(scope="module")
def ranks():
    """rank 0 compiles the 10K-rule set, rank 1 imports its image."""
    pols, info = synth.http10k_rules()
    a, b = Classifier(device=0), Classifier(device=0)
    a.update_http_policy(pols)
    b.import_http_policy(a.export_http_policy())
    yield pols, info, a, b
    a.close()
    b.close()


def test_gpu_imported_image_decides_config5_sample(ranks):
    pols, info, a, b = ranks
    rq = synth.http10k_requests(200_000, info, seed=808, distinct=100_000)
    exp = oracle.HttpOracle(pols).eval(**rq, nthreads=16)
    va = a.http_verdicts(a.pack_http(**rq))
    vb = b.http_verdicts(b.pack_http(**rq))  # packed against the imported snapshot
    assert np.array_equal(vb, exp) and np.array_equal(va, vb)
    assert 0.2 < exp.mean() < 0.8
    assert b.http_policy_index("ep-10k") == a.http_policy_index("ep-10k")


def test_gpu_counter_vectors_summed_on_device(ranks):
    torch = _torch()
    pols, info, a, b = ranks
    rq = synth.http10k_requests(120_000, info, seed=809, distinct=60_000)
    n = len(rq["policy"])
    half = n // 2

    def shard(lo, hi):
        d = {k: v[lo:hi] for k, v in rq.items() if k not in ("hdr_blob", "hdr_off")}
        off = rq["hdr_off"][lo:hi + 1]
        d["hdr_blob"] = rq["hdr_blob"][int(off[0]):int(off[-1])].copy()
        d["hdr_off"] = (off - off[0]).astype(np.uint64)
        return d

    a.reset_counters()
    b.reset_counters()
    va = a.http_verdicts(a.pack_http(**shard(0, half)))
    vb = b.http_verdicts(b.pack_http(**shard(half, n)))
    m = a.allreduce_counter_count()
    assert m == b.allreduce_counter_count()
    dev = torch.device("cuda", 0)
    bufs = [torch.zeros(m, dtype=torch.int64, device=dev) for _ in range(2)]
    s = torch.cuda.current_stream().cuda_stream
    a.counters_copy_dev(bufs[0], m, stream=s)
    b.counters_copy_dev(bufs[1], m, stream=s)
    total = (bufs[0] + bufs[1]).cpu().numpy().astype(np.uint64)  # what the RCCL sum leaves on every rank
    info_r = a.http_rule_info()
    v, _, counts = _oracle_counts(pols, rq, info_r, nthreads=16)
    assert np.array_equal(np.concatenate([va, vb]), v)
    nprog2 = len(a.read_counters(N.CG_CTR_HTTP_PROGRAMS))
    progs = total[:nprog2]
    assert int(progs[0::2].sum()) == int(v.sum()) and int(progs.sum()) == n
    assert int(total[nprog2]) == 0  # no stale batches
    assert np.array_equal(total[nprog2 + 1:], counts)
