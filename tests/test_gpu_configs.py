"""The reference's own fixtures through the HIP kernels, and every BASELINE
config at its stated size on the GPU.

* KATs: tests/golden/{http,kafka,lpm}_kat.json (Envoy BASIC_POLICY and the
  runtime/star-wars e2e assertions, pkg/kafka/policy_test.go, unit-test.c LPM
  cases) evaluated by http_kernel / kafka_kernel / lpm_kernel — the same
  fixtures test_cpu_kat.py pins the oracle with.
* Configs (BASELINE.json "configs"): star-wars over 1M requests; the L4
  policymap with 100M tuples; the CIDR prefilter with 1M prefixes and 1B
  addresses; Kafka with 1K rules over 100M requests; the 10K-rule HTTP set
  with a 125M-request (1B / 8 GPUs) batch.  Where the oracle cannot walk the
  full size in seconds, the full-size batch is built on the device from
  copies of a few million distinct items the oracle does walk: every copy
  must carry its original's verdict (a bit-exact check of all items) and the
  counters must equal the copies' multiple of the oracle's (a checksum of
  the whole run).
"""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import synth
from kat_util import http_requests, kafka_case, load, lpm_case

pytestmark = pytest.mark.gpu

HTTP = load("http_kat.json")


def _torch():
    import torch
    return torch


# ------------------------------------------------- reference fixtures ----
@pytest.mark.parametrize("suite", HTTP["suites"], ids=lambda s: s["name"])
def test_gpu_http_kat(gpu, suite):
    """Envoy cilium_integration_test.cc:738-776,821-854 (BASIC_POLICY), the
    runtime method matrix (Policies.go:1015-1085) and star wars
    (demos.go:137-159) on http_kernel."""
    names = [p["name"] for p in suite["policy"]]
    rq = http_requests(suite["requests"], lambda n: names.index(n) if n in names else 0xFFFFFFFF)
    exp = np.array([r["expect"] for r in suite["requests"]], np.uint8)
    gpu.update_http_policy(suite["policy"])
    got = gpu.http_verdicts(gpu.pack_http(**rq))
    bad = [r["name"] + " @" + r["source"] for r, a, b in zip(suite["requests"], got, exp) if a != b]
    assert not bad


def test_gpu_kafka_kat(gpu):
    """pkg/kafka/policy_test.go:85-127 on kafka_kernel."""
    for c in load("kafka_kat.json")["matches_rule"]:
        pol, req = kafka_case(c)
        gpu.update_kafka_policy(pol)
        reqs, arena = gpu.pack_kafka(**req)
        assert int(gpu.kafka_verdicts(reqs, arena)[0]) == c["expect"], c["source"]


def test_gpu_lpm_kat(gpu):
    """test/bpf/unit-test.c:77-102 prefix cases on lpm_kernel."""
    for c in load("lpm_kat.json")["covers"]:
        pfx, v4, ep4 = lpm_case(c)
        pf = gpu.prefilter(dyn4=True)
        pf.insert(0, pfx)
        pf.set_endpoints(ep4, np.zeros((0, 16), np.uint8))
        g4, _ = pf.verdicts(v4, np.zeros((0, 32), np.uint8))
        assert int(g4[0]) == (1 if c["covered"] else 2), c
        pf.destroy()


# -------------------------------------------------------- config 1 ----
def test_config1_starwars_1m(gpu):
    """examples/demo star-wars L7 rules over 1M synthetic requests."""
    pols = synth.starwars_policy()
    rq = synth.starwars_requests(1_000_000, seed=101)
    gpu.update_http_policy(pols)
    got = gpu.http_verdicts(gpu.pack_http(**rq))
    exp = oracle.HttpOracle(pols).eval(**rq, nthreads=16)
    assert np.array_equal(got, exp)
    assert 0 < got.sum() < len(got)


# -------------------------------------------------------- config 2 ----
def test_config2_l4_100m(gpu):
    """16K-entry policymap, 100M tuples: 5M distinct tuples (oracle-checked,
    verdicts and per-entry counters) copied 20 times on the device; every
    copy's verdict equals its original's and every entry's packets/bytes are
    20 times the oracle's."""
    torch = _torch()
    keys, ports = synth.l4_table()
    tuples = synth.l4_tuples(5_000_000, keys, seed=202)
    exp, pk, by = oracle.l4(keys, ports, tuples)
    reps = 20
    pm = gpu.policy_map()
    pm.allow_keys(keys, ports)
    d_t = torch.from_numpy(tuples.view(np.uint8)).cuda().repeat(reps)
    d_out = torch.empty(len(tuples) * reps, dtype=torch.int32, device="cuda")
    pm.verdicts_dev(d_t, len(tuples) * reps, d_out, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    d_exp = torch.from_numpy(exp).cuda()
    assert bool((d_out.view(reps, -1) == d_exp).all())
    dump = {(k.Identity, k.DestPort, k.Nexthdr, k.TrafficDirection): e for k, e in pm.dump_to_slice()}
    gpk = np.array([dump[(int(k["sec_label"]), int(k["dport"]), int(k["protocol"]), int(k["egress"]))].Packets
                    for k in keys], np.uint64)
    gby = np.array([dump[(int(k["sec_label"]), int(k["dport"]), int(k["protocol"]), int(k["egress"]))].Bytes
                    for k in keys], np.uint64)
    assert np.array_equal(gpk, pk * reps) and np.array_equal(gby, by * reps)
    pm.destroy()


# -------------------------------------------------------- config 3 ----
def test_config3_prefilter_1m_prefixes_1b_addresses(gpu):
    """1M mixed prefixes (700K v4 / 300K v6, dyn and fix maps), 1B addresses
    (700M v4 + 300M v6): 4M distinct addresses checked against the oracle,
    copied 250 times on the device."""
    torch = _torch()
    pfx = synth.lpm_prefixes()
    v4, v6, ep4, ep6 = synth.lpm_addresses(4_000_000, pfx, seed=303)
    pf = gpu.prefilter(dyn4=True, dyn6=True, max_lpm=1 << 20)
    pf.insert(0, pfx)
    pf.set_endpoints(ep4, ep6)
    o4, o6 = oracle.prefilter(pf.config, pfx, ep4, ep6, v4, v6, nthreads=16)
    reps = 250
    d4 = torch.from_numpy(np.ascontiguousarray(v4).reshape(-1).view(np.uint8)).cuda().repeat(reps)
    d6 = torch.from_numpy(np.ascontiguousarray(v6).reshape(-1).view(np.uint8)).cuda().repeat(reps)
    n4, n6 = len(v4) * reps, len(v6) * reps
    assert n4 + n6 == 1_000_000_000
    d_o4 = torch.empty(n4, dtype=torch.uint8, device="cuda")
    d_o6 = torch.empty(n6, dtype=torch.uint8, device="cuda")
    before = gpu.read_counters(2, pf.id)
    if len(before) == 0:  # counters appear with the first table build
        before = np.zeros(2, np.uint64)
    pf.verdicts_dev(d4, n4, d_o4, d6, n6, d_o6, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert bool((d_o4.view(reps, -1) == torch.from_numpy(o4).cuda()).all())
    assert bool((d_o6.view(reps, -1) == torch.from_numpy(o6).cuda()).all())
    c = gpu.read_counters(2, pf.id) - before
    drops = reps * (int((o4 == 1).sum()) + int((o6 == 1).sum()))
    assert int(c[0]) == drops and int(c[0] + c[1]) == 1_000_000_000
    del d4, d6, d_o4, d_o6
    pf.destroy()


# -------------------------------------------------------- config 4 ----
def test_config4_kafka_1k_rules_100m(gpu):
    """1K Kafka rules over 100M requests: 1M distinct requests checked
    against the oracle, copied 100 times on the device; the redirect's
    allowed/denied counters are 100 times the oracle's."""
    torch = _torch()
    pols, info = synth.kafka_policy(n_rules=1000)
    gpu.update_kafka_policy(pols)
    rq = synth.kafka_requests(1_000_000, info, seed=404)
    reqs, arena = gpu.pack_kafka(**rq)
    exp = oracle.KafkaOracle(pols).eval(**rq, nthreads=16)
    reps = 100
    d_r = torch.from_numpy(reqs.view(np.uint8)).cuda().repeat(reps)
    d_a = torch.from_numpy(arena).cuda()
    d_out = torch.empty(len(reqs) * reps, dtype=torch.uint8, device="cuda")
    gpu.reset_counters()
    gpu.kafka_verdicts_dev(d_r, len(reqs) * reps, d_a, d_out, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert bool((d_out.view(reps, -1) == torch.from_numpy(exp).cuda()).all())
    c = gpu.read_counters(1)
    assert int(c[0]) == reps * int(exp.sum()) and int(c[0] + c[1]) == reps * len(exp)


# -------------------------------------------------------- config 5 ----
def test_config5_http10k_125m_batch(gpu):
    """The 10K-rule set and one GPU's share of 1B requests (124.8M), laid out
    as the packer lays out a batch that size: 262,144 distinct requests
    checked against the oracle, every copy's verdict equal to its
    original's, and the program counters summing to the batch (allowed = the
    copies' multiple of the oracle's allowed count)."""
    torch = _torch()
    from bench import replicate_batch
    pols, info = synth.http10k_rules()
    gpu.update_http_policy(pols)
    D = 262_144
    rq = synth.http10k_requests(D, info, seed=505)
    b = gpu.pack_http(**rq)
    exp = oracle.HttpOracle(pols).eval(**rq, nthreads=16)
    reps = 476  # 476 x 262,144 = 124.8M
    dev = torch.device("cuda", 0)
    d_batch, nslots, _, _, groups = replicate_batch(b, reps, dev, torch, return_groups=True)
    d_arena = torch.from_numpy(b.arena).to(dev)
    d_out = torch.zeros(nslots, dtype=torch.uint8, device=dev)
    gpu.reset_counters()
    gpu.http_verdicts_dev(d_batch, nslots, d_arena, d_out, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    # expected verdict per slot of b (padding slots: 0)
    slot_exp = np.zeros(b.nslots, np.uint8)
    real = b.order < D
    slot_exp[real] = exp[b.order[real]]
    tiles_out = d_out.view(-1, 64)
    slot_exp_t = torch.from_numpy(slot_exp.reshape(-1, 64)).to(dev)
    for first, nt, at in groups:
        # tile-major replication (bench.replicate_batch): b's tile first + j
        # is tiles at + j * reps ... at + j * reps + reps - 1
        got = tiles_out[at:at + nt * reps].view(nt, reps, 64)
        assert bool((got == slot_exp_t[first:first + nt].unsqueeze(1)).all()), (first, nt)
    c = gpu.read_counters(0)
    assert int(c[0::2].sum() + c[1::2].sum()) == reps * D
    assert int(c[0::2].sum()) == reps * int(exp.sum())
    del d_batch, d_out
