"""Per-rule hit counters (north_star: "all-reduce per-rule hit/deny
counters"; pkg/metrics/metrics.go:270-296, pkg/endpoint/endpoint.go:2207).

A request Envoy allows is attributed to the FIRST rule that allows it in
Envoy's evaluation order (cilium_network_policy.h:90-192: the port's
PortNetworkPolicyRules, then port 0's; each rule's HttpNetworkPolicyRules in
order).  The oracle restates that order rule by rule (oracle.cc
PortPolicy::first); the engine takes the lowest set bit of its rule masks.
CPU: the host walker's per-request attribution equals the oracle's.  GPU:
the kernel's counters equal the oracle's attributions counted per rule, and
the per-program allowed/denied counters agree with them."""
import random
from collections import Counter

import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import synth
from kat_util import http_requests, load
from test_cpu_differential import _rand_policy, _rand_requests


def _key_index(info):
    return {tuple(int(x) for x in r): i for i, r in enumerate(info)}


def _oracle_counts(pols, rq, info, nthreads=8):
    """Oracle attribution → per-rule-counter counts (same order as info)."""
    v, attr = oracle.HttpOracle(pols).eval_attr(**rq, nthreads=nthreads)
    idx = _key_index(info)
    counts = np.zeros(len(info), np.uint64)
    per_req = np.full(len(v), 0xFFFFFFFF, np.uint32)
    for i in np.nonzero(attr[:, 0] != 0xFFFFFFFF)[0]:
        k = (int(rq["policy"][i]), int(rq["ingress"][i])) + tuple(int(x) for x in attr[i])
        j = idx[k]
        counts[j] += 1
        per_req[i] = j
    return v, per_req, counts


def _host_case(host, pols, rq):
    host.update_http_policy(pols)
    b = host.pack_http(**rq)
    info = host.http_rule_info()
    v, per_req, _ = _oracle_counts(pols, rq, info)
    got = host.http_rules_host_diag(b)
    assert np.array_equal(host.http_eval_host_diag(b), v)
    assert np.array_equal(got, per_req)
    return info


@pytest.mark.parametrize("seed", range(10))
def test_first_rule_random_policies(host, seed):
    rng = random.Random(500 + seed)
    pols = _rand_policy(rng)
    rq = _rand_requests(rng, 800, len(pols))
    try:
        oracle.HttpOracle(pols)
    except ValueError:
        return
    _host_case(host, pols, rq)


def test_first_rule_kat_suites(host):
    for suite in load("http_kat.json")["suites"]:
        names = [p["name"] for p in suite["policy"]]
        rq = http_requests(suite["requests"], lambda n: names.index(n) if n in names else 0xFFFFFFFF)
        _host_case(host, suite["policy"], rq)


def test_rule_info_shapes(host):
    """A wildcard port without HTTP rules behind a port with HTTP rules gets
    a SCOPE_ALLOW counter; a PNPR without HTTP rules a NO_HTTP one; rules of
    port 0 appear once per exact-port program and once in port 0's own."""
    pols = [{"name": "p", "policy": 1, "ingress_per_port_policies": [
        {"port": 80, "rules": [{"http_rules": {"http_rules": [{"headers": [{"name": ":path", "exact_match": "/a"}]},
                                                              {"headers": [{"name": ":path", "exact_match": "/b"}]}]}},
                               {"remote_policies": [5], "http_rules": {"http_rules": []}}]},
        {"port": 0, "rules": [{"remote_policies": [7]}]}]}]
    host.update_http_policy(pols)
    info = [tuple(int(x) for x in r) for r in host.http_rule_info()]
    assert (0, 1, 80, 0, 0, 0) in info and (0, 1, 80, 0, 0, 1) in info
    assert (0, 1, 80, 0, 1, N.CG_HTTP_RULE_NO_HTTP) in info
    assert (0, 1, 80, 1, 0, N.CG_HTTP_RULE_SCOPE_ALLOW) in info
    rq = http_requests([{"policy": "p", "ingress": 1, "port": 80, "remote": r, "headers": [[":path", p]]}
                        for r, p in ((1, "/a"), (1, "/b"), (5, "/c"), (1, "/c"), (7, "/a"))], lambda n: 0)
    _host_case(host, pols, rq)


@pytest.mark.gpu
def test_gpu_rule_counters_10k(gpu):
    """10K-rule set, 300K requests: the kernel's per-rule hit counters equal
    the oracle's first-match attributions, and allowed = attributed hits +
    unattributed allows per program."""
    pols, info10 = synth.http10k_rules()
    rq = synth.http10k_requests(300_000, info10, seed=77, distinct=150_000)
    gpu.update_http_policy(pols)
    gpu.reset_counters()
    b = gpu.pack_http(**rq)
    got = gpu.http_verdicts(b)
    info = gpu.http_rule_info()
    v, _, counts = _oracle_counts(pols, rq, info, nthreads=16)
    assert np.array_equal(got, v)
    hits = gpu.http_rule_hits()
    assert np.array_equal(hits, counts)
    assert int(hits.sum()) == int(v.sum())  # every allowed request of this set is attributed
    allv = gpu.read_counters(N.CG_CTR_HTTP_ALLREDUCE)
    progs = gpu.read_counters(N.CG_CTR_HTTP_PROGRAMS)
    assert np.array_equal(allv[:len(progs)], progs) and np.array_equal(allv[len(progs) + 1:], hits)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_rule_counters_random(gpu, seed):
    rng = random.Random(900 + seed)
    pols = _rand_policy(rng)
    rq = _rand_requests(rng, 3000, len(pols))
    try:
        oracle.HttpOracle(pols)
    except ValueError:
        return
    gpu.update_http_policy(pols)
    gpu.reset_counters()
    got = gpu.http_verdicts(gpu.pack_http(**rq))
    info = gpu.http_rule_info()
    v, _, counts = _oracle_counts(pols, rq, info)
    assert np.array_equal(got, v)
    assert np.array_equal(gpu.http_rule_hits(), counts)


@pytest.mark.gpu
def test_gpu_per_request_rule_attribution_10k(gpu):
    """cg_http_verdicts_rules_*: every request's first matching rule from the
    kernel equals the oracle's first-match attribution (or_http_eval_attr,
    Envoy's evaluation order) and the host walker's (cg_diag_http_rules_host);
    verdicts unchanged."""
    pols, info10 = synth.http10k_rules()
    rq = synth.http10k_requests(200_000, info10, seed=91, distinct=100_000)
    gpu.update_http_policy(pols)
    b = gpu.pack_http(**rq)
    v, rule = gpu.http_verdicts_rules(b)
    info = gpu.http_rule_info()
    ov, per_req, _ = _oracle_counts(pols, rq, info, nthreads=16)
    assert np.array_equal(v, ov)
    assert np.array_equal(rule, per_req)
    assert np.array_equal(rule, gpu.http_rules_host_diag(b))
    assert 0.2 < (rule != 0xFFFFFFFF).mean() < 0.8


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_per_request_rule_attribution_random(gpu, seed):
    rng = random.Random(950 + seed)
    pols = _rand_policy(rng)
    rq = _rand_requests(rng, 3000, len(pols))
    try:
        oracle.HttpOracle(pols)
    except ValueError:
        return
    gpu.update_http_policy(pols)
    b = gpu.pack_http(**rq)
    v, rule = gpu.http_verdicts_rules(b)
    ov, per_req, _ = _oracle_counts(pols, rq, gpu.http_rule_info())
    assert np.array_equal(v, ov) and np.array_equal(rule, per_req)
