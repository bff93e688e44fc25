"""Known-answer tests from the reference's own tests, on the CPU: the oracle
must reproduce every reference assertion, and the engine's host-side
compilers (walked by the diagnostic table walkers — never a verdict path)
must agree with both."""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd.classifier import PreFilter
from cilium_amd.policy import PortRuleHTTP, PortRuleKafka, PolicyValidationError, get_http_rule
from kat_util import http_requests, kafka_case, load, lpm_case

HTTP = load("http_kat.json")


@pytest.mark.parametrize("suite", HTTP["suites"], ids=lambda s: s["name"])
def test_http_kat_oracle_and_compiler(host, suite):
    names = [p["name"] for p in suite["policy"]]
    rq = http_requests(suite["requests"], lambda n: names.index(n) if n in names else 0xFFFFFFFF)
    exp = np.array([r["expect"] for r in suite["requests"]], np.uint8)
    o = oracle.HttpOracle(suite["policy"]).eval(**rq)
    bad = [r["name"] + " @" + r["source"] for r, a, b in zip(suite["requests"], o, exp) if a != b]
    assert not bad, f"oracle disagrees with the reference assertions: {bad}"
    host.update_http_policy(suite["policy"])
    b = host.pack_http(**rq)
    g = host.http_eval_host_diag(b)
    assert np.array_equal(g, exp)


def test_http_rejected_policy(host):
    for case in HTTP["rejected_policies"]:
        with pytest.raises(ValueError):
            oracle.HttpOracle(case["policy"])
        with pytest.raises(N.CiliumGPUError) as ei:
            host.update_http_policy(case["policy"])
        assert ei.value.code == N.CG_POLICY_REJECTED


def test_translation_kat():
    t = load("translation_kat.json")
    for c in t["get_http_rule"]:
        got, _ = get_http_rule(PortRuleHTTP(**c["rule"]))
        assert got == c["expected"], c["source"]
    for c in t["sanitize_rejects"]:
        with pytest.raises(PolicyValidationError):
            PortRuleHTTP(**c["rule"]).sanitize()


def test_kafka_kat(host):
    k = load("kafka_kat.json")
    for c in k["matches_rule"]:
        pol, req = kafka_case(c)
        assert int(oracle.KafkaOracle(pol).eval(**req)[0]) == c["expect"], c["source"]
        host.update_kafka_policy(pol)
        reqs, arena = host.pack_kafka(**req)
        assert int(host.kafka_eval_host_diag(reqs, arena)[0]) == c["expect"], c["source"]


def test_kafka_sanitize_kat(host):
    for c in load("kafka_kat.json")["sanitize"]:
        rule = PortRuleKafka(Role=c["rule"].get("role", ""), APIKey=c["rule"].get("apiKey", ""),
                             APIVersion=c["rule"].get("apiVersion", ""), Topic=c["rule"].get("topic", ""))
        pol = [{"name": "r", "selectors": [{"identities": None, "rules": [rule]}]}]
        if c["valid"]:
            rule.sanitize()
            host.update_kafka_policy(pol)
            oracle.KafkaOracle(pol)
        else:
            with pytest.raises(PolicyValidationError):
                rule.sanitize()
            with pytest.raises(N.CiliumGPUError):
                host.update_kafka_policy(pol)
            with pytest.raises(ValueError):
                oracle.KafkaOracle(pol)


def test_lpm_kat(host):
    for c in load("lpm_kat.json")["covers"]:
        pfx, v4, ep4 = lpm_case(c)
        expect = 1 if c["covered"] else 2
        o4, _ = oracle.prefilter(N.CG_PF_DYN4 | N.CG_PF_FIX4 | N.CG_PF_FIX6, pfx, ep4, np.zeros((0, 16)), v4,
                                 np.zeros((0, 32)))
        assert int(o4[0]) == expect, c
        pf = host.prefilter(dyn4=True)
        pf.insert(0, pfx)
        pf.set_endpoints(ep4, np.zeros((0, 16), np.uint8))
        g4, _ = pf.eval_host_diag(v4, np.zeros((0, 32), np.uint8))
        assert int(g4[0]) == expect, c


def test_regex_vectors():
    """Engine regex compiler and the oracle against the committed vectors."""
    import ctypes as C
    res = C.c_uint8()
    for c in load("regex_vectors.json")["cases"]:
        p = c["pattern"].encode()
        for s, exp in zip(c["strings"], c["full_match"]):
            sb = s.encode()
            assert oracle.regex_match(p, sb) == exp
            buf = np.frombuffer(sb, np.uint8) if sb else np.zeros(1, np.uint8)
            assert N.lib.cg_diag_regex_match(p, len(p), buf.ctypes.data, len(sb), 0, C.byref(res)) == 0
            assert res.value == exp, (c["pattern"], s)


def test_oracle_l4_wrappers_branch_table():
    """The oracle's policy_can_access_ingress / policy_can_egress restatement
    (bpf/lib/policy.h:126-163) on the branch-table rows, against the values
    derived by hand from the reference's branch structure."""
    from test_gpu_parity import WRAPPER_EXPECT, wrapper_case
    from cilium_amd.policy import htons
    keys, ports, t = wrapper_case()
    for mode, want in WRAPPER_EXPECT.items():
        got, _, _ = oracle.l4(keys, ports, t, mode)
        assert got.tolist() == [htons(v) if v > 0 else v for v in want], mode
    # mode 0 is __policy_can_access itself: fragments and ingress misses keep their codes
    raw, _, _ = oracle.l4(keys, ports, t, 0)
    assert -157 in raw.tolist()
