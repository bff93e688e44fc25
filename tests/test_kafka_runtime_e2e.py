"""test/runtime/kafka.go:149-200 and test/k8sT/KafkaPolicies.go:150-247 end to
end (tests/golden/kafka_runtime_kat.json):
the policy files → Repository → the kafka endpoint's ingress map (9092
redirected to the Kafka proxy) and its redirect's rules (redirect.go:68-82)
→ the requests that decide what the runtime test observes, and which
endpoints have policy enforcement on.  CPU: the oracle and the compiled
tables' host walks; GPU: l4_fp_kernel and kafka_kernel.
"""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import resolve as R
from cilium_amd.classifier import L4_TUPLE_DTYPE
from cilium_amd.policy import htons
from kat_util import load
from test_policy_merge import _keys_ports

KAT = load("kafka_runtime_kat.json")
PROXY = {(True, "TCP", KAT["port"]): 15010}


def _world(suite):
    names = suite.get("containers", KAT["containers"])
    ids = {n: 256 + i for i, n in enumerate(names)}
    ids["host"] = R.RESERVED_HOST
    cache = {R.RESERVED_HOST: {"reserved:host": ""}, R.RESERVED_WORLD: {"reserved:world": ""}}
    for n in names:
        cache[ids[n]] = suite["labels"][n] if "labels" in suite else {f"container:id.{n}": ""}
    return names, ids, cache


def _resolve(suite):
    names, ids, cache = _world(suite)
    # allow-localhost "auto": "policy" outside Kubernetes (the runtime suites),
    # "always" under it (daemon.go:1144-1147)
    always = "labels" in suite
    repo = R.Repository([R.Rule.from_json(r) for r in suite["policy"]], R.PolicyConfig(always_allow_localhost=always))
    enforced = {n: list(repo.get_rules_matching(cache[ids[n]])) for n in names}
    maps = {n: _keys_ports(R.endpoint_policy_map_state(repo, cache[ids[n]], cache, PROXY)) for n in names}
    f = repo.resolve_l4_ingress_policy(cache[ids["kafka"]])[f"{KAT['port']}/TCP"]
    assert f.L7Parser == R.PARSER_KAFKA
    redirect = R.kafka_redirect("kafka-9092-ingress", f, cache)
    reqs = suite["requests"]
    rq = dict(redirect=[0] * len(reqs), remote=[ids[q["from"]] for q in reqs], api_key=[q["api_key"] for q in reqs],
              api_version=[q["api_version"] for q in reqs], kind=[q["kind"] for q in reqs],
              client_id=[q["client_id"].encode() for q in reqs], topics=[[t.encode() for t in q["topics"]] for q in reqs])
    want = np.array([q["allow"] for q in reqs], np.uint8)
    return ids, enforced, maps, redirect, rq, want


def _l4_expect(suite, ids):
    t = np.zeros(len(suite["l4"]), L4_TUPLE_DTYPE)
    for i, (src, _, port, _) in enumerate(suite["l4"]):
        t[i] = (ids[src], htons(port), 6, N.CG_L4_F_INGRESS, 100)
    kinds = [k for *_, k in suite["l4"]]
    return t, kinds


def _classify(v, kind):
    return {"redirect": v > 0, "drop": v < 0, "allow": v == 0}[kind]


def _check(suite, l4_fn, kafka_fn):
    ids, enforced, maps, redirect, rq, want = _resolve(suite)
    assert enforced == suite["enforced"]
    t, kinds = _l4_expect(suite, ids)
    for i, (_, dst, _, kind) in enumerate(suite["l4"]):
        v = int(l4_fn(dst, maps[dst], t[i:i + 1])[0])
        assert _classify(v, kind), (suite["l4"][i], v)
    got = kafka_fn(redirect, rq)
    bad = [q["note"] for q, g, w in zip(suite["requests"], got, want) if bool(g) != bool(w)]
    assert not bad, bad


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_kafka_runtime_oracle(suite):
    _check(suite, lambda dst, kp, t: oracle.l4(*kp, t, oracle.L4_INGRESS)[0],
           lambda red, rq: oracle.KafkaOracle([red]).eval(**rq))


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_kafka_runtime_host_tables(host, suite):
    def l4(dst, kp, t):
        pm = host.policy_map()
        pm.allow_keys(*kp)
        v = pm.eval_host_diag(t)
        pm.destroy()
        return v

    def kafka(red, rq):
        host.update_kafka_policy([red])
        return host.kafka_eval_host_diag(*host.pack_kafka(**rq))
    _check(suite, l4, kafka)


@pytest.mark.gpu
@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_gpu_kafka_runtime(gpu, suite):
    def l4(dst, kp, t):
        pm = gpu.policy_map()
        pm.allow_keys(*kp)
        v = pm.verdicts(t, mode=N.CG_L4_INGRESS)
        pm.destroy()
        return v

    def kafka(red, rq):
        gpu.update_kafka_policy([red])
        return gpu.kafka_verdicts(*gpu.pack_kafka(**rq))
    _check(suite, l4, kafka)
