"""test/runtime/cassandra.go:127-170 end to end (tests/golden/cassandra_runtime_kat.json):
the cassandra policy files → Repository → the server endpoint's NPDS
(key-value L7 rules under l7_proto "cassandra") → proxylib's policy
translation → each cqlsh request path through http_kernel.  The rules have
no fromEndpoints, so any client identity is subject to them; enforcement is
on for the server only.
"""
import numpy as np
import pytest

from cilium_amd import proxylib as P
from cilium_amd import resolve as R
from kat_util import load
from oracle.proxylib_ref import ProxylibOracle

KAT = load("cassandra_runtime_kat.json")
PORT = KAT["port"]
IDS = {"cass-server": 300, "cass-client": 301}
CACHE = {300: {"container:id.cass-server": ""}, 301: {"container:id.cass-client": ""},
         R.RESERVED_HOST: {"reserved:host": ""}}


def _npds(suite):
    repo = R.Repository([R.Rule.from_json(r) for r in suite["policy"]], R.PolicyConfig(always_allow_localhost=False))
    assert [repo.get_rules_matching(CACHE[i]) for i in (300, 301)] == [(True, False), (False, False)]
    lbl = CACHE[IDS["cass-server"]]
    l4 = R.L4Policy(Ingress=repo.resolve_l4_ingress_policy(lbl), Egress={})
    npds = R.get_network_policy("ep-cass", IDS["cass-server"], l4, True, False, CACHE)
    rule = npds["ingress_per_port_policies"][0]["rules"][0]
    assert rule["l7_proto"] == "cassandra" and rule["remote_policies"] == []
    return npds


def _want(suite):
    return np.array([o["allow"] for o in suite["ops"]], np.uint8)


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_cassandra_runtime_oracle(suite):
    o = ProxylibOracle([_npds(suite)])
    got = [o.matches_path("ep-cass", True, PORT, IDS["cass-client"], op["path"].encode()) for op in suite["ops"]]
    assert got == [bool(w) for w in _want(suite)], [op["note"] for op, g in zip(suite["ops"], got) if g != op["allow"]]


def _run(cl, suite, host_diag):
    pl = P.ProxylibPolicy(cl)
    pl.update([_npds(suite)])
    n = len(suite["ops"])
    fields = [P.cassandra_request(op["path"].encode()) for op in suite["ops"]]
    got = pl.matches_fields([pl.index("ep-cass")] * n, [1] * n, [PORT] * n, [IDS["cass-client"]] * n, fields,
                            host_diag=host_diag)
    bad = [op["note"] for op, g, w in zip(suite["ops"], got, _want(suite)) if bool(g) != bool(w)]
    assert not bad, bad


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_cassandra_runtime_host_tables(host, suite):
    _run(host, suite, True)


@pytest.mark.gpu
@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_gpu_cassandra_runtime(gpu, suite):
    _run(gpu, suite, False)
