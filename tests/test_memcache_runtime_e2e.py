"""test/runtime/memcache.go:96-320 end to end (tests/golden/memcache_runtime_kat.json):
the memcache policy files → Repository → the memcache endpoint's NPDS
(getPortNetworkPolicyRule's key-value L7 rules under l7_proto "memcache",
server.go:519-533) → proxylib's policy translation → each client operation's
request frame through http_kernel, from the memcache-client identity.  The
L4 half: the client reaches 11211 through the proxy redirect.
"""
import numpy as np
import pytest

import oracle
from cilium_amd import proxylib as P
from cilium_amd import resolve as R
from cilium_amd.classifier import L4_TUPLE_DTYPE
from cilium_amd import _native as N
from cilium_amd.policy import htons
from kat_util import load
from test_policy_merge import _keys_ports

KAT = load("memcache_runtime_kat.json")
PORT = KAT["port"]
IDS = {"memcache": 300, "client": 301, "other": 302}
CACHE = {300: {"container:id.memcache": ""}, 301: {"container:memcache-client": ""}, 302: {"container:id.other": ""},
         R.RESERVED_HOST: {"reserved:host": ""}}


def _chain(suite):
    repo = R.Repository([R.Rule.from_json(r) for r in suite["policy"]], R.PolicyConfig(always_allow_localhost=False))
    lbl = CACHE[IDS["memcache"]]
    ing_on, eg_on = repo.get_rules_matching(lbl)
    l4 = R.L4Policy(Ingress=repo.resolve_l4_ingress_policy(lbl), Egress={})
    npds = R.get_network_policy("ep-memcache", IDS["memcache"], l4, ing_on, eg_on, CACHE)
    rule = npds["ingress_per_port_policies"][0]["rules"][0]
    assert rule["l7_proto"] == "memcache" and rule["remote_policies"] == [IDS["client"]]
    keys, ports = _keys_ports(R.endpoint_policy_map_state(repo, lbl, CACHE, {(True, "TCP", PORT): 15020}))
    ops = suite["ops"]
    fields = [P.memcache_request(o["command"].encode(), o["opcode"], [k.encode() for k in o["keys"]]) for o in ops]
    want = np.array([o["allow"] for o in ops], np.uint8)
    t = np.zeros(2, L4_TUPLE_DTYPE)
    t[0] = (IDS["client"], htons(PORT), 6, N.CG_L4_F_INGRESS, 100)
    t[1] = (IDS["other"], htons(PORT), 6, N.CG_L4_F_INGRESS, 100)
    return npds, fields, want, keys, ports, t


def _run(cl, suite, host_diag):
    npds, fields, want, keys, ports, t = _chain(suite)
    pl = P.ProxylibPolicy(cl)
    pl.update([npds])
    n = len(fields)
    args = ([pl.index("ep-memcache")] * n, [1] * n, [PORT] * n, [IDS["client"]] * n, fields)
    got = pl.matches_fields(*args, host_diag=host_diag)
    bad = [o["note"] for o, g, w in zip(suite["ops"], got, want) if bool(g) != bool(w)]
    assert not bad, bad
    pm = cl.policy_map()
    pm.allow_keys(keys, ports)
    v = pm.eval_host_diag(t) if host_diag else pm.verdicts(t, mode=N.CG_L4_INGRESS)
    pm.destroy()
    assert int(v[0]) == htons(15020) and int(v[1]) < 0, v  # client → proxy, anyone else dropped


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_memcache_runtime_oracle(suite):
    """The NPDS rules through oracle/memcache_ref.py (parser.go:35-110): a
    frame passes when a rule whose remotes include the client matches it."""
    from oracle import memcache_ref as MR
    npds, fields, want, keys, ports, t = _chain(suite)
    rules = [r for r in npds["ingress_per_port_policies"][0]["rules"] if IDS["client"] in r["remote_policies"]]
    mr = [MR.Rule(x["rule"]) for r in rules for x in r["l7_rules"]["l7_rules"]]
    got = [any(r.matches(MR.Meta(o["command"].encode(), o["opcode"], [k.encode() for k in o["keys"]])) for r in mr)
           for o in suite["ops"]]
    assert got == [bool(w) for w in want], [o["note"] for o, g, w in zip(suite["ops"], got, want) if g != w]
    v = oracle.l4(keys, ports, t, oracle.L4_INGRESS)[0]
    assert int(v[0]) == htons(15020) and int(v[1]) < 0


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_memcache_runtime_host_tables(host, suite):
    _run(host, suite, True)


@pytest.mark.gpu
@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_gpu_memcache_runtime(gpu, suite):
    _run(gpu, suite, False)
