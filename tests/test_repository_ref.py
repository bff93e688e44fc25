"""Repository resolution pinned to
pkg/policy/repository_test.go (tests/golden/repository_kat.json, written by
make_golden.py repository_kats()):

- TestCanReachIngress / TestCanReachEgress: every label decision;
- pkg/policy/rule_test.go TestL4Policy, TestMergeL4Policy{Ingress,Egress},
  TestMergeL7Policy{Ingress,Egress}: rule-level results (nil, error or the
  whole expected map);
- TestWildcardL3Rules*, TestWildcardL4Rules*, the FromEntities / ToEntities
  variants, TestL3DependentL4*FromRequires and TestMinikubeGettingStarted:
  the whole expected L4PolicyMap (ports, selectors in order, parser, L7 rules
  per selector, DerivedFromRules label lists);
- TestMinikubeGettingStarted carried on through NPDS → http_kernel and the
  endpoint's policy map → l4_fp_kernel (host walk on the CPU, the kernels on
  the GPU).
"""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import resolve as R
from cilium_amd.classifier import L4_TUPLE_DTYPE, POLICY_KEY_DTYPE
from cilium_amd.policy import L7Rules, PortRuleHTTP, PortRuleKafka, htons
from kat_util import load

KAT = load("repository_kat.json")
PROXY_PORT = 15001


def _rules(case):
    return [R.Rule.from_json(r) for r in case["rules"]]


def _l7(entry) -> L7Rules:
    http = [PortRuleHTTP(Path=h.get("path", ""), Method=h.get("method", "")) for h in entry["http"]] \
        if "http" in entry else None
    kafka = [PortRuleKafka(APIKey=k.get("apiKey", ""), Topic=k.get("topic", "")) for k in entry["kafka"]] \
        if "kafka" in entry else None
    if "l7proto" in entry:
        return L7Rules(L7Proto=entry["l7proto"], L7=list(entry["l7"]))
    return L7Rules(HTTP=http, Kafka=kafka)


# the unit tests run with option.Config's zero value: AllowLocalhost is not
# "always", so no host override selector is added (rule.go:166-172)
CFG = R.PolicyConfig(always_allow_localhost=False)


def _resolve(case):
    egress = case.get("dir") == "egress"
    if case["level"] == "rule":  # rule.resolveL4{In,E}gressPolicy into one result, in turn
        res, found = R.L4Policy(), None
        for r in _rules(case):
            r.sanitize()
            found = (R.resolve_rule_l4_egress(r, case["from"], (), res) if egress else
                     R.resolve_rule_l4_ingress(r, case["to"], (), res, CFG))
        if found is None:
            return None
        return found.Egress if egress else found.Ingress
    repo = R.Repository(_rules(case), CFG)
    if egress:
        return repo.resolve_l4_egress_policy(case["from"])
    return repo.resolve_l4_ingress_policy(case["to"], case.get("ctx_from"))


RESOLVE = [c for c in KAT["cases"] if c.get("level") in ("repo", "rule")]
REACH = [c for c in KAT["cases"] if c.get("kind") == "reach"]


@pytest.mark.parametrize("case", RESOLVE, ids=lambda c: c["case"])
def test_repository_resolution(case):
    if case.get("error"):
        with pytest.raises(R.PolicyMergeError):
            _resolve(case)
        return
    got = _resolve(case)
    if case["expect"] is None:
        assert got is None
        return
    assert set(got) == set(case["expect"])
    for key, want in case["expect"].items():
        f = got[key]
        assert (f.Port, f.Protocol, f.U8Proto, f.Ingress) == (want["port"], want["protocol"], want["u8proto"],
                                                             want["ingress"])
        assert f.Endpoints == [R.selector_from_json(s) for s in want["endpoints"]]
        assert f.L7Parser == want["parser"]
        assert dict(f.L7RulesPerEp) == {R.selector_from_json(e["sel"]): _l7(e) for e in want["l7"]}
        assert [tuple(x) for x in f.DerivedFromRules] == [tuple(sorted(d)) for d in want["derived_labels"]]


@pytest.mark.parametrize("case", REACH + [c for c in RESOLVE if "empty_repo" in c], ids=lambda c: c["case"])
def test_repository_reach(case):
    empty = R.Repository()
    for frm, to, decision, allowed in case.get("empty_repo", []):
        assert empty.can_reach_ingress(frm, to) == decision
        assert empty.allows_ingress_label_access(frm, to) == allowed
    if case.get("kind") != "reach":
        return
    repo = R.Repository(_rules(case))
    for frm, to, allowed in case["asserts"]:
        if case["dir"] == "ingress":
            assert repo.allows_ingress_label_access(frm, to) == allowed, (frm, to)
        else:
            assert repo.allows_egress_label_access(frm, to) == allowed, (frm, to)


# ----------------------------------- TestMinikubeGettingStarted → kernels ----
MK = next(c for c in KAT["cases"] if c["case"] == "MinikubeGettingStarted")
MK_IDS = {"app1": 300, "app2": 301, "app3": 302}
MK_CACHE = {i: {"id": n} for n, i in MK_IDS.items()}


def _mk_chain():
    """Endpoint app1's NPDS and policy map (port 80 redirected to the proxy);
    GET / and POST / from app2 and app3."""
    repo = R.Repository(_rules(MK), CFG)
    l4map = repo.resolve_l4_ingress_policy(MK["to"])
    npds = R.get_network_policy("ep-app1", MK_IDS["app1"], R.L4Policy(Ingress=l4map), True, False, MK_CACHE)
    state = R.endpoint_policy_map_state(repo, MK["to"], MK_CACHE, {(True, "TCP", 80): PROXY_PORT})
    srcs = list(MK["l7_outcome"]["allow"])
    blob, off, remote = b"", [0], []
    for s in srcs:
        for m in ("GET", "POST"):
            blob += b":method\0" + m.encode() + b"\0:path\0/\0"
            off.append(len(blob))
            remote.append(MK_IDS[s])
    n = len(remote)
    rq = dict(policy=np.zeros(n, np.uint32), ingress=np.ones(n, np.uint8), port=np.full(n, 80, np.uint16),
              remote=np.array(remote, np.uint32), hdr_blob=np.frombuffer(blob, np.uint8).copy(),
              hdr_off=np.array(off, np.uint64))
    want = np.array([a for s in srcs for a in MK["l7_outcome"]["allow"][s]], np.uint8)
    keys = np.zeros(len(state), POLICY_KEY_DTYPE)
    ports = np.zeros(len(state), np.uint16)
    for i, (k, p) in enumerate(state.items()):
        keys[i] = (k.Identity, htons(k.DestPort), k.Nexthdr, k.TrafficDirection)
        ports[i] = htons(p)
    t = np.zeros(len(srcs), L4_TUPLE_DTYPE)
    t["identity"] = [MK_IDS[s] for s in srcs]
    t["dport"] = htons(80)
    t["proto"] = 6
    t["flags"] = N.CG_L4_F_INGRESS
    t["len"] = 100
    exp_l4 = np.array([htons(PROXY_PORT) if any(MK["l7_outcome"]["allow"][s]) else -133 for s in srcs], np.int32)
    assert np.array_equal(oracle.HttpOracle([npds]).eval(**rq), want)
    assert np.array_equal(oracle.l4(keys, ports, t)[0], exp_l4)
    return npds, rq, want, keys, ports, t, exp_l4


def test_minikube_chain_host(host):
    npds, rq, want, keys, ports, t, exp_l4 = _mk_chain()
    host.update_http_policy([npds])
    assert np.array_equal(host.http_eval_host_diag(host.pack_http(**rq)), want)
    pm = host.policy_map()
    pm.allow_keys(keys, ports)
    assert np.array_equal(pm.eval_host_diag(t), exp_l4)


@pytest.mark.gpu
def test_gpu_minikube_chain(gpu):
    npds, rq, want, keys, ports, t, exp_l4 = _mk_chain()
    gpu.update_http_policy([npds])
    assert np.array_equal(gpu.http_verdicts(gpu.pack_http(**rq)), want)
    pm = gpu.policy_map()
    pm.allow_keys(keys, ports)
    assert np.array_equal(pm.verdicts(t), exp_l4)
    pm.destroy()


def test_add_search_delete():
    """repository_test.go:29-112 (TestAddSearchDelete): revisions, search and
    delete by rule labels."""
    repo = R.Repository()
    with pytest.raises(ValueError):
        repo.add(R.Rule(EndpointSelector=None))
    assert repo.revision == 1
    lbls1, lbls2 = ("tag1", "tag2"), ("tag3",)
    rule1 = R.Rule(R.EndpointSelector.of({"foo": ""}), Labels=lbls1)
    rule2 = R.Rule(R.EndpointSelector.of({"bar": ""}), Labels=lbls1)
    rule3 = R.Rule(R.EndpointSelector.of({"bar": ""}), Labels=lbls2)
    assert repo.add(rule1) == 2 and repo.add(rule2) == 3
    assert repo.search(lbls2) == []
    assert repo.add(rule3) == 4
    assert repo.search(lbls1) == [rule1, rule2] and repo.search(lbls2) == [rule3]
    assert repo.delete_by_labels(lbls1) == (5, 2)
    assert repo.delete_by_labels(lbls1) == (5, 0)
    assert repo.search(lbls2) == [rule3]
    assert repo.delete_by_labels(lbls2) == (6, 1)
    assert repo.search(lbls2) == []


def test_policy_command_labels():
    """test/runtime/Policies.go:1658-1712 ("Policy command"): three rules
    labelled key1..key3; each found by its label; deleting key2 leaves key1
    and key3; deleting everything then succeeds with nothing left."""
    doc = [{"endpointSelector": {"matchLabels": {"role": "frontend"}}, "labels": [k]} for k in ("key1", "key2", "key3")]
    repo = R.Repository([R.Rule.from_json(r) for r in doc])
    assert all(len(repo.search([k])) == 1 for k in ("key1", "key2", "key3"))
    assert repo.delete_by_labels(["key2"])[1] == 1 and repo.search(["key2"]) == []
    for k in ("key1", "key3"):
        assert len(repo.search([k])) == 1 and repo.delete_by_labels([k])[1] == 1
    assert repo.rules == [] and repo.delete_by_labels([])[1] == 0


def test_contains_all():
    """repository_test.go:114-191 (TestContainsAllRLocked); labels
    NewLabel(key, value, source) written "source:key=value"."""
    lab = lambda *ks: tuple(sorted(f"1:{k}={k}" for k in ks))  # noqa: E731
    a = [lab("1", "2", "3"), lab("4", "5", "6"), lab("7", "8", "9")]
    b = [lab("1", "2", "3"), lab("4", "5", "6")]
    sel = lambda k: R.EndpointSelector.of({k: ""})  # noqa: E731
    repo_a = R.Repository()
    for lbls, k in zip(a, ("foo", "bar", "bar")):
        repo_a.add(R.Rule(sel(k), Labels=lbls))
    repo_b = R.Repository()
    for lbls, k in zip(b, ("foo", "bar")):
        repo_b.add(R.Rule(sel(k), Labels=lbls))
    repo_empty = R.Repository()
    repo_empty.add(R.Rule(sel("bar")))
    assert repo_a.contains_all(b)
    assert not repo_b.contains_all(a)
    assert repo_a.contains_all([])
    assert repo_empty.contains_all([])
    assert not repo_empty.contains_all(a)


def _one(rule):
    return R.Repository([R.Rule.from_json(rule)], CFG)


def _L(*ks):
    return {k.split("=")[0]: (k.split("=", 1)[1] if "=" in k else "") for k in ks}


LOCAL_CLUSTER = f"k8s:{R.POLICY_LABEL_CLUSTER}=default"
OTHER_CLUSTER = f"k8s:{R.POLICY_LABEL_CLUSTER}=non-local"  # rule_test.go:34-35


def test_rule_can_reach():
    """rule_test.go:38-115 (TestRuleCanReach): a FromEndpoints selector of two
    labels, then FromRequires."""
    r1 = _one({"endpointSelector": {"matchLabels": {"bar": ""}},
               "ingress": [{"fromEndpoints": [{"matchLabels": {"foo": "", "foo2": ""}}]}]})
    assert r1.can_reach_ingress(_L("foo", "foo2"), _L("bar")) == "allowed"
    assert r1.can_reach_ingress(_L("foo"), _L("bar")) == "undecided"
    r2 = _one({"endpointSelector": {"matchLabels": {"bar": ""}},
               "ingress": [{"fromEndpoints": [{"matchLabels": {"foo": ""}}],
                            "fromRequires": [{"matchLabels": {"baz": ""}}]}]})
    assert r2.can_reach_ingress(_L("foo"), _L("bar")) == "denied"
    assert r2.can_reach_ingress(_L("baz"), _L("bar")) == "undecided"
    assert r2.can_reach_ingress(_L("foo", "baz"), _L("bar")) == "allowed"


def test_rule_can_reach_entities():
    """rule_test.go:1074-1166 (TestRuleCanReachFromEntity / ToEntity): world
    and this cluster's workloads, not another cluster's."""
    ing = _one({"endpointSelector": {"matchLabels": {"bar": ""}}, "ingress": [{"fromEntities": ["world", "cluster"]}]})
    assert ing.can_reach_ingress(_L("reserved:world"), _L("bar")) == "allowed"
    assert ing.can_reach_ingress(_L("foo", LOCAL_CLUSTER), _L("bar")) == "allowed"
    assert ing.can_reach_ingress(_L("foo", OTHER_CLUSTER), _L("bar")) == "undecided"
    eg = _one({"endpointSelector": {"matchLabels": {"bar": ""}}, "egress": [{"toEntities": ["world", "cluster"]}]})
    assert eg.can_reach_egress(_L("bar"), _L("reserved:world")) == "allowed"
    assert eg.can_reach_egress(_L("bar"), _L("foo", LOCAL_CLUSTER)) == "allowed"
    assert eg.can_reach_egress(_L("bar"), _L("foo", OTHER_CLUSTER)) == "undecided"


ALLOW_ALL_CASES = [  # rule_test.go: (name, ingress rules of the rule selecting id=c, {dport: allowed from id=a})
    ("IngressAllowAll:1504-1529", [{"fromEndpoints": [{}]}], {80: True, 90: True}),
    ("IngressAllowAllL4Overlap:1531-1563", [{"fromEndpoints": [{}]},
                                            {"toPorts": [{"ports": [{"port": "80", "protocol": "TCP"}]}]}],
     {80: True, 90: True}),
    ("IngressL4AllowAll:1565-1599", [{"toPorts": [{"ports": [{"port": "80", "protocol": "TCP"}]}]}],
     {80: True, 90: False}),
]


@pytest.mark.parametrize("case", ALLOW_ALL_CASES, ids=lambda c: c[0])
def test_ingress_allow_all_datapath(host, case):
    """The checkIngress decisions for a → c (c selected) as c's policy map
    decides them: the map state through the oracle and the compiled table."""
    from test_policy_merge import _keys_ports
    _, ingress, want = case
    ids = {"a": 300, "c": 301}
    cache = {300: {"id": "a"}, 301: {"id": "c"}}
    repo = R.Repository([R.Rule.from_json({"endpointSelector": {"matchLabels": {"id": "c"}}, "ingress": ingress})],
                        CFG)
    keys, ports = _keys_ports(R.endpoint_policy_map_state(repo, cache[301], cache))
    t = np.zeros(len(want), L4_TUPLE_DTYPE)
    for i, dport in enumerate(want):
        t[i] = (300, htons(dport), 6, N.CG_L4_F_INGRESS, 100)
    exp = [want[d] for d in want]
    assert [int(v) >= 0 for v in oracle.l4(keys, ports, t, oracle.L4_INGRESS)[0]] == exp
    pm = host.policy_map()
    pm.allow_keys(keys, ports)
    assert [int(v) >= 0 for v in pm.eval_host_diag(t)] == exp
    if case[0].startswith("IngressL4AllowAll"):  # :1589-1598
        f = repo.resolve_l4_ingress_policy(cache[301])["80/TCP"]
        assert (f.Port, f.Ingress, f.Endpoints) == (80, True, [R.WILDCARD])


P80 = [{"ports": [{"port": "80", "protocol": "TCP"}]}]
EGRESS_ALLOW_ALL_CASES = [  # rule_test.go: (name, egress rules of the id=a rule, {(dst, dport): allowed})
    ("EgressAllowAll:1601-1622", [{"toEndpoints": [{}]}], {("c", 80): True, ("c", 90): True}),
    ("EgressL4AllowAll:1623-1656", [{"toPorts": P80}], {("c", 80): True, ("c", 90): False}),
    ("EgressL4AllowWorld:1657-1705", [{"toEntities": ["world"], "toPorts": P80}],
     {("world", 80): True, ("world", 90): False, ("foo", 80): False, ("foo", 90): False}),
    ("EgressL4AllowAllEntity:1706-1754", [{"toEntities": ["all"], "toPorts": P80}],
     {("world", 80): True, ("world", 90): False, ("foo", 80): True, ("foo", 90): False}),
    ("EgressL3AllowWorld:1755-1790", [{"toEntities": ["world"]}],
     {("world", 80): True, ("world", 90): True, ("foo", 80): False, ("foo", 90): False}),
    ("EgressL3AllowAllEntity:1791-1834", [{"toEntities": ["all"]}],
     {("world", 80): True, ("world", 90): True, ("foo", 80): True, ("foo", 90): True}),
]


@pytest.mark.parametrize("case", EGRESS_ALLOW_ALL_CASES, ids=lambda c: c[0])
def test_egress_allow_all_datapath(host, case):
    """The checkEgress decisions from a as a's egress map decides them
    (policy_can_egress: the oracle wrapper and the compiled table)."""
    from test_policy_merge import _keys_ports
    _, egress, want = case
    ids = {"a": 300, "c": 301, "foo": 302, "world": R.RESERVED_WORLD}
    cache = {300: {"id": "a"}, 301: {"id": "c"}, 302: {"foo": ""}, R.RESERVED_WORLD: {"reserved:world": ""}}
    repo = R.Repository([R.Rule.from_json({"endpointSelector": {"matchLabels": {"id": "a"}}, "egress": egress})], CFG)
    keys, ports = _keys_ports(R.endpoint_policy_map_state(repo, cache[300], cache))
    t = np.zeros(len(want), L4_TUPLE_DTYPE)
    for i, (dst, dport) in enumerate(want):
        t[i] = (ids[dst], htons(dport), 6, 0, 100)
    exp = list(want.values())
    assert [int(v) >= 0 for v in oracle.l4(keys, ports, t, oracle.L4_EGRESS)[0]] == exp
    pm = host.policy_map()
    pm.allow_keys(keys, ports)
    assert [int(v) >= 0 for v in pm.eval_host_diag(t)] == exp
