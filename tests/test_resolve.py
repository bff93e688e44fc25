"""Control-plane steps that feed the engine (cilium_amd/resolve.py), pinned by
the reference's own translation tests (pkg/envoy/server_test.go) and by the
policy-map key semantics of pkg/endpoint/policy.go.  No GPU needed."""
import numpy as np

import oracle
from cilium_amd import resolve as R
from cilium_amd.policy import L7Rules, PolicyKey, PortRuleHTTP, PortRuleKafka, TrafficDirection, htons

# pkg/envoy/server_test.go:38-53
HTTP1 = PortRuleHTTP(Path="/foo", Method="GET", Host="foo.cilium.io", Headers=["header2 value", "header1"])
HTTP2 = PortRuleHTTP(Path="/bar", Method="PUT")
# :55-98
H1 = [{"name": ":authority", "regex_match": "foo.cilium.io"}, {"name": ":method", "regex_match": "GET"},
      {"name": ":path", "regex_match": "/foo"}, {"name": "header1", "present_match": True},
      {"name": "header2", "exact_match": "value"}]
H2 = [{"name": ":method", "regex_match": "PUT"}, {"name": ":path", "regex_match": "/bar"}]
# :100-125
SEL1 = R.EndpointSelector.of({"k8s:app": "etcd"})
SEL2 = R.EndpointSelector.of({"k8s:version": "v1"})
L7_1 = L7Rules(HTTP=[HTTP1, HTTP2])
L7_2 = L7Rules(HTTP=[HTTP1])
CACHE = {1001: {"k8s:app": "etcd", "k8s:version": "v1"},
         1002: {"k8s:app": "etcd", "k8s:version": "v2"},
         1003: {"k8s:app": "cassandra", "k8s:version": "v1"}}


def _http(*hs):
    return {"http_rules": [{"headers": h} for h in hs]}


# :131-192
RULE1 = {"remote_policies": [1001, 1002], "http_rules": _http(H2, H1)}
RULE2 = {"remote_policies": [1001, 1003], "http_rules": _http(H1)}
RULE3 = {"remote_policies": [], "http_rules": _http(H2, H1)}
RULE4 = {"remote_policies": [1002], "http_rules": _http(H2, H1)}
RULE5 = {"remote_policies": [1002, 1003], "http_rules": _http(H2, H1)}
RULE6 = {"remote_policies": [1001, 1002]}


def _filter(port, proto, parser, per_ep):
    f = R.L4Filter(Port=port, Protocol=proto, U8Proto=R.U8PROTO[proto], L7Parser=parser)
    f.L7RulesPerEp.update(per_ep)
    f.Endpoints = list(per_ep)
    return f


# :194-247
MAP1 = {"80/TCP": _filter(80, "TCP", R.PARSER_HTTP, {SEL1: L7_1})}
MAP2 = {"8080/UDP": _filter(8080, "UDP", R.PARSER_HTTP, {SEL2: L7_2})}
MAP3 = {"80/UDP": _filter(80, "TCP", R.PARSER_HTTP, {R.WILDCARD: L7_1})}
MAP4 = {"80/TCP": _filter(80, "TCP", R.PARSER_NONE, {SEL1: L7Rules()})}
MAP5 = {"80/TCP": _filter(80, "TCP", R.PARSER_NONE, {R.WILDCARD: L7Rules()})}


def _pp(port, proto, *rules):
    return [{"port": port, "protocol": proto, "rules": list(rules)}]


def test_get_port_network_policy_rule():
    """TestGetPortNetworkPolicyRule (server_test.go:331-339)."""
    assert R.get_port_network_policy_rule(SEL1, R.PARSER_HTTP, L7_1, CACHE) == RULE1
    assert R.get_port_network_policy_rule(SEL2, R.PARSER_HTTP, L7_2, CACHE) == RULE2


def test_get_direction_network_policy():
    """TestGetDirectionNetworkPolicy (server_test.go:341-357)."""
    assert R.get_direction_network_policy(MAP1, True, CACHE) == _pp(80, "TCP", RULE1)
    assert R.get_direction_network_policy(MAP2, True, CACHE) == _pp(8080, "UDP", RULE2)
    assert R.get_direction_network_policy(MAP4, True, CACHE) == _pp(80, "TCP", RULE6)
    assert R.get_direction_network_policy(MAP5, True, CACHE) == _pp(80, "TCP")


def test_get_network_policy_variants():
    """TestGetNetworkPolicy* (server_test.go:359-434)."""
    pol1 = R.L4Policy(Ingress=MAP1, Egress=MAP2)
    pol2 = R.L4Policy(Ingress=MAP3, Egress=MAP2)
    base = {"name": "10.1.1.1", "policy": 123}
    eg = _pp(8080, "UDP", RULE2)
    assert R.get_network_policy("10.1.1.1", 123, pol1, True, True, CACHE) == \
        dict(base, ingress_per_port_policies=_pp(80, "TCP", RULE1), egress_per_port_policies=eg)
    assert R.get_network_policy("10.1.1.1", 123, pol2, True, True, CACHE) == \
        dict(base, ingress_per_port_policies=_pp(80, "TCP", RULE3), egress_per_port_policies=eg)
    assert R.get_network_policy("10.1.1.1", 123, pol1, True, True, CACHE, denied_ingress=[1001]) == \
        dict(base, ingress_per_port_policies=_pp(80, "TCP", RULE4), egress_per_port_policies=eg)
    assert R.get_network_policy("10.1.1.1", 123, pol2, True, True, CACHE, denied_ingress=[1001]) == \
        dict(base, ingress_per_port_policies=_pp(80, "TCP", RULE5), egress_per_port_policies=eg)
    assert R.get_network_policy("10.1.1.1", 123, None, True, True, CACHE, denied_ingress=[1001]) == base
    allow_all = [{"port": 0, "protocol": "TCP", "rules": []}, {"port": 0, "protocol": "UDP", "rules": []}]
    assert R.get_network_policy("10.1.1.1", 123, pol2, False, True, CACHE, denied_ingress=[1001]) == \
        dict(base, ingress_per_port_policies=allow_all, egress_per_port_policies=eg)
    assert R.get_network_policy("10.1.1.1", 123, pol2, True, False, CACHE, denied_ingress=[1001]) == \
        dict(base, ingress_per_port_policies=_pp(80, "TCP", RULE5), egress_per_port_policies=allow_all)


def test_selector_semantics():
    """EndpointSelector.Matches (selector.go:279-304) incl. reserved:all and
    match expressions."""
    assert R.WILDCARD.matches({"k8s:app": "x"}) and R.WILDCARD.is_wildcard()
    assert SEL1.matches(CACHE[1001]) and not SEL1.matches(CACHE[1003])
    assert R.EndpointSelector.of({"reserved:all": ""}).matches({})
    assert R.EndpointSelector.of({"any:app": "etcd"}).matches(CACHE[1002])
    assert not R.EndpointSelector.of({"cidr:app": "etcd"}).matches(CACHE[1002])
    ex = R.EndpointSelector.of(match_expressions=[("k8s:version", "NotIn", ["v1"])])
    assert [i for i in CACHE if ex.matches(CACHE[i])] == [1002]
    ex = R.EndpointSelector.of(match_expressions=[("k8s:app", "In", ["etcd", "cassandra"]),
                                                  ("k8s:tier", "DoesNotExist", [])])
    assert all(ex.matches(CACHE[i]) for i in CACHE)


def test_create_l4_filter_and_relevant_rules():
    """CreateL4Filter / CreateL4IngressFilter (l4.go:162-223) and
    GetRelevantRules (l4.go:118-141)."""
    rules = L7Rules(HTTP=[HTTP2])
    f = R.create_l4_ingress_filter([SEL1], [SEL2], rules, 80, "TCP")
    assert f.L7Parser == R.PARSER_HTTP and f.is_redirect() and f.Ingress
    assert f.L7RulesPerEp[SEL1] is rules and f.L7RulesPerEp[SEL2].is_empty()
    assert R.L7DataMap(f.L7RulesPerEp).get_relevant_rules(CACHE[1002]).HTTP == [HTTP2]
    assert R.L7DataMap(f.L7RulesPerEp).get_relevant_rules(None).HTTP == []
    # UDP: no L7 (l4.go:185); wildcard peers → [WildcardEndpointSelector]
    u = R.create_l4_filter([], rules, 53, "UDP", False)
    assert u.L7Parser == R.PARSER_NONE and not u.L7RulesPerEp and u.Endpoints == [R.WILDCARD]
    k = R.create_l4_filter([], L7Rules(Kafka=[PortRuleKafka(Topic="t")]), 9092, "TCP", True)
    assert k.L7Parser == R.PARSER_KAFKA
    lr = k.L7RulesPerEp.get_relevant_rules(None)
    assert [r.Topic for r in lr.Kafka] == ["t"]


def test_policymap_keys_and_sync(host):
    """convertL4FilterToPolicyMapKeys + computeDesired* (pkg/endpoint/policy.go)
    then syncPolicyMap (endpoint.go:2621-2701) into an engine policy map."""
    l4 = R.L4Policy(Ingress={"80/TCP": R.create_l4_ingress_filter([SEL1], [], L7Rules(HTTP=[HTTP2]), 80, "TCP"),
                             "53/UDP": R.create_l4_filter([SEL2], None, 53, "UDP", True)},
                    Egress={"443/TCP": R.create_l4_egress_filter([], None, 443, "TCP")})
    desired = R.compute_desired_l4_policymap_entries(l4, CACHE, {(True, "TCP", 80): 10001})
    assert desired[PolicyKey(1001, 80, 6, TrafficDirection.Ingress)] == 10001
    assert desired[PolicyKey(1003, 53, 17, TrafficDirection.Ingress)] == 0
    assert PolicyKey(1003, 80, 6, TrafficDirection.Ingress) not in desired
    assert all(PolicyKey(i, 443, 6, TrafficDirection.Egress) in desired for i in CACHE)
    # a redirect without an allocated port is skipped (policy.go:159-167)
    assert not any(k.DestPort == 80 for k in R.compute_desired_l4_policymap_entries(l4, CACHE, {}))
    R.determine_allow_localhost(desired, l4, False)
    R.determine_allow_from_world(desired, True)
    assert R.LOCALHOST_KEY in desired and R.WORLD_KEY in desired

    pm = host.policy_map()
    pm.allow(999, 22, 6, 0, 0)  # stale entry: removed by the sync
    realized = R.sync_policy_map(pm, desired)
    dumped = {PolicyKey(k.Identity, htons(k.DestPort), k.Nexthdr, k.TrafficDirection): htons(e.ProxyPort)
              for k, e in pm.dump_to_slice()}
    assert dumped == desired == realized
    # the engine's table now answers like the reference map would
    keys = np.array([(k.Identity, htons(k.DestPort), k.Nexthdr, k.TrafficDirection) for k in desired],
                    dtype=[("sec_label", "<u4"), ("dport", "<u2"), ("protocol", "u1"), ("egress", "u1")])
    ports = np.array([htons(p) for p in desired.values()], np.uint16)
    tup = np.zeros(4, dtype=[("identity", "<u4"), ("dport", "<u2"), ("proto", "u1"), ("flags", "u1"),
                             ("len", "<u4")])
    tup[0] = (1001, htons(80), 6, 1, 100)    # ingress, proxied
    tup[1] = (1002, htons(53), 17, 1, 100)   # ingress: 1002 is v2 → no key
    tup[2] = (1003, htons(443), 6, 0, 100)   # egress to any
    tup[3] = (2, htons(8080), 6, 1, 100)     # world L3 key
    got = pm.eval_host_diag(tup)
    exp, _, _ = oracle.l4(keys, ports, tup)
    assert got.tolist() == exp.tolist() == [htons(10001), -133, 0, 0]


def test_npds_from_resolution_compiles(host):
    """getNetworkPolicy output is accepted by cg_http_policy_update and the
    compiled tables agree with the oracle on requests covering each rule."""
    pol = R.get_network_policy("ep", 123, R.L4Policy(Ingress=MAP1, Egress=MAP2), True, True, CACHE)
    host.update_http_policy([pol])
    from cilium_amd import synth
    reqs = [
        (1001, [(b":method", b"PUT"), (b":path", b"/bar")]),
        (1003, [(b":method", b"PUT"), (b":path", b"/bar")]),
        (1002, [(b":method", b"GET"), (b":path", b"/foo"), (b":authority", b"foo.cilium.io"),
                (b"header1", b""), (b"header2", b"value")]),
        (1002, [(b":method", b"GET"), (b":path", b"/foo"), (b":authority", b"foo.cilium.io"),
                (b"header2", b"value")]),
    ]
    blob, off = synth._blob([h for _, h in reqs])
    n = len(reqs)
    rq = dict(policy=np.zeros(n, np.uint32), ingress=np.ones(n, np.uint8), port=np.full(n, 80, np.uint16),
              remote=np.array([r for r, _ in reqs], np.uint32), hdr_blob=blob, hdr_off=off)
    b = host.pack_http(**rq)
    got = host.http_eval_host_diag(b)
    exp = oracle.HttpOracle([pol]).eval(**rq)
    assert got.tolist() == exp.tolist() == [1, 0, 1, 0]


def test_kafka_redirect_resolution():
    f = R.create_l4_ingress_filter([SEL1], [], L7Rules(Kafka=[PortRuleKafka(Role="produce", Topic="a")]), 9092,
                                   "TCP")
    f.L7RulesPerEp[R.WILDCARD] = L7Rules(Kafka=[PortRuleKafka(APIKey="metadata")])
    rd = R.kafka_redirect("r", f, CACHE)
    sels = {(tuple(s["identities"]) if s["identities"] is not None else None): s["rules"] for s in rd["selectors"]}
    assert [r.Topic for r in sels[(1001, 1002)]] == ["a"]
    assert [r.APIKey for r in sels[None]] == ["metadata"]
