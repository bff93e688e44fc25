"""Control-plane steps that produce the engine's inputs (host side).

Restated from the reference so that a caller holding resolved L4 policy can
fill the device tables the way the agent fills the BPF map, Envoy's NPDS
cache and the Kafka redirect:

* ``EndpointSelector``          — pkg/policy/api/selector.go:279-379
* ``L4Filter`` / ``create_l4_filter`` / ``create_l4_ingress_filter``
                                — pkg/policy/l4.go:89-233
* ``L7DataMap.get_relevant_rules`` — pkg/policy/l4.go:118-141
* ``convert_l4_filter_to_policymap_keys``, ``compute_desired_l4_policymap_entries``,
  ``determine_allow_localhost`` / ``determine_allow_from_world``
                                — pkg/endpoint/policy.go:93-130,144-193,267-296
* ``sync_policy_map``           — pkg/endpoint/endpoint.go:2621-2701
* ``get_port_network_policy_rule``, ``get_direction_network_policy``,
  ``get_network_policy``        — pkg/envoy/server.go:476-622 (+ sort.go)
* ``kafka_redirect``            — pkg/proxy/redirect.go:68-82 (the L7DataMap a
  Kafka redirect holds), resolved to identity lists for cg_kafka_policy_update
* ``Rule`` / ``IngressRule`` / ``EgressRule`` / ``PortRule`` — pkg/policy/api
  (rule.go, ingress.go, egress.go, l4.go; JSON tags of the policy files)
* ``Repository``                — pkg/policy/repository.go: AddList,
  GetRulesMatching (:624-643), CanReachIngress/EgressRLocked (:80-99),
  AllowsIngress/EgressLabelAccess, ResolveL4Ingress/EgressPolicy (:245-330),
  wildcardL3L4Rule / wildcardL3L4Rules (:128-243); rule.go canReachIngress /
  canReachEgress (:352-440), resolveL4Ingress/EgressPolicy (:227-294,
  :521-566), mergeL4Ingress/Egress(Port) (:111-225, :442-519), mergeL4Port
  (:36-109)
* ``Endpoint`` policy compile   — pkg/endpoint/policy.go:195-371,616-639:
  ComputePolicyEnforcement, resolveL4Policy, computeDesiredPolicyMapState
  (L4 entries, localhost, world, L3 entries)

Identity caches are ``{numeric_identity: labels}`` with labels given as
``{"source:key": value}`` (or plain ``{"key": value}``, source "any").
"""
from __future__ import annotations

import functools
from dataclasses import dataclass, field
from typing import Iterable, Mapping, Optional

from .policy import (L7Rules, PolicyKey, PortRuleHTTP, PortRuleKafka, TrafficDirection, get_http_rule, go_fields,
                     htons, port_network_policy_rule)

# pkg/identity/numericidentity.go:27-75
RESERVED_UNKNOWN, RESERVED_HOST, RESERVED_WORLD, RESERVED_UNMANAGED, RESERVED_HEALTH, RESERVED_INIT = 0, 1, 2, 3, 4, 5
# pkg/u8proto/u8proto.go:24-29
U8PROTO = {"ANY": 0, "TCP": 6, "UDP": 17}
LABEL_RESERVED_ALL = "reserved:all"  # labels.LabelSourceReservedKeyPrefix + IDNameAll

PARSER_NONE, PARSER_HTTP, PARSER_KAFKA = "", "http", "kafka"  # pkg/policy/l4.go:80-87


def _split(key: str) -> tuple[str, str]:
    if ":" in key:
        src, k = key.split(":", 1)
        return src, k
    return "any", key


def _label_get(labels: Mapping[str, str], key: str) -> Optional[str]:
    """Value of the label selected by `key` ("source:key"; source "any"
    matches every source), or None."""
    src, k = _split(key)
    for lk, lv in labels.items():
        ls, lk2 = _split(lk)
        if lk2 == k and (src == "any" or ls == src or ls == "any"):
            return lv
    return None


@dataclass(frozen=True)
class EndpointSelector:
    """api.EndpointSelector: k8s LabelSelector (matchLabels +
    matchExpressions with In / NotIn / Exists / DoesNotExist)."""
    match_labels: tuple = ()       # ((key, value), ...)
    match_expressions: tuple = ()  # ((key, operator, (values...)), ...)

    @staticmethod
    def of(match_labels: Optional[Mapping[str, str]] = None,
           match_expressions: Iterable[tuple] = ()) -> "EndpointSelector":
        ml = tuple(sorted((match_labels or {}).items()))
        me = tuple((k, op, tuple(vs)) for k, op, vs in match_expressions)
        return EndpointSelector(ml, me)

    def is_wildcard(self) -> bool:
        """selector.go:307-310"""
        return not self.match_labels and not self.match_expressions

    def matches(self, labels: Mapping[str, str]) -> bool:
        """selector.go:279-304: reserved:all matches everything; otherwise
        every requirement must hold."""
        for k, _ in self.match_labels:
            if k == LABEL_RESERVED_ALL:
                return True
        for k, v in self.match_labels:
            if _label_get(labels, k) != v:
                return False
        for k, op, vs in self.match_expressions:
            got = _label_get(labels, k)
            if op == "In" and (got is None or got not in vs):
                return False
            if op == "NotIn" and got is not None and got in vs:
                return False
            if op == "Exists" and got is None:
                return False
            if op == "DoesNotExist" and got is not None:
                return False
        return True

    def label_selector_string(self) -> str:
        parts = [f"{k}={v}" for k, v in self.match_labels]
        parts += [f"{k} {op} ({','.join(vs)})" for k, op, vs in self.match_expressions]
        return ",".join(parts)


WILDCARD = EndpointSelector()


def selects_all(sels: Iterable[EndpointSelector]) -> bool:
    """EndpointSelectorSlice.SelectsAllEndpoints (selector.go:367-379)."""
    sels = list(sels)
    return not sels or any(s.is_wildcard() for s in sels)


class L7DataMap(dict):
    """map[EndpointSelector]api.L7Rules (pkg/policy/l4.go:32)."""

    def get_relevant_rules(self, labels: Optional[Mapping[str, str]]) -> L7Rules:
        """GetRelevantRules (l4.go:118-141): rules of every selector matching
        the identity's labels, then the wildcard selector's rules.  With
        labels None (unknown identity) only the wildcard rules apply.  The
        reference iterates a Go map (random order); the OR/AND semantics of
        the consumers make the order irrelevant."""
        out = L7Rules()
        out_http: list = []
        out_kafka: list = []
        if labels is not None:
            for sel, r in self.items():
                if sel.matches(labels):
                    out_http += r.HTTP or []
                    out_kafka += r.Kafka or []
        r = self.get(WILDCARD)
        if r is not None:
            out_http += r.HTTP or []
            out_kafka += r.Kafka or []
        out.HTTP, out.Kafka = out_http, out_kafka
        return out


@dataclass
class L4Filter:
    """policy.L4Filter (pkg/policy/l4.go:89-109)."""
    Port: int
    Protocol: str = "TCP"
    U8Proto: int = 6
    Endpoints: list = field(default_factory=list)
    L7Parser: str = PARSER_NONE
    L7RulesPerEp: L7DataMap = field(default_factory=L7DataMap)
    Ingress: bool = True
    DerivedFromRules: list = field(default_factory=list)  # labels.LabelArrayList

    def is_redirect(self) -> bool:
        """l4.go:236-238"""
        return self.L7Parser != PARSER_NONE

    def allows_all_at_l3(self) -> bool:
        return selects_all(self.Endpoints)


def _rules_empty(r: Optional[L7Rules]) -> bool:
    """L7Rules.IsEmpty (api/l4.go:95-99), a nil *L7Rules included."""
    return r is None or r.is_empty()


def create_l4_filter(peer_endpoints: list, rules: Optional[L7Rules], port: int, protocol: str,
                     ingress: bool, rule_labels=None) -> L4Filter:
    """CreateL4Filter (l4.go:162-200): a wildcard peer list becomes
    [WildcardEndpointSelector]; L7 rules only on TCP, parser HTTP > Kafka >
    the generic l7proto."""
    eps = [WILDCARD] if selects_all(peer_endpoints) else list(peer_endpoints)
    f = L4Filter(Port=int(port), Protocol=protocol, U8Proto=U8PROTO.get(protocol, 0), Endpoints=eps,
                 Ingress=ingress, DerivedFromRules=[rule_labels])
    if protocol == "TCP" and rules is not None:
        if rules.HTTP:
            f.L7Parser = PARSER_HTTP
        elif rules.Kafka:
            f.L7Parser = PARSER_KAFKA
        elif rules.L7Proto:
            f.L7Parser = rules.L7Proto
        if not _rules_empty(rules) and rules.len():
            # addRulesForEndpoints (l4.go:143-156): eps is never empty here
            for sel in eps:
                f.L7RulesPerEp[sel] = rules
    return f


def create_l4_ingress_filter(from_endpoints: list, endpoints_with_l3_override: list, rules: Optional[L7Rules],
                             port: int, protocol: str, rule_labels=None) -> L4Filter:
    """CreateL4IngressFilter (l4.go:209-223): selectors with an L3 override
    (host / world in the relevant modes) get wildcard L7 rules."""
    f = create_l4_filter(from_endpoints, rules, port, protocol, True, rule_labels)
    if not _rules_empty(rules):
        for sel in endpoints_with_l3_override:
            f.L7RulesPerEp[sel] = L7Rules()
    return f


def create_l4_egress_filter(to_endpoints: list, rules: Optional[L7Rules], port: int, protocol: str,
                            rule_labels=None) -> L4Filter:
    return create_l4_filter(to_endpoints, rules, port, protocol, False, rule_labels)


@dataclass
class L4Policy:
    """policy.L4Policy: Ingress/Egress L4PolicyMap keyed "port/proto"."""
    Ingress: dict = field(default_factory=dict)
    Egress: dict = field(default_factory=dict)

    def has_redirect(self) -> bool:
        return any(f.is_redirect() for f in list(self.Ingress.values()) + list(self.Egress.values()))


def get_security_identities(identity_cache: Mapping[int, Mapping[str, str]], sel: EndpointSelector) -> list[int]:
    """getSecurityIdentities (pkg/endpoint/policy.go:93-106)."""
    return sorted(i for i, lbls in identity_cache.items() if sel.matches(lbls))


def convert_l4_filter_to_policymap_keys(f: L4Filter, direction: TrafficDirection,
                                        identity_cache: Mapping[int, Mapping[str, str]]) -> list[PolicyKey]:
    """convertL4FilterToPolicyMapKeys (pkg/endpoint/policy.go:111-130).
    Keys are in HOST byte order, as the desired map state holds them."""
    keys = []
    for sel in f.Endpoints:
        for ident in get_security_identities(identity_cache, sel):
            keys.append(PolicyKey(ident, f.Port & 0xFFFF, f.U8Proto, int(direction)))
    return keys


def compute_desired_l4_policymap_entries(l4: L4Policy, identity_cache: Mapping[int, Mapping[str, str]],
                                         redirect_ports: Mapping[tuple, int]) -> dict[PolicyKey, int]:
    """computeDesiredL4PolicyMapEntries (policy.go:144-193).  redirect_ports
    maps (ingress, protocol, port) → the allocated proxy port (host order);
    a redirect without an allocated port is skipped until one exists."""
    out: dict[PolicyKey, int] = {}
    for filters, direction in ((l4.Ingress, TrafficDirection.Ingress), (l4.Egress, TrafficDirection.Egress)):
        for f in filters.values():
            for k in convert_l4_filter_to_policymap_keys(f, direction, identity_cache):
                proxy = 0
                if f.is_redirect():
                    proxy = int(redirect_ports.get((f.Ingress, f.Protocol, f.Port), 0))
                    if proxy == 0:
                        continue
                out[k] = proxy
    return out


LOCALHOST_KEY = PolicyKey(RESERVED_HOST, 0, 0, int(TrafficDirection.Ingress))   # policy.go:50-54
WORLD_KEY = PolicyKey(RESERVED_WORLD, 0, 0, int(TrafficDirection.Ingress))      # policy.go:56-60


def determine_allow_localhost(desired: dict, l4: Optional[L4Policy], always_allow_localhost: bool) -> None:
    """determineAllowLocalhost (policy.go:267-276)."""
    if always_allow_localhost or (l4 is not None and l4.has_redirect()):
        desired[LOCALHOST_KEY] = 0


def determine_allow_from_world(desired: dict, host_allows_world: bool) -> None:
    """determineAllowFromWorld (policy.go:286-296); run after localhost."""
    if host_allows_world and LOCALHOST_KEY in desired:
        desired[WORLD_KEY] = 0


def sync_policy_map(pm, desired: Mapping[PolicyKey, int], realized: Optional[dict] = None) -> dict:
    """syncPolicyMap (pkg/endpoint/endpoint.go:2621-2701) against a device
    PolicyMap: delete dumped keys absent from the desired state (dump keys are
    network order → host order for the lookup), then insert keys whose entry
    differs from the realized state.  Returns the new realized state."""
    realized = dict(realized or {})
    errors = []
    for k, _ in pm.dump_to_slice():
        host = PolicyKey(k.Identity, htons(k.DestPort), k.Nexthdr, k.TrafficDirection)
        if host not in desired:
            try:
                pm.delete_key(host)
                realized.pop(host, None)
            except Exception as e:  # collected like the reference's errors slice
                errors.append(e)
    for k, proxy in desired.items():
        if realized.get(k) != proxy:
            try:
                pm.allow_key(k, proxy)
                realized[k] = proxy
            except Exception as e:
                errors.append(e)
    if errors:
        raise RuntimeError(f"synchronizing desired PolicyMap state failed: {errors}")
    return realized


# ------------------------------------------------------------- NPDS (HTTP) --
def _hm_key(m: dict):
    # HeaderMatcherLess (sort.go:209-302)
    return (m["name"], m.get("exact_match", ""), m.get("regex_match", ""), bool(m.get("present_match", False)))


def _http_rule_cmp(a: list, b: list) -> int:
    # HTTPNetworkPolicyRuleLess (sort.go:163-184): length first, then matchers
    if len(a) != len(b):
        return -1 if len(a) < len(b) else 1
    for x, y in zip(a, b):
        kx, ky = _hm_key(x), _hm_key(y)
        if kx != ky:
            return -1 if kx < ky else 1
    return 0


def _pnpr_cmp(r1: dict, r2: dict) -> int:
    # PortNetworkPolicyRuleLess (sort.go:87-138): L3/L4-only before L7
    h1 = r1.get("http_rules")
    h2 = r2.get("http_rules")
    if h1 is None and h2 is not None:
        return -1
    if h1 is not None and h2 is None:
        return 1
    if h1 is not None and h2 is not None:
        l1, l2 = h1["http_rules"], h2["http_rules"]
        if len(l1) != len(l2):
            return -1 if len(l1) < len(l2) else 1
        for x, y in zip(l1, l2):
            c = _http_rule_cmp(x["headers"], y["headers"])
            if c:
                return c
    p1, p2 = r1.get("remote_policies", []), r2.get("remote_policies", [])
    if len(p1) != len(p2):
        return -1 if len(p1) < len(p2) else 1
    for x, y in zip(p1, p2):
        if x != y:
            return -1 if x < y else 1
    return 0


def _pnp_cmp(p1: dict, p2: dict) -> int:
    # PortNetworkPolicySlice.Less (sort.go:32-69)
    a = (0 if p1["protocol"] == "TCP" else 1, p1["port"])
    b = (0 if p2["protocol"] == "TCP" else 1, p2["port"])
    if a != b:
        return -1 if a < b else 1
    r1, r2 = p1.get("rules") or [], p2.get("rules") or []
    if len(r1) != len(r2):
        return -1 if len(r1) < len(r2) else 1
    for x, y in zip(r1, r2):
        c = _pnpr_cmp(x, y)
        if c:
            return c
    return 0


def get_port_network_policy_rule(sel: EndpointSelector, parser: str, rules: L7Rules,
                                 identity_cache: Mapping[int, Mapping[str, str]],
                                 denied: Iterable[int] = ()) -> Optional[dict]:
    """getPortNetworkPolicyRule (server.go:476-537).  None = no remote
    identity matches (rule discarded).  Kafka rules are not translated for
    Envoy (:516-517); any other parser's rules are key-value pairs
    (getL7Rule, :326-334) under `l7_proto`, unsorted (:519-533)."""
    denied = set(denied)
    remotes: list[int] = []
    if not sel.is_wildcard() or denied:
        remotes = sorted(i for i, lbls in identity_cache.items() if i not in denied and sel.matches(lbls))
        if not remotes:
            return None
    http = None
    if parser == PARSER_HTTP and rules.HTTP:
        hs = [get_http_rule(h)[0] or [] for h in rules.HTTP]
        hs.sort(key=functools.cmp_to_key(_http_rule_cmp))   # SortHTTPNetworkPolicyRules
        http = hs
    r = port_network_policy_rule(remotes, http)
    if parser not in (PARSER_NONE, PARSER_HTTP, PARSER_KAFKA) and rules.L7:
        r["l7_proto"] = parser
        r["l7_rules"] = {"l7_rules": [{"rule": dict(kv)} for kv in rules.L7]}
    return r


ALLOW_ALL_PORT_NETWORK_POLICY = [  # server.go:50-57: port 0, no rules
    {"port": 0, "protocol": "TCP", "rules": []},
    {"port": 0, "protocol": "UDP", "rules": []},
]


def get_direction_network_policy(l4map: Mapping[str, L4Filter], enforced: bool,
                                 identity_cache: Mapping[int, Mapping[str, str]],
                                 denied: Iterable[int] = ()) -> Optional[list]:
    """getDirectionNetworkPolicy (server.go:539-604)."""
    if not enforced:
        return [dict(p, rules=[]) for p in ALLOW_ALL_PORT_NETWORK_POLICY]
    if not l4map:
        return None
    out = []
    for f in l4map.values():
        pnp = {"port": int(f.Port), "protocol": "UDP" if f.Protocol == "UDP" else "TCP", "rules": []}
        allow_all = False
        # Go iterates L7RulesPerEp (a map) in random order; an allow-all rule
        # short-circuits (:567-580) whatever the order
        for sel, l7 in f.L7RulesPerEp.items():
            r = get_port_network_policy_rule(sel, f.L7Parser, l7, identity_cache, denied)
            if r is None:
                continue
            if not r["remote_policies"] and "http_rules" not in r and "l7_rules" not in r:  # rule.L7 == nil
                allow_all = True
                pnp["rules"] = []
                break
            pnp["rules"].append(r)
        if not allow_all and not pnp["rules"]:
            continue
        pnp["rules"].sort(key=functools.cmp_to_key(_pnpr_cmp))
        out.append(pnp)
    if not out:
        return None
    out.sort(key=functools.cmp_to_key(_pnp_cmp))
    return out


def get_network_policy(name: str, ident: int, l4: Optional[L4Policy], ingress_enforced: bool,
                       egress_enforced: bool, identity_cache: Mapping[int, Mapping[str, str]],
                       denied_ingress: Iterable[int] = (), denied_egress: Iterable[int] = ()) -> dict:
    """getNetworkPolicy (server.go:607-622): the NPDS resource for one
    endpoint; l4 None → no per-port policies (deny all)."""
    p: dict = {"name": name, "policy": int(ident)}
    if l4 is not None:
        ing = get_direction_network_policy(l4.Ingress, ingress_enforced, identity_cache, denied_ingress)
        eg = get_direction_network_policy(l4.Egress, egress_enforced, identity_cache, denied_egress)
        if ing is not None:
            p["ingress_per_port_policies"] = ing
        if eg is not None:
            p["egress_per_port_policies"] = eg
    return p


# -------------------------------------------------------------------- Kafka --
def kafka_redirect(name: str, f: L4Filter, identity_cache: Mapping[int, Mapping[str, str]]) -> dict:
    """The rules a Kafka redirect holds (redirect.go:68-82 copies
    L4Filter.L7RulesPerEp) with each selector resolved to its identities;
    the wildcard selector keeps identities None (rules for every source,
    including unknown ones — GetRelevantRules appends them always)."""
    sels = []
    for sel, l7 in f.L7RulesPerEp.items():
        rules = [r if isinstance(r, PortRuleKafka) else PortRuleKafka(**r) for r in (l7.Kafka or [])]
        if sel.is_wildcard():
            sels.append({"identities": None, "rules": rules})
        else:
            sels.append({"identities": get_security_identities(identity_cache, sel), "rules": rules})
    return {"name": name, "selectors": sels}


# ------------------------------------------------------------- api.Rule ----
class PolicyMergeError(ValueError):
    """mergeL4Port's conflicting-parser / conflicting-L7-type errors
    (rule.go:52-96); the whole resolution fails, as the reference's does."""


# EntitySelectorMapping (api/entity.go:71-84); "cluster" is filled in by
# init_entities (InitEntities, :128-140)
_ENTITY_SELECTORS = {
    "all": [EndpointSelector()],
    "world": [EndpointSelector.of({"reserved:world": ""})],
    "host": [EndpointSelector.of({"reserved:host": ""})],
    "init": [EndpointSelector.of({"reserved:init": ""})],
    "cluster": [],
}
POLICY_LABEL_CLUSTER = "io.cilium.k8s.policy.cluster"  # k8s/apis/cilium.io/const.go:35
DEFAULT_CLUSTER_NAME = "default"                       # defaults/cluster.go:19


def init_entities(cluster_name: str = DEFAULT_CLUSTER_NAME) -> None:
    """InitEntities (api/entity.go:128-140): the cluster entity is the host,
    init and unmanaged identities plus every workload labelled with this
    cluster's name (k8s:io.cilium.k8s.policy.cluster, which the Kubernetes
    workload labels carry: workloads/kubernetes.go:112)."""
    _ENTITY_SELECTORS["cluster"] = [EndpointSelector.of({"reserved:host": ""}),
                                    EndpointSelector.of({"reserved:init": ""}),
                                    EndpointSelector.of({"reserved:unmanaged": ""}),
                                    EndpointSelector.of({f"k8s:{POLICY_LABEL_CLUSTER}": cluster_name})]


init_entities()  # the daemon calls it with option.Config.ClusterName at start-up


def selector_from_json(d: Optional[dict]) -> EndpointSelector:
    """api.EndpointSelector from its JSON (a k8s LabelSelector)."""
    d = go_fields(d)
    me = [(e["key"], e["operator"], tuple(e.get("values") or ()))
          for e in map(go_fields, d.get("matchexpressions") or [])]
    return EndpointSelector.of(d.get("matchlabels") or {}, me)


def requirements_of(sel: EndpointSelector) -> tuple:
    """ConvertToLabelSelectorRequirementSlice (api/selector.go): matchLabels
    as In-requirements with one value, then the matchExpressions."""
    return tuple((k, "In", (v,)) for k, v in sel.match_labels) + tuple(sel.match_expressions)


def with_requirements(sel: EndpointSelector, reqs: tuple) -> EndpointSelector:
    """A copy of `sel` whose MatchExpressions carry `reqs` as well
    (rule.go:243-253, :530-541)."""
    return EndpointSelector(sel.match_labels, tuple(sel.match_expressions) + tuple(reqs))


@dataclass
class PortProtocol:
    """api.PortProtocol (api/l4.go:27-40)."""
    Port: str
    Protocol: str = "ANY"


def parse_l4_proto(p: str) -> str:
    """ParseL4Proto: "" → ANY, else upper-cased and validated."""
    if not p:
        return "ANY"
    u = p.upper()
    if u not in ("TCP", "UDP", "ANY"):
        raise ValueError(f'invalid protocol "{u}", must be {{ tcp | udp | any }}')
    return u


def parse_port(port: str) -> int:
    """strconv.ParseUint(port, 0, 16) as Go 1.10 has it: base 0 reads a
    "0x"/"0X" prefix as hex and a leading "0" as octal, else decimal; every
    remaining byte must be a digit of that base (no sign, space or '_'; the
    0b / 0o prefixes came in Go 1.13); the value must fit 16 bits."""
    s, base = port, 10
    if s[:1] == "0" and len(s) > 1 and s[1] in "xX":
        if len(s) < 3:
            raise ValueError(f"Unable to parse port: {port!r}")
        s, base = s[2:], 16
    elif s[:1] == "0":
        s, base = s[1:], 8
    if not port:
        raise ValueError(f"Unable to parse port: {port!r}")
    v = 0
    for c in s:
        o = ord(c)
        d = o - 48 if 48 <= o <= 57 else o - 87 if 97 <= o <= 122 else o - 55 if 65 <= o <= 90 else 99
        if d >= base:
            raise ValueError(f"Unable to parse port: {port!r}")
        v = v * base + d
        if v > 0xFFFF:
            raise ValueError(f"Unable to parse port: {port!r}")
    return v


@dataclass
class PortRule:
    """api.PortRule (api/l4.go:44-60)."""
    Ports: list = field(default_factory=list)   # [PortProtocol]
    Rules: Optional[L7Rules] = None


@dataclass
class IngressRule:
    """api.IngressRule (api/ingress.go); CIDR members are kept only to be
    refused by the label-based resolution (not on this path)."""
    FromEndpoints: list = field(default_factory=list)
    FromRequires: list = field(default_factory=list)
    FromEntities: list = field(default_factory=list)
    ToPorts: list = field(default_factory=list)
    FromCIDR: list = field(default_factory=list)

    def source_selectors(self) -> list:
        """GetSourceEndpointSelectors (ingress.go:111-115)."""
        out = list(self.FromEndpoints)
        for e in self.FromEntities:
            out += _ENTITY_SELECTORS.get(e, [])
        return out

    def is_label_based(self) -> bool:
        """IsLabelBased (ingress.go:120-122)."""
        return not self.FromRequires and not self.FromCIDR


@dataclass
class EgressRule:
    """api.EgressRule (api/egress.go)."""
    ToEndpoints: list = field(default_factory=list)
    ToRequires: list = field(default_factory=list)
    ToEntities: list = field(default_factory=list)
    ToPorts: list = field(default_factory=list)
    ToCIDR: list = field(default_factory=list)

    def destination_selectors(self) -> list:
        """GetDestinationEndpointSelectors (egress.go:139-143)."""
        out = list(self.ToEndpoints)
        for e in self.ToEntities:
            out += _ENTITY_SELECTORS.get(e, [])
        return out

    def is_label_based(self) -> bool:
        """IsLabelBased (egress.go:148-150)."""
        return not self.ToRequires and not self.ToCIDR


@dataclass
class Rule:
    """api.Rule (api/rule.go:32-64)."""
    EndpointSelector: EndpointSelector = field(default_factory=EndpointSelector)
    Ingress: list = field(default_factory=list)
    Egress: list = field(default_factory=list)
    Labels: tuple = ()

    @staticmethod
    def from_json(d: dict) -> "Rule":
        """A rule of a policy file (`cilium policy import` JSON)."""
        def ports(lst):
            out = []
            for pr in map(go_fields, lst or []):
                pps = [PortProtocol(str(p.get("port", "")), p.get("protocol", ""))
                       for p in map(go_fields, pr.get("ports") or [])]
                out.append(PortRule(pps, L7Rules.from_json(pr.get("rules"))))
            return out
        d = go_fields(d)  # json.Unmarshal's field matching (policy.go_fields)
        ing = [IngressRule([selector_from_json(x) for x in r.get("fromendpoints") or []],
                           [selector_from_json(x) for x in r.get("fromrequires") or []],
                           list(r.get("fromentities") or []), ports(r.get("toports")),
                           list(r.get("fromcidr") or []) + list(r.get("fromcidrset") or []))
               for r in map(go_fields, d.get("ingress") or [])]
        eg = [EgressRule([selector_from_json(x) for x in r.get("toendpoints") or []],
                         [selector_from_json(x) for x in r.get("torequires") or []],
                         list(r.get("toentities") or []), ports(r.get("toports")),
                         list(r.get("tocidr") or []) + list(r.get("tocidrset") or []) +
                         list(r.get("toservices") or []))
              for r in map(go_fields, d.get("egress") or [])]
        labels = tuple(sorted(str(x) for x in d.get("labels") or []))
        return Rule(selector_from_json(d.get("endpointselector")), ing, eg, labels)

    def sanitize(self) -> None:
        """Rule.Sanitize (rule_validation.go:37-69, :316-358): every port
        parses as a non-zero uint16, protocols are normalised (ParseL4Proto),
        L7 rules only on TCP, at most 40 ports per PortRule, L7 rule
        validation (PortRuleHTTP / PortRuleKafka Sanitize)."""
        for rs in (self.Ingress, self.Egress):
            for r in rs:
                for pr in r.ToPorts:
                    if len(pr.Ports) > 40:
                        raise ValueError("too many ports, the max is 40")
                    for pp in pr.Ports:
                        if pp.Port == "":
                            raise ValueError("Port must be specified")
                        if parse_port(pp.Port) == 0:
                            raise ValueError("Port cannot be 0")
                        pp.Protocol = parse_l4_proto(pp.Protocol)
                        if not _rules_empty(pr.Rules) and pp.Protocol != "TCP":
                            raise ValueError(f"L7 rules can only apply exclusively to TCP, not {pp.Protocol}")
                    if not _rules_empty(pr.Rules):  # L7Rules.sanitize (:277-313)
                        r, kinds = pr.Rules, 0
                        if r.HTTP is not None:
                            kinds += 1
                            for h in r.HTTP:
                                h.sanitize()
                        if r.Kafka is not None:
                            kinds += 1
                            for k in r.Kafka:
                                k.sanitize()
                        if r.L7 is not None and not r.L7Proto:
                            raise ValueError("'l7' may only be specified when a 'l7proto' is also specified")
                        if r.L7Proto:
                            kinds += 1
                            for kv in r.L7 or []:  # PortRuleL7.Sanitize (l7.go:27-34)
                                if "" in kv:
                                    raise ValueError("Empty key not allowed")
                        if kinds > 1:
                            raise ValueError("multiple L7 protocol rule types specified in single rule")


def _copy_l7(r: L7Rules) -> L7Rules:
    return L7Rules(HTTP=None if r.HTTP is None else list(r.HTTP), Kafka=None if r.Kafka is None else list(r.Kafka),
                   L7Proto=r.L7Proto, L7=None if r.L7 is None else list(r.L7))


def merge_l4_port(endpoints: list, existing: L4Filter, to_merge: L4Filter) -> None:
    """mergeL4Port (rule.go:36-109): L3 union (a wildcard absorbs all), the
    parsers must agree, L7 rules per selector appended without duplicates."""
    if existing.allows_all_at_l3() or to_merge.allows_all_at_l3():
        existing.Endpoints = [WILDCARD]
    else:
        existing.Endpoints = list(existing.Endpoints) + list(endpoints)
    if to_merge.L7Parser != PARSER_NONE:
        if existing.L7Parser == PARSER_NONE:
            existing.L7Parser = to_merge.L7Parser
        elif to_merge.L7Parser != existing.L7Parser:
            raise PolicyMergeError(f"Cannot merge conflicting L7 parsers ({to_merge.L7Parser}/{existing.L7Parser})")
    for sel, new in to_merge.L7RulesPerEp.items():
        if sel not in existing.L7RulesPerEp:
            existing.L7RulesPerEp[sel] = new
            continue
        ep = _copy_l7(existing.L7RulesPerEp[sel])
        if new.HTTP:
            if ep.Kafka or ep.L7Proto:
                raise PolicyMergeError("Cannot merge conflicting L7 rule types")
            for r in new.HTTP:
                if r not in (ep.HTTP or []):
                    ep.HTTP = (ep.HTTP or []) + [r]
        elif new.Kafka:
            if ep.HTTP or ep.L7Proto:
                raise PolicyMergeError("Cannot merge conflicting L7 rule types")
            for r in new.Kafka:
                if r not in (ep.Kafka or []):
                    ep.Kafka = (ep.Kafka or []) + [r]
        elif new.L7Proto:
            if ep.Kafka or ep.HTTP or (ep.L7Proto and ep.L7Proto != new.L7Proto):
                raise PolicyMergeError("Cannot merge conflicting L7 rule types")
            if not ep.L7Proto:
                ep.L7Proto = new.L7Proto
            for r in new.L7 or []:
                if r not in (ep.L7 or []):
                    ep.L7 = (ep.L7 or []) + [r]
        existing.L7RulesPerEp[sel] = ep


def _filter_key(pp: PortProtocol, proto: str) -> str:
    return f"{pp.Port}/{proto}"


def _merge_port(endpoints, override, r: PortRule, pp: PortProtocol, proto: str, labels, res: dict,
                ingress: bool) -> int:
    """mergeL4IngressPort (rule.go:121-141) / mergeL4EgressPort (:480-500)."""
    def create():
        port = parse_port(pp.Port)
        if ingress:
            return create_l4_ingress_filter(endpoints, override, r.Rules, port, proto, labels)
        return create_l4_egress_filter(endpoints, r.Rules, port, proto, labels)
    key = _filter_key(pp, proto)
    if key not in res:
        res[key] = create()
        return 1
    existing = res[key]
    merged = L4Filter(existing.Port, existing.Protocol, existing.U8Proto, list(existing.Endpoints),
                      existing.L7Parser, L7DataMap(existing.L7RulesPerEp), existing.Ingress,
                      list(existing.DerivedFromRules))
    merge_l4_port(endpoints, merged, create())
    merged.DerivedFromRules.append(labels)
    res[key] = merged
    return 1


def _merge_l4(peers: list, override: list, to_ports: list, labels, res: dict, ingress: bool) -> int:
    """mergeL4Ingress (rule.go:143-225) / mergeL4Egress (:442-478): every
    port of every PortRule; ANY becomes TCP then UDP."""
    if not to_ports:
        return 0
    found = 0
    for r in to_ports:
        for pp in r.Ports:
            protos = [pp.Protocol] if pp.Protocol != "ANY" else ["TCP", "UDP"]
            for proto in protos:
                found += _merge_port(peers, override, r, pp, proto, labels, res, ingress)
    return found


@dataclass
class PolicyConfig:
    """The daemon options that change resolution (pkg/option):
    AlwaysAllowLocalhost() and HostAllowsWorld (rule.go:166-172)."""
    always_allow_localhost: bool = True
    host_allows_world: bool = False
    enforcement: str = "default"  # option.Config.EnablePolicy: default | always | never


def resolve_rule_l4_ingress(r: Rule, to_labels, requirements: tuple, result: L4Policy,
                            cfg: PolicyConfig = PolicyConfig(), from_labels=None) -> Optional[L4Policy]:
    """rule.resolveL4IngressPolicy (rule.go:227-294): None when the rule does
    not select `to_labels` or contributes no filter; raises PolicyMergeError.
    `from_labels` is SearchContext.From: when given, an ingress rule whose
    source selectors all miss it contributes nothing (mergeL4Ingress,
    rule.go:152-157)."""
    if not r.EndpointSelector.matches(to_labels):
        return None
    override = []
    if cfg.always_allow_localhost:
        override.append(_ENTITY_SELECTORS["host"][0])
        if cfg.host_allows_world:
            override.append(_ENTITY_SELECTORS["world"][0])
    found = 0
    for ing in r.Ingress:
        if requirements:
            ing = IngressRule([with_requirements(sel, requirements) for sel in ing.FromEndpoints], ing.FromRequires,
                              ing.FromEntities, ing.ToPorts, ing.FromCIDR)
        peers = ing.source_selectors()
        if from_labels is not None and ing.ToPorts and peers and not any(p.matches(from_labels) for p in peers):
            continue
        found += _merge_l4(peers, override, ing.ToPorts, r.Labels, result.Ingress, True)
    return result if found else None


def resolve_rule_l4_egress(r: Rule, from_labels, requirements: tuple, result: L4Policy) -> Optional[L4Policy]:
    """rule.resolveL4EgressPolicy (rule.go:521-566)."""
    if not r.EndpointSelector.matches(from_labels):
        return None
    found = 0
    for eg in r.Egress:
        if requirements:
            eg = EgressRule([with_requirements(sel, requirements) for sel in eg.ToEndpoints], eg.ToRequires,
                            eg.ToEntities, eg.ToPorts, eg.ToCIDR)
        peers = eg.destination_selectors()
        found += _merge_l4(peers, [], eg.ToPorts, r.Labels, result.Egress, False)
    return result if found else None


def wildcard_l3l4_rule(proto: str, port: int, endpoints: list, labels, l4map: dict) -> None:
    """wildcardL3L4Rule (repository.go:128-166): a redirecting filter on the
    port (any port when 0) gets an allow-all L7 rule for selectors allowed at
    L3 (or L3/L4) only: HTTP [{}], a sanitized empty Kafka rule, or an
    empty list of the generic parser's rules."""
    for k, f in list(l4map.items()):
        if proto != f.Protocol or (port != 0 and port != f.Port):
            continue
        if f.L7Parser == PARSER_NONE:
            continue
        per_ep = L7DataMap(f.L7RulesPerEp)
        for sel in endpoints:
            if f.L7Parser == PARSER_HTTP:
                per_ep[sel] = L7Rules(HTTP=[PortRuleHTTP()])
            elif f.L7Parser == PARSER_KAFKA:
                kr = PortRuleKafka()
                kr.sanitize()
                per_ep[sel] = L7Rules(Kafka=[kr])
            else:
                per_ep[sel] = L7Rules(L7Proto=f.L7Parser, L7=[])
        l4map[k] = L4Filter(f.Port, f.Protocol, f.U8Proto, list(f.Endpoints) + list(endpoints), f.L7Parser, per_ep,
                            f.Ingress, list(f.DerivedFromRules) + [labels])


class Repository:
    """policy.Repository (pkg/policy/repository.go): an ordered rule list."""

    def __init__(self, rules: Iterable[Rule] = (), cfg: Optional[PolicyConfig] = None):
        self.rules: list[Rule] = []
        self.cfg = cfg or PolicyConfig()
        self.revision = 1  # NewPolicyRepository (repository.go:41-45)
        rules = list(rules)
        if rules:
            self.add_list(rules)

    def add_list(self, rules: Iterable[Rule]) -> int:
        """AddListLocked after PolicyAdd's Sanitize (daemon/policy.go:171):
        all or nothing, one revision for the list."""
        rules = list(rules)
        for r in rules:
            if r.EndpointSelector is None:  # Rule.Sanitize (rule_validation.go:39-41)
                raise ValueError("rule cannot have nil EndpointSelector")
            r.sanitize()
        self.rules += rules
        self.revision += 1
        return self.revision

    def add(self, rule: Rule) -> int:
        """Add (repository.go:531-547): the new revision; a rule that does
        not sanitize is refused and the revision stays."""
        return self.add_list([rule])

    def search(self, labels) -> list[Rule]:
        """SearchRLocked (repository.go:495-505): the rules whose labels
        contain every one of `labels`."""
        need = set(labels)
        return [r for r in self.rules if need <= set(r.Labels)]

    def contains_all(self, needed) -> bool:
        """ContainsAllRLocked (repository.go:507-526): every label array of
        `needed` contains the labels of some rule that has labels."""
        return all(any(r.Labels and set(r.Labels) <= set(n) for r in self.rules) for n in needed)

    def delete_by_labels(self, labels) -> tuple[int, int]:
        """DeleteByLabelsLocked (repository.go:566-586): (revision, deleted);
        the revision moves only when something was deleted."""
        need = set(labels)
        keep = [r for r in self.rules if not need <= set(r.Labels)]
        n = len(self.rules) - len(keep)
        if n:
            self.rules = keep
            self.revision += 1
        return self.revision, n

    def get_rules_matching(self, labels) -> tuple[bool, bool]:
        """GetRulesMatching (:624-643): (ingress, egress) enforcement."""
        ing = eg = False
        for r in self.rules:
            if r.EndpointSelector.matches(labels):
                ing = ing or bool(r.Ingress)
                eg = eg or bool(r.Egress)
        return ing, eg

    def can_reach_ingress(self, from_labels, to_labels) -> str:
        """CanReachIngressRLocked (:80-99) over rule.canReachIngress
        (rule.go:352-395): "allowed" / "denied" / "undecided"."""
        decision = "undecided"
        for r in self.rules:
            d = self._rule_reach(r.EndpointSelector, r.Ingress, to_labels, from_labels, True)
            if d == "denied":
                return "denied"
            if d == "allowed":
                decision = "allowed"
        return decision

    def can_reach_egress(self, from_labels, to_labels) -> str:
        """CanReachEgressRLocked over rule.canReachEgress (rule.go:399-440)."""
        decision = "undecided"
        for r in self.rules:
            d = self._rule_reach(r.EndpointSelector, r.Egress, from_labels, to_labels, False)
            if d == "denied":
                return "denied"
            if d == "allowed":
                decision = "allowed"
        return decision

    @staticmethod
    def _rule_reach(subject: EndpointSelector, dir_rules: list, subject_labels, peer_labels, ingress: bool) -> str:
        if not subject.matches(subject_labels):
            return "undecided"
        for dr in dir_rules:
            for sel in (dr.FromRequires if ingress else dr.ToRequires):
                if not sel.matches(peer_labels):
                    return "denied"
        for dr in dir_rules:
            for sel in (dr.source_selectors() if ingress else dr.destination_selectors()):
                if sel.matches(peer_labels) and not dr.ToPorts:
                    return "allowed"
        return "undecided"

    def allows_ingress_label_access(self, from_labels, to_labels) -> bool:
        """AllowsIngressLabelAccess (:111-127)."""
        return bool(self.rules) and self.can_reach_ingress(from_labels, to_labels) == "allowed"

    def allows_egress_label_access(self, from_labels, to_labels) -> bool:
        """AllowsEgressLabelAccess."""
        return bool(self.rules) and self.can_reach_egress(from_labels, to_labels) == "allowed"

    def resolve_l4_ingress_policy(self, to_labels, from_labels=None) -> dict:
        """ResolveL4IngressPolicy (:245-281): FromRequires of every rule
        selecting to_labels constrain every FromEndpoints selector; rules are
        merged in order; then wildcardL3L4Rules.  `from_labels`: the search
        context's From (None for endpoint regeneration, which sets only To)."""
        reqs: tuple = ()
        for r in self.rules:
            if r.EndpointSelector.matches(to_labels):
                for ing in r.Ingress:
                    for sel in ing.FromRequires:
                        reqs += requirements_of(sel)
        result = L4Policy()
        for r in self.rules:
            resolve_rule_l4_ingress(r, to_labels, reqs, result, self.cfg, from_labels)
        self._wildcard_l3l4_rules(to_labels, True, result.Ingress)
        return result.Ingress

    def resolve_l4_egress_policy(self, from_labels) -> dict:
        """ResolveL4EgressPolicy (:289-330)."""
        reqs: tuple = ()
        for r in self.rules:
            if r.EndpointSelector.matches(from_labels):
                for eg in r.Egress:
                    for sel in eg.ToRequires:
                        reqs += requirements_of(sel)
        result = L4Policy()
        for r in self.rules:
            resolve_rule_l4_egress(r, from_labels, reqs, result)
        self._wildcard_l3l4_rules(from_labels, False, result.Egress)
        return result.Egress

    def _wildcard_l3l4_rules(self, labels, ingress: bool, l4map: dict) -> None:
        """wildcardL3L4Rules (:170-243)."""
        for r in self.rules:
            if not r.EndpointSelector.matches(labels):
                continue
            for dr in (r.Ingress if ingress else r.Egress):
                if not dr.is_label_based():
                    continue
                peers = dr.source_selectors() if ingress else dr.destination_selectors()
                if not dr.ToPorts:
                    wildcard_l3l4_rule("TCP", 0, peers, r.Labels, l4map)
                    wildcard_l3l4_rule("UDP", 0, peers, r.Labels, l4map)
                else:
                    for tp in dr.ToPorts:
                        if _rules_empty(tp.Rules):
                            for pp in tp.Ports:
                                wildcard_l3l4_rule(pp.Protocol, parse_port(pp.Port), peers, r.Labels, l4map)


def compute_policy_enforcement(repo: Repository, labels) -> tuple[bool, bool]:
    """Endpoint.ComputePolicyEnforcement (pkg/endpoint/policy.go:616-639):
    "always" enforces both directions, "never" neither; "default" enforces
    both for an endpoint still labelled reserved:init, else the directions
    some rule selecting it has rules for (GetRulesMatching)."""
    mode = repo.cfg.enforcement
    if mode == "always":
        return True, True
    if mode == "default":
        if "reserved:init" in labels:
            return True, True
        return repo.get_rules_matching(labels)
    return False, False


def endpoint_policy_map_state(repo: Repository, labels, identity_cache: Mapping[int, Mapping[str, str]],
                              redirect_ports: Optional[Mapping[tuple, int]] = None) -> dict[PolicyKey, int]:
    """One endpoint's desired policy map state, as regeneratePolicy computes
    it (pkg/endpoint/policy.go:482-560): ComputePolicyEnforcement
    (GetRulesMatching, default enforcement mode), resolveL4Policy for the
    enforced directions, then computeDesiredPolicyMapState — L4 entries,
    localhost, world, and L3 entries for every identity (an unenforced
    direction allows every identity)."""
    ing_on, eg_on = compute_policy_enforcement(repo, labels)
    l4 = L4Policy(Ingress=repo.resolve_l4_ingress_policy(labels) if ing_on else {},
                  Egress=repo.resolve_l4_egress_policy(labels) if eg_on else {})
    desired = compute_desired_l4_policymap_entries(l4, identity_cache, redirect_ports or {})
    determine_allow_localhost(desired, l4, repo.cfg.always_allow_localhost)
    determine_allow_from_world(desired, repo.cfg.host_allows_world)
    for ident, peer in identity_cache.items():
        if not ing_on or repo.allows_ingress_label_access(peer, labels):
            desired[PolicyKey(int(ident), 0, 0, int(TrafficDirection.Ingress))] = 0
        if not eg_on or repo.allows_egress_label_access(labels, peer):
            desired[PolicyKey(int(ident), 0, 0, int(TrafficDirection.Egress))] = 0
    return desired


__all__ = [n for n in dir() if not n.startswith("_")] + ["PortRuleHTTP"]
