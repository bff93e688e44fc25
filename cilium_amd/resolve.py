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

Identity caches are ``{numeric_identity: labels}`` with labels given as
``{"source:key": value}`` (or plain ``{"key": value}``, source "any").
"""
from __future__ import annotations

import functools
from dataclasses import dataclass, field
from typing import Iterable, Mapping, Optional

from .policy import (L7Rules, PolicyKey, PortRuleHTTP, PortRuleKafka, TrafficDirection, get_http_rule, htons,
                     port_network_policy_rule)

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
                    out_http += r.HTTP
                    out_kafka += r.Kafka
        r = self.get(WILDCARD)
        if r is not None:
            out_http += r.HTTP
            out_kafka += r.Kafka
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

    def is_redirect(self) -> bool:
        """l4.go:236-238"""
        return self.L7Parser != PARSER_NONE

    def allows_all_at_l3(self) -> bool:
        return selects_all(self.Endpoints)


def _rules_empty(r: Optional[L7Rules]) -> bool:
    return r is None or (not r.HTTP and not r.Kafka)


def create_l4_filter(peer_endpoints: list, rules: Optional[L7Rules], port: int, protocol: str,
                     ingress: bool) -> L4Filter:
    """CreateL4Filter (l4.go:162-200): a wildcard peer list becomes
    [WildcardEndpointSelector]; L7 rules only on TCP, parser HTTP > Kafka."""
    eps = [WILDCARD] if selects_all(peer_endpoints) else list(peer_endpoints)
    f = L4Filter(Port=int(port), Protocol=protocol, U8Proto=U8PROTO.get(protocol, 0), Endpoints=eps,
                 Ingress=ingress)
    if protocol == "TCP" and rules is not None:
        if rules.HTTP:
            f.L7Parser = PARSER_HTTP
        elif rules.Kafka:
            f.L7Parser = PARSER_KAFKA
        if not _rules_empty(rules):
            # addRulesForEndpoints (l4.go:143-156)
            for sel in eps:
                f.L7RulesPerEp[sel] = rules
    return f


def create_l4_ingress_filter(from_endpoints: list, endpoints_with_l3_override: list, rules: Optional[L7Rules],
                             port: int, protocol: str) -> L4Filter:
    """CreateL4IngressFilter (l4.go:209-223): selectors with an L3 override
    (host / world in the relevant modes) get wildcard L7 rules."""
    f = create_l4_filter(from_endpoints, rules, port, protocol, True)
    if not _rules_empty(rules):
        for sel in endpoints_with_l3_override:
            f.L7RulesPerEp[sel] = L7Rules()
    return f


def create_l4_egress_filter(to_endpoints: list, rules: Optional[L7Rules], port: int, protocol: str) -> L4Filter:
    return create_l4_filter(to_endpoints, rules, port, protocol, False)


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
    Envoy (:516-517)."""
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
    return port_network_policy_rule(remotes, http)


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
            if not r["remote_policies"] and "http_rules" not in r:
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


__all__ = [n for n in dir() if not n.startswith("_")] + ["PortRuleHTTP"]
