"""Host-side mirror of the reference's rule types and their translation.

Field names and JSON tags follow the reference so callers can switch over:

* ``PortRuleHTTP``   — pkg/policy/api/http.go:28-84
* ``PortRuleKafka``  — pkg/policy/api/kafka.go:26-293, rule_validation.go:232-275
* ``L7Rules``        — pkg/policy/api/l4.go:65-85
* ``get_http_rule``  — pkg/envoy/server.go:336-399 (+ SortHeaderMatchers, sort.go:209-300)
* ``PolicyKey`` / ``PolicyEntry`` / ``TrafficDirection`` — pkg/maps/policymap
* NPDS builders      — envoy/cilium/npds.proto:31-182 (protobuf-JSON field names)

These are control-plane helpers: they build the JSON the engine compiles.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from enum import IntEnum
from typing import Iterable, Optional


class PolicyValidationError(ValueError):
    pass


# ------------------------------------------------------------------- HTTP --
@dataclass
class PortRuleHTTP:
    """api.PortRuleHTTP (pkg/policy/api/http.go:28-60)."""
    Path: str = ""
    Method: str = ""
    Host: str = ""
    Headers: list[str] = field(default_factory=list)

    def sanitize(self) -> None:
        """PortRuleHTTP.Sanitize (http.go:66-84): Path and Method must compile
        as Go regexps (regexp.Compile: Go 1.10 regexp/syntax, checked by the
        engine's Go front end, cg_regex_validate); Host and Headers are not
        validated."""
        from . import _native as N
        for what, v in (("path", self.Path), ("method", self.Method)):
            if v:
                try:
                    N.regex_validate(v, N.CG_REGEX_GO)
                except N.CiliumGPUError as e:
                    raise PolicyValidationError(f"invalid {what} regexp {v!r}: {e}") from e

    def to_json(self) -> dict:
        d: dict = {}
        if self.Path:
            d["path"] = self.Path
        if self.Method:
            d["method"] = self.Method
        if self.Host:
            d["host"] = self.Host
        if self.Headers:
            d["headers"] = list(self.Headers)
        return d


def _header_matcher_key(m: dict):
    # HeaderMatcherLess (pkg/envoy/sort.go:209-300): name, exact, regex, ..., present
    return (m["name"], m.get("exact_match", ""), m.get("regex_match", ""), bool(m.get("present_match", False)))


def get_http_rule(h: PortRuleHTTP) -> tuple[Optional[list[dict]], str]:
    """getHTTPRule (pkg/envoy/server.go:336-399): PortRuleHTTP → sorted Envoy
    HeaderMatchers (Path→:path regex, Method→:method regex, Host→:authority
    regex, each Headers entry "Name: value" → exact, "Name" → present)."""
    headers: list[dict] = []
    ref = ""
    if h.Path:
        headers.append({"name": ":path", "regex_match": h.Path})
        ref = f'PathRegexp("{h.Path}")'
    if h.Method:
        headers.append({"name": ":method", "regex_match": h.Method})
        ref += (" && " if ref else "") + f'MethodRegexp("{h.Method}")'
    if h.Host:
        headers.append({"name": ":authority", "regex_match": h.Host})
        ref += (" && " if ref else "") + f'HostRegexp("{h.Host}")'
    for hdr in h.Headers:
        strs = hdr.split(" ", 1)
        ref += (" && " if ref else "") + 'Header("'
        if len(strs) == 2:
            key = strs[0].rstrip(":")
            headers.append({"name": key, "exact_match": strs[1]})
            ref += key + '","' + strs[1]
        else:
            headers.append({"name": strs[0], "present_match": True})
            ref += strs[0]
        ref += '")'
    if not headers:
        return None, ref
    headers.sort(key=_header_matcher_key)
    return headers, ref


# ------------------------------------------------------------------ Kafka --
# KafkaAPIKeyMap, pkg/policy/api/kafka.go:153-188
KAFKA_API_KEY_MAP = {
    "produce": 0, "fetch": 1, "offsets": 2, "metadata": 3, "leaderandisr": 4, "stopreplica": 5,
    "updatemetadata": 6, "controlledshutdown": 7, "offsetcommit": 8, "offsetfetch": 9, "findcoordinator": 10,
    "joingroup": 11, "heartbeat": 12, "leavegroup": 13, "syncgroup": 14, "describegroups": 15, "listgroups": 16,
    "saslhandshake": 17, "apiversions": 18, "createtopics": 19, "deletetopics": 20, "deleterecords": 21,
    "initproducerid": 22, "offsetforleaderepoch": 23, "addpartitionstotxn": 24, "addoffsetstotxn": 25,
    "endtxn": 26, "writetxnmarkers": 27, "txnoffsetcommit": 28, "describeacls": 29, "createacls": 30,
    "deleteacls": 31, "describeconfigs": 32, "alterconfigs": 33,
}
KAFKA_MAX_TOPIC_LEN = 255
# api/kafka.go:244, the Go raw string `^[a-zA-Z0-9\\._\\-]+$`; Go's '$' is the
# end of text (Python's would also take a final "\n"), hence \Z
_KAFKA_TOPIC_VALID = re.compile(r"^[a-zA-Z0-9\\._\\-]+\Z")


@dataclass
class PortRuleKafka:
    """api.PortRuleKafka (pkg/policy/api/kafka.go:26-107)."""
    Role: str = ""
    APIKey: str = ""
    APIVersion: str = ""
    ClientID: str = ""
    Topic: str = ""

    def sanitize(self) -> None:
        """PortRuleKafka.Sanitize (rule_validation.go:232-275)."""
        if self.APIKey and self.Role:
            raise PolicyValidationError(f'Cannot set both Role:"{self.Role}" and APIKey :"{self.APIKey}" together')
        if self.APIKey and self.APIKey.lower() not in KAFKA_API_KEY_MAP:
            raise PolicyValidationError(f'invalid Kafka APIKey :"{self.APIKey}"')
        if self.Role and self.Role.lower() not in ("produce", "consume"):
            raise PolicyValidationError(f'invalid Kafka APIRole :"{self.Role}"')
        if self.APIVersion:
            if not re.fullmatch(r"[+-]?[0-9]+", self.APIVersion) or not -32768 <= int(self.APIVersion) <= 32767:
                raise PolicyValidationError(f'invalid Kafka APIVersion :"{self.APIVersion}"')
        if self.Topic:
            if len(self.Topic) > KAFKA_MAX_TOPIC_LEN:
                raise PolicyValidationError("kafka topic exceeds maximum len of 255")
            if not _KAFKA_TOPIC_VALID.match(self.Topic):
                raise PolicyValidationError(f'invalid Kafka Topic name "{self.Topic}"')

    def to_json(self) -> dict:
        return {"role": self.Role, "apiKey": self.APIKey, "apiVersion": self.APIVersion,
                "clientID": self.ClientID, "topic": self.Topic}


def go_fields(d: Optional[dict]) -> dict:
    """A JSON object's members as encoding/json matches them to struct
    fields: a key names the field whose tag it equals under case folding
    (json.Unmarshal; the reference's policy files write "HTTP" for the `http`
    tag, test/runtime/manifests/Policies-l7-simple.json:14), and of several
    keys naming one field the last decoded wins.  Keys are returned
    lower-cased; callers look up lower-case tags.  Label maps (matchLabels)
    are data, not fields, and are not passed through this."""
    return {k.lower(): v for k, v in (d or {}).items()}


@dataclass
class L7Rules:
    """api.L7Rules (pkg/policy/api/l4.go:65-85).  None stands for Go's nil
    slice: IsEmpty (l4.go:96-99) tells a nil list from an empty one."""
    HTTP: Optional[list[PortRuleHTTP]] = None
    Kafka: Optional[list[PortRuleKafka]] = None
    L7Proto: str = ""
    L7: Optional[list[dict]] = None  # []PortRuleL7 (key/value maps)

    def len(self) -> int:
        """Len (l4.go:87-93)."""
        return len(self.HTTP or []) + len(self.Kafka or []) + len(self.L7 or [])

    def is_empty(self) -> bool:
        """IsEmpty (l4.go:95-99): every rule list nil."""
        return self.HTTP is None and self.Kafka is None and self.L7 is None

    @staticmethod
    def from_json(d: Optional[dict]) -> Optional["L7Rules"]:
        """The `rules` member of an api.PortRule (JSON tags http, kafka,
        l7proto, l7; field names matched as encoding/json does: go_fields)."""
        if d is None:
            return None
        d = go_fields(d)
        http = [PortRuleHTTP(Path=h.get("path", ""), Method=h.get("method", ""), Host=h.get("host", ""),
                             Headers=list(h.get("headers") or [])) for h in map(go_fields, d["http"])] \
            if d.get("http") is not None else None
        kafka = [PortRuleKafka(Role=k.get("role", ""), APIKey=k.get("apikey", ""), APIVersion=k.get("apiversion", ""),
                               ClientID=k.get("clientid", ""), Topic=k.get("topic", ""))
                 for k in map(go_fields, d["kafka"])] if d.get("kafka") is not None else None
        l7 = [dict(x) for x in d["l7"]] if d.get("l7") is not None else None
        return L7Rules(HTTP=http, Kafka=kafka, L7Proto=d.get("l7proto", ""), L7=l7)


# -------------------------------------------------------------- policymap --
class TrafficDirection(IntEnum):
    """pkg/maps/policymap/trafficdirection.go:20-29"""
    Ingress = 0
    Egress = 1
    Invalid = 2


@dataclass(frozen=True)
class PolicyKey:
    """policymap.PolicyKey (policymap.go:64-69); DestPort in network byte order."""
    Identity: int
    DestPort: int
    Nexthdr: int
    TrafficDirection: int


@dataclass
class PolicyEntry:
    """policymap.PolicyEntry (policymap.go:73-80); ProxyPort in network byte order."""
    ProxyPort: int = 0
    Packets: int = 0
    Bytes: int = 0


def htons(v: int) -> int:
    """byteorder.HostToNetwork for uint16 on a little-endian host."""
    return ((v & 0xFF) << 8) | ((v >> 8) & 0xFF)


# ------------------------------------------------------------------- NPDS --
def header_matchers(rule: PortRuleHTTP) -> list[dict]:
    hs, _ = get_http_rule(rule)
    return hs or []


def port_network_policy_rule(remote_policies: Iterable[int] = (), http_rules: Optional[list[list[dict]]] = None
                             ) -> dict:
    """cilium.PortNetworkPolicyRule; http_rules=None leaves the L7 rule set
    unset (an L3/L4-only rule), [] installs an empty HTTP rule set."""
    r: dict = {"remote_policies": sorted(int(x) for x in remote_policies)}
    if http_rules is not None:
        r["http_rules"] = {"http_rules": [{"headers": hs} for hs in http_rules]}
    return r


def port_network_policy(port: int, rules: list[dict], protocol: str = "TCP") -> dict:
    return {"port": int(port), "protocol": protocol, "rules": rules}


def network_policy(name: str, policy: int = 0, ingress: Optional[list[dict]] = None,
                   egress: Optional[list[dict]] = None) -> dict:
    d: dict = {"name": name, "policy": int(policy)}
    if ingress is not None:
        d["ingress_per_port_policies"] = ingress
    if egress is not None:
        d["egress_per_port_policies"] = egress
    return d


def npds_json(policies: list[dict]) -> bytes:
    return json.dumps(policies, separators=(",", ":")).encode()


def matcher_kind(m: dict) -> tuple[str, str]:
    """Envoy HeaderData match type of an NPDS HeaderMatcher:
    ('E'|'R'|'P'|'X' prefix|'S' suffix|'N' range, value), the type followed by
    '!' for invert_match; a range's value is "start end"."""
    inv = "!" if m.get("invert_match") else ""
    if "exact_match" in m:
        return "E" + inv, m["exact_match"]
    if "regex_match" in m:
        return "R" + inv, m["regex_match"]
    if "prefix_match" in m:
        return "X" + inv, m["prefix_match"]
    if "suffix_match" in m:
        return "S" + inv, m["suffix_match"]
    if "range_match" in m:
        r = m["range_match"] or {}
        return "N" + inv, "%d %d" % (int(r.get("start", 0)), int(r.get("end", 0)))
    if "present_match" in m:
        return "P" + inv, ""
    if "value" in m:
        v = m["value"]
        if not v:
            return "P" + inv, ""
        rx = m.get("regex", False)
        if isinstance(rx, dict):
            rx = rx.get("value", False)
        return ("R" if rx else "E") + inv, v
    return "P" + inv, ""
