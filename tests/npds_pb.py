"""Test helper: encode NPDS policies (the JSON form the engine takes) as a
serialized xDS DiscoveryResponse of Any-wrapped cilium.NetworkPolicy — the
protobuf wire format of envoy/cilium/npds.proto:31-182 and the Envoy v2
HeaderMatcher (pkg/envoy/envoy/api/v2/route/route.pb.go field numbers).
Written from the proto definitions; independent of the C++ decoder it tests."""
from __future__ import annotations


def varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def key(field: int, wt: int) -> bytes:
    return varint(field << 3 | wt)


def ld(field: int, payload: bytes) -> bytes:
    return key(field, 2) + varint(len(payload)) + payload


def vi(field: int, v: int) -> bytes:
    return key(field, 0) + varint(v)


def s(field: int, text) -> bytes:
    return ld(field, text.encode("latin-1") if isinstance(text, str) else bytes(text))


def zigzag_free_int64(v: int) -> int:
    """int64 as a protobuf varint (two's complement, 10 bytes when negative)."""
    return v & ((1 << 64) - 1)


def header_matcher(h: dict) -> bytes:
    out = s(1, h["name"])
    if "exact_match" in h:
        out += s(4, h["exact_match"])
    elif "regex_match" in h:
        out += s(5, h["regex_match"])
    elif "present_match" in h:
        out += vi(7, 1 if h["present_match"] else 0)
    elif "prefix_match" in h:
        out += s(9, h["prefix_match"])
    elif "suffix_match" in h:
        out += s(10, h["suffix_match"])
    elif "range_match" in h:
        r = h["range_match"]
        out += ld(6, vi(1, zigzag_free_int64(int(r.get("start", 0)))) + vi(2, zigzag_free_int64(int(r.get("end", 0)))))
    elif "value" in h:
        out += s(2, h["value"])
        if h.get("regex"):
            out += ld(3, vi(1, 1))
    if h.get("invert_match"):
        out += vi(8, 1)
    return out


def port_rule(r: dict, packed: bool = True) -> bytes:
    out = b""
    rem = r.get("remote_policies", [])
    if rem:
        out += ld(1, b"".join(varint(x) for x in rem)) if packed else b"".join(vi(1, x) for x in rem)
    if r.get("l7_proto"):
        out += s(2, r["l7_proto"])
    if "http_rules" in r:
        rules = b"".join(ld(1, b"".join(ld(1, header_matcher(h)) for h in hr.get("headers", [])))
                         for hr in r["http_rules"]["http_rules"])
        out += ld(100, rules)
    if "kafka_rules" in r:
        rules = b""
        for k in r["kafka_rules"]["kafka_rules"]:
            rules += ld(1, vi(1, k.get("api_key", 0)) + vi(2, k.get("api_version", 0)) + s(3, k.get("topic", "")) +
                        s(4, k.get("client_id", "")))
        out += ld(101, rules)
    if "l7_rules" in r:
        rules = b""
        for lr in r["l7_rules"]["l7_rules"]:
            m = b"".join(ld(1, s(1, k) + s(2, v)) for k, v in lr.get("rule", {}).items())
            rules += ld(1, m)
        out += ld(102, rules)
    return out


def port_policy(pp: dict, packed: bool = True) -> bytes:
    proto = pp.get("protocol", 0)
    proto = {"TCP": 0, "UDP": 1}.get(proto, proto) if isinstance(proto, str) else proto
    out = vi(1, pp.get("port", 0))
    if proto:
        out += vi(2, proto)
    for r in pp.get("rules", []):
        out += ld(3, port_rule(r, packed))
    return out


def network_policy(p: dict, packed: bool = True) -> bytes:
    out = s(1, p["name"]) + vi(2, p.get("policy", 0))
    for pp in p.get("ingress_per_port_policies", []):
        out += ld(3, port_policy(pp, packed))
    for pp in p.get("egress_per_port_policies", []):
        out += ld(4, port_policy(pp, packed))
    return out


TYPE_URL = "type.googleapis.com/cilium.NetworkPolicy"


def discovery_response(policies: list[dict], version: str = "1", packed: bool = True,
                       type_url: str = TYPE_URL) -> bytes:
    out = s(1, version)
    for p in policies:
        out += ld(2, s(1, type_url) + ld(2, network_policy(p, packed)))
    out += s(4, TYPE_URL) + s(5, "nonce")
    return out
