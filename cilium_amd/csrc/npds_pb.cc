// npds_pb.cc — NPDS protobuf ingestion: an xDS DiscoveryResponse whose
// resources are Any-wrapped cilium.NetworkPolicy messages (the form Envoy's
// and proxylib's NPDS clients receive on StreamNetworkPolicies), decoded from
// the protobuf wire format into the engine's NPDS JSON.
//
//   envoy/cilium/npds.proto:31-182            the messages and field numbers
//   pkg/envoy/envoy/api/v2/route/route.pb.go  HeaderMatcher (name 1, value 2,
//                                             regex 3, exact 4, regex_match 5,
//                                             range 6, present 7, invert 8,
//                                             prefix 9, suffix 10)
//   pkg/envoy/cilium/npds.pb.validate.go      Validate(): port <= 65535, unique
//                                             remote_policies, at least one
//                                             http/kafka/l7 rule per list, Kafka
//                                             topic/client_id patterns
//   proxylib/proxylib/instance.go:180-215     every resource must unpack as a
//                                             NetworkPolicy, else the update fails
//
// Proto3 wire rules kept: unknown fields are skipped, repeated scalars may be
// packed or not, a repeated singular scalar's last occurrence wins, the
// occurrences of a singular embedded message merge (their bytes are
// concatenated and parsed once: HeaderMatcher.regex, range_match and the
// http_rules / kafka_rules / l7_rules oneof members, whose rule lists
// append), a oneof keeps its last member, map entries with the same key keep
// the last value.
//
// String fields and UTF-8: Envoy's C++ protobuf runtime rejects a proto3
// string field that is not valid UTF-8 at parse time, so the HTTP update
// (cg_http_policy_update_npds) refuses the whole response; golang/protobuf
// of the reference's era (proxylib, cg_proxylib_policy_update_npds) does not
// check, and those bytes pass through unchanged (the engine's JSON reader
// copies non-ASCII bytes verbatim).
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/cilium_gpu.h"
#include "common.h"
#include "http.h"

namespace cg {

namespace {

thread_local bool t_strict_utf8 = false;

bool utf8_ok(const std::string& s) {
  size_t i = 0, n = s.size();
  const auto* b = (const unsigned char*)s.data();
  while (i < n) {
    const unsigned c = b[i];
    size_t k;
    uint32_t cp;
    if (c < 0x80) { ++i; continue; }
    if ((c & 0xE0) == 0xC0) { k = 1; cp = c & 0x1F; }
    else if ((c & 0xF0) == 0xE0) { k = 2; cp = c & 0x0F; }
    else if ((c & 0xF8) == 0xF0) { k = 3; cp = c & 0x07; }
    else return false;
    if (n - i <= k) return false;  // truncated sequence
    for (size_t j = 1; j <= k; ++j) {
      if ((b[i + j] & 0xC0) != 0x80) return false;
      cp = cp << 6 | (b[i + j] & 0x3F);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && (cp < 0x10000 || cp > 0x10FFFF)) ||
        (cp >= 0xD800 && cp <= 0xDFFF))
      return false;
    i += k + 1;
  }
  return true;
}

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool done() const { return p >= e; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 70; s += 7) {
      if (p >= e) fail(CG_POLICY_REJECTED, "NPDS protobuf: truncated varint");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    fail(CG_POLICY_REJECTED, "NPDS protobuf: varint too long");
  }
  std::string bytes() {
    const uint64_t n = varint();
    if (n > (uint64_t)(e - p)) fail(CG_POLICY_REJECTED, "NPDS protobuf: truncated field");
    std::string s((const char*)p, (size_t)n);
    p += n;
    return s;
  }
  // next field: number and wire type; false at the end
  bool next(uint32_t* field, uint32_t* wt) {
    if (done()) return false;
    const uint64_t k = varint();
    *field = (uint32_t)(k >> 3);
    *wt = (uint32_t)(k & 7);
    if (*field == 0) fail(CG_POLICY_REJECTED, "NPDS protobuf: field number 0");
    return true;
  }
  void skip(uint32_t wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: need(8); p += 8; break;
      case 2: bytes(); break;
      case 5: need(4); p += 4; break;
      default: fail(CG_POLICY_REJECTED, "NPDS protobuf: unsupported wire type");
    }
  }
  void need(size_t n) {
    if ((size_t)(e - p) < n) fail(CG_POLICY_REJECTED, "NPDS protobuf: truncated field");
  }
};

Reader sub(const std::string& s) { return Reader{(const uint8_t*)s.data(), (const uint8_t*)s.data() + s.size()}; }

// varint scalars of a repeated field, packed (wire type 2) or not (0)
void repeated_varints(Reader& r, uint32_t wt, std::vector<uint64_t>* out) {
  if (wt == 0) {
    out->push_back(r.varint());
  } else if (wt == 2) {
    const std::string b = r.bytes();
    Reader q = sub(b);
    while (!q.done()) out->push_back(q.varint());
  } else {
    fail(CG_POLICY_REJECTED, "NPDS protobuf: bad wire type for a varint field");
  }
}

uint64_t scalar(Reader& r, uint32_t wt) {
  if (wt != 0) fail(CG_POLICY_REJECTED, "NPDS protobuf: bad wire type for a varint field");
  return r.varint();
}

// a proto3 `string` field (UTF-8 checked on the Envoy path)
std::string str(Reader& r, uint32_t wt) {
  if (wt != 2) fail(CG_POLICY_REJECTED, "NPDS protobuf: bad wire type for a string field");
  std::string s = r.bytes();
  if (t_strict_utf8 && !utf8_ok(s)) fail(CG_POLICY_REJECTED, "NPDS protobuf: string field is not valid UTF-8");
  return s;
}

// an embedded message or `bytes` field (no UTF-8 rule)
std::string msg_bytes(Reader& r, uint32_t wt) {
  if (wt != 2) fail(CG_POLICY_REJECTED, "NPDS protobuf: bad wire type for an embedded message");
  return r.bytes();
}

std::string jstr(const std::string& s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
    } else {
      o += (char)c;
    }
  }
  return o + "\"";
}

// HeaderMatcher → the engine's matcher JSON.  The oneof keeps its last member
// (an embedded member's occurrences merge); range_match is envoy.type.Int64Range
// {int64 start = 1; int64 end = 2}.
std::string header_matcher(const std::string& msg) {
  Reader r = sub(msg);
  std::string name, spec, value, bool_msg, range_msg;
  bool has_value = false, invert = false;
  uint32_t spec_field = 0;
  uint32_t f, wt;
  while (r.next(&f, &wt)) {
    switch (f) {
      case 1: name = str(r, wt); break;
      case 2: value = str(r, wt); has_value = true; break;
      case 3: bool_msg += msg_bytes(r, wt); break;  // google.protobuf.BoolValue {bool value = 1}
      case 4: spec = "\"exact_match\":" + jstr(str(r, wt)); spec_field = 4; break;
      case 5: spec = "\"regex_match\":" + jstr(str(r, wt)); spec_field = 5; break;
      case 6:
        if (spec_field != 6) range_msg.clear();
        range_msg += msg_bytes(r, wt);
        spec_field = 6;
        break;
      case 7: spec = std::string("\"present_match\":") + (scalar(r, wt) ? "true" : "false"); spec_field = 7; break;
      case 8: invert = scalar(r, wt) != 0; break;
      case 9: spec = "\"prefix_match\":" + jstr(str(r, wt)); spec_field = 9; break;
      case 10: spec = "\"suffix_match\":" + jstr(str(r, wt)); spec_field = 10; break;
      default: r.skip(wt);
    }
  }
  bool regex = false;
  {
    Reader q = sub(bool_msg);
    uint32_t g, w;
    while (q.next(&g, &w)) {
      if (g == 1) regex = scalar(q, w) != 0;
      else q.skip(w);
    }
  }
  if (spec_field == 6) {
    int64_t start = 0, end = 0;
    Reader q = sub(range_msg);
    uint32_t g, w;
    while (q.next(&g, &w)) {
      if (g == 1) start = (int64_t)scalar(q, w);
      else if (g == 2) end = (int64_t)scalar(q, w);
      else q.skip(w);
    }
    spec = "\"range_match\":{\"start\":" + std::to_string(start) + ",\"end\":" + std::to_string(end) + "}";
  }
  std::string o = "{\"name\":" + jstr(name);
  if (!spec.empty()) o += "," + spec;
  if (has_value) o += ",\"value\":" + jstr(value) + ",\"regex\":" + (regex ? "true" : "false");
  if (invert) o += ",\"invert_match\":true";
  return o + "}";
}

bool kafka_name_ok(const std::string& s) {  // ^[a-zA-Z0-9._-]*$
  for (unsigned char c : s)
    if (!(isalnum(c) || c == '.' || c == '_' || c == '-')) return false;
  return true;
}

std::string kafka_rule(const std::string& msg) {
  Reader r = sub(msg);
  int64_t api_key = 0, api_version = 0;
  std::string topic, client;
  uint32_t f, wt;
  while (r.next(&f, &wt)) {
    switch (f) {
      case 1: api_key = (int32_t)scalar(r, wt); break;
      case 2: api_version = (int32_t)scalar(r, wt); break;
      case 3: topic = str(r, wt); break;
      case 4: client = str(r, wt); break;
      default: r.skip(wt);
    }
  }
  if (topic.size() > 255 || !kafka_name_ok(topic) || !kafka_name_ok(client))
    fail(CG_POLICY_REJECTED, "KafkaNetworkPolicyRule: invalid topic or client_id");
  return "{\"api_key\":" + std::to_string(api_key) + ",\"api_version\":" + std::to_string(api_version) +
         ",\"topic\":" + jstr(topic) + ",\"client_id\":" + jstr(client) + "}";
}

std::string join(const std::vector<std::string>& xs) {
  std::string o;
  for (size_t i = 0; i < xs.size(); ++i) o += (i ? "," : "") + xs[i];
  return o;
}

// HttpNetworkPolicyRules {repeated HttpNetworkPolicyRule http_rules = 1}
std::string http_rules_json(const std::string& msg) {
  Reader q = sub(msg);
  std::vector<std::string> rules;
  uint32_t g, w;
  while (q.next(&g, &w)) {
    if (g != 1) {
      q.skip(w);
      continue;
    }
    const std::string h_msg = msg_bytes(q, w);  // outlives its reader
    Reader h = sub(h_msg);
    std::vector<std::string> hs;
    uint32_t k, x;
    while (h.next(&k, &x)) {
      if (k == 1) hs.push_back(header_matcher(msg_bytes(h, x)));
      else h.skip(x);
    }
    rules.push_back("{\"headers\":[" + join(hs) + "]}");
  }
  if (rules.empty()) fail(CG_POLICY_REJECTED, "HttpNetworkPolicyRules: value must contain at least 1 item");
  return "\"http_rules\":{\"http_rules\":[" + join(rules) + "]}";
}

// KafkaNetworkPolicyRules {repeated KafkaNetworkPolicyRule kafka_rules = 1}
std::string kafka_rules_json(const std::string& msg) {
  Reader q = sub(msg);
  std::vector<std::string> rules;
  uint32_t g, w;
  while (q.next(&g, &w)) {
    if (g == 1) rules.push_back(kafka_rule(msg_bytes(q, w)));
    else q.skip(w);
  }
  if (rules.empty()) fail(CG_POLICY_REJECTED, "KafkaNetworkPolicyRules: value must contain at least 1 item");
  return "\"kafka_rules\":{\"kafka_rules\":[" + join(rules) + "]}";
}

// L7NetworkPolicyRules {repeated L7NetworkPolicyRule l7_rules = 1}, each a
// map<string, string> rule = 1
std::string l7_rules_json(const std::string& msg) {
  Reader q = sub(msg);
  std::vector<std::string> rules;
  uint32_t g, w;
  while (q.next(&g, &w)) {
    if (g != 1) {
      q.skip(w);
      continue;
    }
    const std::string m_msg = msg_bytes(q, w);  // outlives its reader
    Reader m = sub(m_msg);
    std::map<std::string, std::string> kv;
    uint32_t k, x;
    while (m.next(&k, &x)) {
      if (k != 1) {
        m.skip(x);
        continue;
      }
      const std::string en_msg = msg_bytes(m, x);  // outlives its reader
      Reader en = sub(en_msg);
      std::string key, val;
      uint32_t a, b;
      while (en.next(&a, &b)) {
        if (a == 1) key = str(en, b);
        else if (a == 2) val = str(en, b);
        else en.skip(b);
      }
      kv[key] = val;
    }
    std::vector<std::string> es;
    for (const auto& [k2, v2] : kv) es.push_back(jstr(k2) + ":" + jstr(v2));
    rules.push_back("{\"rule\":{" + join(es) + "}}");
  }
  if (rules.empty()) fail(CG_POLICY_REJECTED, "L7NetworkPolicyRules: value must contain at least 1 item");
  return "\"l7_rules\":{\"l7_rules\":[" + join(rules) + "]}";
}

std::string port_rule(const std::string& msg) {
  Reader r = sub(msg);
  std::vector<uint64_t> remotes;
  std::string l7_proto;
  // the l7 oneof: its last member; occurrences of the same member merge
  uint32_t l7_field = 0;
  std::string l7_msg;
  uint32_t f, wt;
  while (r.next(&f, &wt)) {
    switch (f) {
      case 1: repeated_varints(r, wt, &remotes); break;
      case 2: l7_proto = str(r, wt); break;
      case 100:
      case 101:
      case 102:
        if (l7_field != f) l7_msg.clear();
        l7_msg += msg_bytes(r, wt);
        l7_field = f;
        break;
      default: r.skip(wt);
    }
  }
  std::string l7;
  if (l7_field == 100) l7 = http_rules_json(l7_msg);
  else if (l7_field == 101) l7 = kafka_rules_json(l7_msg);
  else if (l7_field == 102) l7 = l7_rules_json(l7_msg);
  std::set<uint64_t> uniq(remotes.begin(), remotes.end());
  if (uniq.size() != remotes.size())
    fail(CG_POLICY_REJECTED, "PortNetworkPolicyRule.RemotePolicies: repeated value must contain unique items");
  std::vector<std::string> ids;
  for (uint64_t id : remotes) ids.push_back(std::to_string(id));
  std::string o = "{\"remote_policies\":[" + join(ids) + "]";
  if (!l7_proto.empty()) o += ",\"l7_proto\":" + jstr(l7_proto);
  if (!l7.empty()) o += "," + l7;
  return o + "}";
}

std::string port_policy(const std::string& msg) {
  Reader r = sub(msg);
  uint64_t port = 0, proto = 0;
  std::vector<std::string> rules;
  uint32_t f, wt;
  while (r.next(&f, &wt)) {
    switch (f) {
      case 1: port = (uint32_t)scalar(r, wt); break;
      case 2: proto = (uint32_t)scalar(r, wt); break;
      case 3: rules.push_back(port_rule(msg_bytes(r, wt))); break;
      default: r.skip(wt);
    }
  }
  if (port > 65535) fail(CG_POLICY_REJECTED, "PortNetworkPolicy.Port: value must be less than or equal to 65535");
  return "{\"port\":" + std::to_string(port) + ",\"protocol\":" + std::to_string(proto) + ",\"rules\":[" +
         join(rules) + "]}";
}

std::string network_policy(const std::string& msg) {
  Reader r = sub(msg);
  std::string name;
  uint64_t policy = 0;
  std::vector<std::string> in, eg;
  uint32_t f, wt;
  while (r.next(&f, &wt)) {
    switch (f) {
      case 1: name = str(r, wt); break;
      case 2: policy = scalar(r, wt); break;
      case 3: in.push_back(port_policy(msg_bytes(r, wt))); break;
      case 4: eg.push_back(port_policy(msg_bytes(r, wt))); break;
      default: r.skip(wt);
    }
  }
  return "{\"name\":" + jstr(name) + ",\"policy\":" + std::to_string(policy) + ",\"ingress_per_port_policies\":[" +
         join(in) + "],\"egress_per_port_policies\":[" + join(eg) + "]}";
}

}  // namespace

std::string npds_pb_to_json(const uint8_t* p, size_t n, bool strict_utf8) {
  struct Mode {
    bool prev;
    explicit Mode(bool m) : prev(t_strict_utf8) { t_strict_utf8 = m; }
    ~Mode() { t_strict_utf8 = prev; }
  } mode(strict_utf8);
  Reader r{p, p + n};
  std::vector<std::string> pols;
  uint32_t f, wt;
  static const std::string kType = "type.googleapis.com/cilium.NetworkPolicy";
  while (r.next(&f, &wt)) {
    if (f != 2) {  // DiscoveryResponse.resources (repeated google.protobuf.Any)
      r.skip(wt);
      continue;
    }
    const std::string a_msg = msg_bytes(r, wt);  // outlives its reader
    Reader a = sub(a_msg);
    std::string type, value;
    uint32_t g, w;
    while (a.next(&g, &w)) {
      if (g == 1) type = str(a, w);
      else if (g == 2) value = msg_bytes(a, w);
      else a.skip(w);
    }
    if (type != kType) fail(CG_POLICY_REJECTED, "NPDS resource is not a cilium.NetworkPolicy: " + type);
    pols.push_back(network_policy(value));
  }
  return "[" + join(pols) + "]";
}

}  // namespace cg
