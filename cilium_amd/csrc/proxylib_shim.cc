// proxylib_shim.cc — the proxylib C ABI (include/cilium_proxylib.h) over the
// verdict engine, plus cg_proxylib_policy_update (include/cilium_gpu.h).
//
//   OpenModule / CloseModule     proxylib/proxylib.go:118-155
//   OnNewConnection / Close      proxylib/proxylib.go:56-111, connection.go:60-100
//   OnData                       connection.go:118-174 (op loop) +
//                                r2d2/r2d2parser.go:148-199 (line framing)
//   policy translation           proxylib/proxylib/policymap.go:118-206 with the
//                                r2d2 (r2d2parser.go:91-123), cassandra
//                                (cassandraparser.go:97-131) and memcache
//                                (memcached/parser.go:104-147) rule parsers
//   memcache OnData              proxylib_memcache.cc (text and binary)
//   cassandra OnData             proxylib_cassandra.cc (frames, queries, prepared ids)
//
// The policy verdicts of every request frame found in one OnData call are
// evaluated as one batch by http_kernel (no CPU evaluation path).
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/cilium_gpu.h"
#include "../../include/cilium_proxylib.h"
#include "common.h"
#include "http.h"
#include "json.h"
#include "proxylib_cassandra.h"
#include "proxylib_memcache.h"

using namespace cg;

namespace {

// One OnData call's request records waiting for their verdicts.
struct VerdictReq {
  const std::vector<std::string>* recs;
  // the connection's policy by name: the flusher resolves it under inst.mu,
  // against the snapshot the batch is packed and decided with (the Go
  // proxylib looks the policy up at match time, policymap.go:208-236)
  const std::string* policy;
  bool ingress;
  uint16_t port;
  uint32_t remote;  // Matches passes SrcId (connection.go:176-179)
  std::vector<uint8_t>* out;
  bool done = false, ok = false;
};

struct Instance {
  uint64_t engine = 0;
  std::string key;
  std::mutex mu;  // serializes verdict batches and policy updates on the engine
  // Cross-connection batching (flat combining): concurrent OnData calls of
  // different connections queue their records; whichever finds no batch in
  // flight takes everything queued and decides it as one GPU batch, while
  // the calls arriving meanwhile queue for the next one.  A lone call is
  // decided at once (no timer); under concurrency one launch and one sync
  // serve many connections.  Each connection's own OnData stays
  // single-threaded (libcilium.h:79-80).
  std::mutex qmu;
  std::condition_variable qcv;
  std::vector<VerdictReq*> queue;
  bool flushing = false;
  uint64_t batches = 0, calls = 0;  // decided batches / calls (cg_proxylib_stats)
  // batching window (cg_proxylib_set_batching): a flusher waits until
  // min_calls calls are queued or max_wait_us has passed since it took over
  uint32_t min_calls = 1, max_wait_us = 0;
};

struct Conn {
  std::shared_ptr<Instance> inst;
  std::string parser, policy;
  McState mc;     // memcache parser state
  CassState cs;   // cassandra parser state
  bool ingress = false;
  uint32_t src_id = 0, dst_id = 0, port = 0;
  GoSlice* orig_buf = nullptr;
  GoSlice* reply_buf = nullptr;
};

std::mutex g_mu;
std::map<uint64_t, std::shared_ptr<Instance>> g_instances;
std::map<std::string, uint64_t> g_instance_by_key;
std::map<uint64_t, std::shared_ptr<Conn>> g_conns;
uint64_t g_next_instance = 1;

std::string gostr(GoString s) { return s.p && s.n > 0 ? std::string(s.p, (size_t)s.n) : std::string(); }

std::shared_ptr<Instance> find_instance(uint64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_instances.find(id);
  return it == g_instances.end() ? nullptr : it->second;
}

// ------------------------------------------------------------ translation
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

std::string m_exact(const char* name, const std::string& v) {
  return std::string("{\"name\":\"") + name + "\",\"exact_match\":" + jstr(v) + "}";
}
std::string m_search(const char* name, const std::string& v) {
  return std::string("{\"name\":\"") + name + "\",\"regex_search\":" + jstr(v) + "}";
}
std::string join(const std::vector<std::string>& xs) {
  std::string o;
  for (size_t i = 0; i < xs.size(); ++i) o += (i ? "," : "") + xs[i];
  return o;
}

// each returned entry: one engine rule (an AND of matchers, JSON array body)
std::vector<std::string> r2d2_rules(const Json* l7) {
  std::vector<std::string> out;
  for (const Json& e : l7->arr) {
    std::string cmd, file;
    bool has_file = false;
    if (const Json* r = e.get("rule"))
      for (const auto& [k, v] : r->obj) {
        if (k == "cmd") cmd = v.as_str("cmd");
        else if (k == "file") {
          file = v.as_str("file");
          has_file = !file.empty();
        } else fail(CG_POLICY_REJECTED, "Unsupported key: " + k);
      }
    if (!cmd.empty() && cmd != "READ" && cmd != "WRITE" && cmd != "HALT" && cmd != "RESET")
      fail(CG_POLICY_REJECTED, "Unable to parse L7 r2d2 rule with invalid cmd: '" + cmd + "'");
    if (has_file && !(cmd.empty() || cmd == "READ" || cmd == "WRITE"))
      fail(CG_POLICY_REJECTED, "Unable to parse L7 r2d2 rule, cmd '" + cmd + "' is not compatible with 'file'");
    std::vector<std::string> ms;
    if (!cmd.empty()) ms.push_back(m_exact("cmd", cmd));
    if (has_file) ms.push_back(m_search("file", file));
    out.push_back(join(ms));
  }
  return out;
}

int cassandra_action_kind(const std::string& a) {
  static const std::set<std::string> table = {"select", "delete", "insert", "update", "create-table",
                                              "drop-table", "alter-table", "truncate-table", "use",
                                              "create-keyspace", "alter-keyspace", "drop-keyspace"};
  static const std::set<std::string> notable = {
      "drop-index", "create-index", "create-materialized-view", "drop-materialized-view", "create-role",
      "alter-role", "drop-role", "grant-role", "revoke-role", "list-roles", "grant-permission",
      "revoke-permission", "list-permissions", "create-user", "alter-user", "drop-user", "list-users",
      "create-function", "drop-function", "create-aggregate", "drop-aggregate", "create-type", "alter-type",
      "drop-type", "create-trigger", "drop-trigger"};
  return table.count(a) ? 1 : notable.count(a) ? 2 : 0;
}

std::vector<std::string> cassandra_rules(const Json* l7) {
  std::vector<std::string> out;
  for (const Json& e : l7->arr) {
    std::string action, table;
    bool has_table = false;
    if (const Json* r = e.get("rule"))
      for (const auto& [k, v] : r->obj) {
        if (k == "query_action") action = v.as_str("query_action");
        else if (k == "query_table") {
          table = v.as_str("query_table");
          has_table = !table.empty();
        } else fail(CG_POLICY_REJECTED, "Unsupported key: " + k);
      }
    if (!action.empty()) {
      const int kind = cassandra_action_kind(action);
      if (kind == 0) fail(CG_POLICY_REJECTED, "Unable to parse L7 cassandra rule with invalid query_action");
      if (kind == 2 && has_table) fail(CG_POLICY_REJECTED, "query_action is not compatible with a query_table match");
    }
    out.push_back(m_exact("cshape", "S"));
    std::vector<std::string> lng{m_exact("cshape", "L")};
    if (!action.empty()) lng.push_back(m_exact("action", action));
    if (!has_table) {
      out.push_back(join(lng));
    } else {
      auto a = lng, b = lng;
      a.push_back(m_exact("table", ""));
      b.push_back(m_search("table", table));
      out.push_back(join(a));
      out.push_back(join(b));
    }
  }
  return out;
}

// MemcacheOpCodeMap (memcached/parser.go:210-474): a rule command → the
// text commands and binary opcodes it allows
struct McCommands {
  std::vector<std::string> text;
  std::vector<uint8_t> binary;
};
const std::map<std::string, McCommands>& memcache_opcode_map() {
  static const std::map<std::string, McCommands> m = [] {
    std::map<std::string, McCommands> x;
    x["add"] = {{"add"}, {2, 18}};
    x["set"] = {{"set"}, {1, 17}};
    x["replace"] = {{"replace"}, {3, 19}};
    x["append"] = {{"append"}, {14, 25}};
    x["prepend"] = {{"prepend"}, {15, 26}};
    x["cas"] = {{"cas"}, {}};
    x["incr"] = {{"incr"}, {5, 21}};
    x["decr"] = {{"decr"}, {6, 22}};
    x["storage"] = {{"add", "set", "replace", "append", "prepend", "cas", "incr", "decr"},
                    {1, 2, 3, 5, 6, 17, 18, 19, 21, 22, 25, 26}};
    x["get"] = {{"get", "gets"}, {0, 9, 12, 13}};
    x["delete"] = {{"delete"}, {4, 20}};
    x["touch"] = {{"touch"}, {28}};
    x["gat"] = {{"gat", "gats"}, {29, 30}};
    x["writeGroup"] = {{"add", "set", "replace", "append", "prepend", "cas", "incr", "decr", "delete", "touch"},
                       {1, 2, 3, 4, 5, 6, 17, 18, 19, 20, 21, 22, 25, 26, 28}};
    x["slabs"] = {{"slabs"}, {}};
    x["lru"] = {{"lru"}, {}};
    x["lru_crawler"] = {{"lru_crawler"}, {}};
    x["watch"] = {{"watch"}, {}};
    x["stats"] = {{"stats"}, {16}};
    x["flush_all"] = {{"flush_all"}, {8, 24}};
    x["cache_memlimit"] = {{"cache_memlimit"}, {}};
    x["version"] = {{"version"}, {11}};
    x["misbehave"] = {{"misbehave"}, {}};
    x["quit"] = {{"quit"}, {7, 23}};
    x["noop"] = {{}, {10}};
    x["verbosity"] = {{}, {27}};
    const char* bin_only[] = {"sasl-list-mechs", "sasl-auth", "sasl-step", "rget", "rset", "rsetq", "rappend",
                              "rappendq", "rprepend", "rprependq", "rdelete", "rdeleteq", "rincr", "rincrq", "rdecr",
                              "rdecrq", "set-vbucket", "get-vbucket", "del-vbucket", "tap-connect", "tap-mutation",
                              "tap-delete", "tap-flush", "tap-opaque", "tap-vbucket-set", "tap-checkpoint-start",
                              "tap-checkpoint-end"};
    const uint8_t bin_code[] = {32, 33, 34, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63, 64, 65,
                                66, 67, 68, 69, 70, 71};
    for (size_t i = 0; i < sizeof(bin_code); ++i) x[bin_only[i]] = {{}, {bin_code[i]}};
    return x;
  }();
  return m;
}

// The request fields a memcache frame is packed as: mccmd = "t" + command
// or "b" + two hex digits of the opcode, mckeys = each key then the separator pair {0x03,
// 0x14} (values escaped, proxylib_shim OnData).
std::string m_list(const char* kind, const std::string& v) {
  return std::string("{\"name\":\"mckeys\",\"") + kind + "\":" + jstr(v) + "}";
}

// L7RuleParser (memcached/parser.go:104-147) → engine rules: one per allowed
// command token (an exact mccmd) AND the key matcher.  A rule with no
// command and no key matches every request; an unknown command with no key
// too (commandFound false, br.empty), with a key it is a parse error.
std::vector<std::string> memcache_rules(const Json* l7) {
  std::vector<std::string> out;
  for (const Json& e : l7->arr) {
    std::string key_exact, key_prefix, key_regex;
    bool found = false, has_regex = false;
    const McCommands* cmds = nullptr;
    if (const Json* r = e.get("rule"))
      for (const auto& [k, v] : r->obj) {
        if (k == "command") {
          auto it = memcache_opcode_map().find(v.as_str("command"));
          found = it != memcache_opcode_map().end();
          cmds = found ? &it->second : nullptr;
        } else if (k == "keyExact") {
          key_exact = v.as_str("keyExact");
        } else if (k == "keyPrefix") {
          key_prefix = v.as_str("keyPrefix");
        } else if (k == "keyRegex") {
          key_regex = v.as_str("keyRegex");
          has_regex = true;  // regexp.MustCompile(""): a regex that matches every key
        } else {
          fail(CG_POLICY_REJECTED, "Unsupported key: " + k);
        }
      }
    if (!found) {
      if (!key_exact.empty() || !key_prefix.empty() || has_regex)
        fail(CG_POLICY_REJECTED, "command not specified but key was provided");
      out.push_back("");  // empty rule: matches everything
      continue;
    }
    // Matches: keyExact if non-empty, else keyPrefix, else the regex
    std::string km;
    if (!key_exact.empty()) km = m_list("list_exact", key_exact);
    else if (!key_prefix.empty()) km = m_list("list_prefix", key_prefix);
    else if (has_regex) km = m_list("list_search", key_regex);
    for (const auto& t : cmds->text) out.push_back(join(km.empty() ? std::vector<std::string>{m_exact("mccmd", "t" + t)}
                                                                   : std::vector<std::string>{m_exact("mccmd", "t" + t), km}));
    for (uint8_t b : cmds->binary) {
      static const char hex[] = "0123456789abcdef";
      const std::string tok{'b', hex[b >> 4], hex[b & 15]};
      out.push_back(join(km.empty() ? std::vector<std::string>{m_exact("mccmd", tok)}
                                    : std::vector<std::string>{m_exact("mccmd", tok), km}));
    }
  }
  return out;
}

bool known_parser(const std::string& p) { return p == "r2d2" || p == "cassandra" || p == "memcache"; }

std::string translate(const char* json, size_t len) {
  Json root = JsonParser(json, len).parse();
  if (root.type != Json::ARR) fail(CG_POLICY_REJECTED, "expected a list of NetworkPolicy");
  std::string out = "[";
  bool firstp = true;
  for (const Json& p : root.arr) {
    const Json* nm = p.get("name");
    if (!nm) fail(CG_POLICY_REJECTED, "NetworkPolicy without name");
    out += std::string(firstp ? "" : ",") + "{\"name\":" + jstr(nm->as_str("name")) + ",\"proxylib\":true";
    firstp = false;
    for (const char* key : {"ingress_per_port_policies", "egress_per_port_policies"}) {
      out += std::string(",\"") + key + "\":[";
      std::set<uint64_t> seen;
      bool firstport = true;
      if (const Json* ports = p.get(key)) {
        if (ports->type != Json::ARR) fail(CG_POLICY_REJECTED, "per_port_policies must be a list");
        for (const Json& pp : ports->arr) {
          std::string proto = "TCP";
          if (const Json* j = pp.get("protocol"))
            proto = j->type == Json::STR ? j->s : (j->as_u64("protocol") == 0 ? "TCP" : j->as_u64("protocol") == 1 ? "UDP" : "?");
          if (proto == "UDP") continue;
          const uint64_t port = pp.get("port") ? pp.get("port")->as_u64("port") : 0;
          if (!seen.insert(port).second) fail(CG_POLICY_REJECTED, "Duplicate port number");
          if (proto != "TCP") fail(CG_POLICY_REJECTED, "Invalid transport protocol");
          std::string rules;
          bool ok = true, firstr = true;
          std::string first_type;
          if (const Json* rs = pp.get("rules")) {
            for (const Json& r : rs->arr) {
              std::string l7p = r.get("l7_proto") ? r.get("l7_proto")->as_str("l7_proto") : "";
              if (!l7p.empty() && !known_parser(l7p)) {
                ok = false;  // newPortNetworkPolicyRule !ok: the port is not installed
                break;
              }
              if (!l7p.empty()) {
                if (first_type.empty()) first_type = l7p;
                else if (l7p != first_type) fail(CG_POLICY_REJECTED, "Mismatching L7 types on the same port");
              }
              std::vector<std::string> ms;
              const Json* l7 = nullptr;
              if (const Json* lr = r.get("l7_rules")) l7 = lr->get("l7_rules");
              if (!l7p.empty() && l7 && l7->type == Json::ARR)
                ms = l7p == "r2d2" ? r2d2_rules(l7) : l7p == "memcache" ? memcache_rules(l7) : cassandra_rules(l7);
              std::string rr = "{";
              bool any = false;
              if (const Json* rp = r.get("remote_policies")) {
                std::vector<std::string> ids;
                for (const Json& id : rp->arr) ids.push_back(std::to_string(id.as_u64("remote_policies")));
                if (!ids.empty()) {
                  rr += "\"remote_policies\":[" + join(ids) + "]";
                  any = true;
                }
              }
              if (!ms.empty()) {
                std::vector<std::string> hr;
                for (auto& m : ms) hr.push_back("{\"headers\":[" + m + "]}");
                rr += std::string(any ? "," : "") + "\"http_rules\":{\"http_rules\":[" + join(hr) + "]}";
              }
              rules += std::string(firstr ? "" : ",") + rr + "}";
              firstr = false;
            }
          }
          if (!ok) continue;
          out += std::string(firstport ? "" : ",") + "{\"port\":" + std::to_string(port) +
                 ",\"protocol\":\"TCP\",\"rules\":[" + rules + "]}";
          firstport = false;
        }
      }
      out += "]";
    }
    out += "}";
  }
  return out + "]";
}

// --------------------------------------------------------------- framing
struct Frame {
  size_t len;  // bytes including "\r\n"
  bool request;
  std::string cmd, file;
};

size_t inject(GoSlice* buf, const char* data, size_t n) {  // connection.go:190-209
  if (!buf || !buf->data) return 0;
  const size_t off = (size_t)buf->len, room = (size_t)(buf->cap - buf->len);
  const size_t k = n < room ? n : room;
  memcpy((char*)buf->data + off, data, k);
  buf->len += (int64_t)k;
  return k;
}

// values escaped for the proxylib snapshot (bytes 0x00-0x03 → 0x03, 0x10 +
// b): a NUL or control byte inside a field stays part of the string the
// rules see, as in r2d2parser.go:157-183
std::string esc(const std::string& v) {
  std::string o;
  o.reserve(v.size());
  for (unsigned char ch : v) {
    if (ch <= 0x03) {
      o += (char)0x03;
      o += (char)(0x10 + ch);
    } else {
      o += (char)ch;
    }
  }
  return o;
}

std::string field(const char* name, const std::string& escaped) {
  return std::string(name) + '\0' + escaped + '\0';
}

// PolicyMatches (connection.go:176-179) for the request records of the
// queued OnData calls, as one host-staged GPU batch.  Caller holds inst.mu
// (decide's flusher).
// Returns false on an engine error.
bool gpu_verdicts(Instance& inst, const std::vector<VerdictReq*>& reqs) {
  size_t n = 0;
  // policy names → indices in the current snapshot; an unknown name (or no
  // policy installed) leaves its calls all-DROP (PolicyMatches false)
  std::map<std::string, uint32_t> idx;
  std::vector<uint32_t> rpol(reqs.size());
  for (size_t j = 0; j < reqs.size(); ++j) {
    const VerdictReq* r = reqs[j];
    r->out->assign(r->recs->size(), 0);
    auto it = idx.find(*r->policy);
    if (it == idx.end()) {
      uint32_t p = 0xFFFFFFFFu;
      if (cg_http_policy_index(inst.engine, r->policy->c_str(), &p) != CG_OK) p = 0xFFFFFFFFu;
      it = idx.emplace(*r->policy, p).first;
    }
    rpol[j] = it->second;
    if (rpol[j] != 0xFFFFFFFFu) n += r->recs->size();
  }
  if (n == 0) return true;
  std::vector<uint32_t> pol, remote;
  std::vector<uint8_t> ing;
  std::vector<uint16_t> port;
  pol.reserve(n), remote.reserve(n), ing.reserve(n), port.reserve(n);
  std::string blob;
  std::vector<uint64_t> off{0};
  for (size_t j = 0; j < reqs.size(); ++j) {
    const VerdictReq* r = reqs[j];
    if (rpol[j] == 0xFFFFFFFFu) continue;
    for (const std::string& rec : *r->recs) {
      pol.push_back(rpol[j]);
      ing.push_back(r->ingress ? 1 : 0);
      port.push_back(r->port);
      remote.push_back(r->remote);
      blob += rec;
      off.push_back(blob.size());
    }
  }
  if (blob.empty()) blob.push_back('\0');
  size_t nslots = 0, used = 0;
  int rc = cg_http_pack(inst.engine, n, pol.data(), ing.data(), port.data(), remote.data(),
                        (const uint8_t*)blob.data(), off.data(), nullptr, 0, nullptr, &nslots, nullptr, 0, &used);
  if (rc != CG_OK) return false;
  std::vector<uint8_t> batch(cg_http_batch_bytes(inst.engine, n));
  std::vector<uint32_t> order(cg_http_batch_slots(inst.engine, n) + 1);
  std::vector<uint8_t> arena(used > 16 ? used : 16), allow(n);
  rc = cg_http_pack(inst.engine, n, pol.data(), ing.data(), port.data(), remote.data(),
                    (const uint8_t*)blob.data(), off.data(), batch.data(), batch.size(), order.data(), &nslots,
                    arena.data(), arena.size(), &used);
  if (rc != CG_OK) return false;
  rc = cg_http_verdicts_host(inst.engine, batch.data(), nslots, order.data(), n, arena.data(), arena.size(),
                             allow.data());
  if (rc != CG_OK) return false;
  size_t k = 0;
  for (size_t j = 0; j < reqs.size(); ++j) {
    if (rpol[j] == 0xFFFFFFFFu) continue;
    VerdictReq* r = reqs[j];
    for (size_t i = 0; i < r->recs->size(); ++i) (*r->out)[i] = allow[k++];
  }
  return true;
}

// Verdicts for one OnData call's records (see Instance: the calls queued
// meanwhile share the GPU batch).
bool decide(Conn& c, const std::vector<std::string>& recs, std::vector<uint8_t>* out) {
  out->assign(recs.size(), 0);
  if (recs.empty()) return true;
  Instance& inst = *c.inst;
  VerdictReq me{&recs, &c.policy, c.ingress, (uint16_t)(c.port > 0xFFFF ? 0 : c.port), c.src_id, out};
  std::unique_lock<std::mutex> lk(inst.qmu);
  inst.queue.push_back(&me);
  if (inst.flushing || inst.min_calls > 1) inst.qcv.notify_all();  // a flusher may be waiting for company
  while (!me.done) {
    if (inst.flushing) {
      inst.qcv.wait(lk);
      continue;
    }
    inst.flushing = true;
    if (inst.min_calls > 1 && inst.max_wait_us > 0) {  // batching window
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(inst.max_wait_us);
      inst.qcv.wait_until(lk, until, [&] { return inst.queue.size() >= inst.min_calls; });
    }
    std::vector<VerdictReq*> batch;
    batch.swap(inst.queue);
    lk.unlock();
    bool ok = false;
    try {  // the waiters must be released whatever happens here
      std::lock_guard<std::mutex> g(inst.mu);
      ok = gpu_verdicts(inst, batch);
    } catch (...) {
      ok = false;
    }
    lk.lock();
    for (VerdictReq* r : batch) {
      r->ok = ok;
      r->done = true;
    }
    inst.batches += 1;
    inst.calls += batch.size();
    inst.flushing = false;
    inst.qcv.notify_all();
  }
  return me.ok;
}

// A memcache request as the fields its rules are compiled over (see
// memcache_rules): mccmd "t" + command or "b" + two hex digits of the
// opcode, mckeys every key then the separator pair {0x03, 0x14}.
std::string memcache_record(const McMeta& m) {
  static const char hex[] = "0123456789abcdef";
  std::string cmd = m.binary() ? std::string{'b', hex[m.opcode >> 4], hex[m.opcode & 15]} : "t" + m.command;
  std::string keys;
  for (const std::string& k : m.keys) keys += esc(k) + "\x03\x14";
  return field("mccmd", esc(cmd)) + field("mckeys", keys);
}

// memcache OnData: a dry run on copies of the parser state collects the
// request frames this call will decide (the frame sequence does not depend
// on the verdicts: a denial is a DROP of the same length), one GPU batch
// decides them, and the real run consumes the verdicts in order.
FilterResult memcache_data(Conn& c, bool reply, bool end_stream, const GoSlice* data, GoSlice* ops) {
  std::vector<uint8_t> allow;
  if (!reply) {
    McState dry = c.mc;
    std::vector<FilterOp> scratch((size_t)(ops->cap > 0 ? ops->cap : 1));
    GoSlice sops{scratch.data(), ops->len, ops->cap};
    std::vector<std::string> recs;
    memcache_on_data(dry, false, end_stream, data, &sops, nullptr, [&](const McMeta& m) {
      recs.push_back(memcache_record(m));
      return true;
    });
    if (!decide(c, recs, &allow)) return FILTER_UNKNOWN_ERROR;
  }
  size_t next = 0;
  return memcache_on_data(c.mc, reply, end_stream, data, ops, c.reply_buf, [&](const McMeta&) {
    return next < allow.size() && allow[next++] != 0;
  });
}

// A cassandra path as the fields its rules are compiled over (see
// cassandra_rules): cshape, then action and table for query-like paths.
std::string cassandra_record(const std::string& path) {
  const CassFields f = cassandra_path_fields(path);
  std::string r = field("cshape", std::string(1, f.shape));
  if (f.shape == 'L') r += field("action", esc(f.action)) + field("table", esc(f.table));
  return r;
}

// cassandra OnData: as memcache_data — the paths a dry run on a copy of the
// parser state collects do not depend on the verdicts (a denial is a DROP of
// the same frame), one GPU batch decides them, the real run consumes them.
FilterResult cassandra_data(Conn& c, bool reply, bool end_stream, const GoSlice* data, GoSlice* ops) {
  std::vector<uint8_t> allow;
  if (!reply) {
    CassState dry = c.cs;
    std::vector<FilterOp> scratch((size_t)(ops->cap > 0 ? ops->cap : 1));
    GoSlice sops{scratch.data(), ops->len, ops->cap};
    std::vector<std::string> recs;
    cassandra_on_data(dry, false, end_stream, data, &sops, nullptr, [&](const std::string& path) {
      recs.push_back(cassandra_record(path));
      return true;
    });
    if (!decide(c, recs, &allow)) return FILTER_UNKNOWN_ERROR;
  }
  size_t next = 0;
  return cassandra_on_data(c.cs, reply, end_stream, data, ops, c.reply_buf, [&](const std::string&) {
    return next < allow.size() && allow[next++] != 0;
  });
}

}  // namespace

extern "C" {

int cg_proxylib_policy_update(uint64_t instance, const char* json, size_t len) {
  auto inst = find_instance(instance);
  if (!inst) return CG_INVALID_INSTANCE;
  std::string eng;
  try {
    eng = translate(json, len);
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (...) {
    set_error("proxylib policy translation failed");
    return CG_UNKNOWN_ERROR;
  }
  std::lock_guard<std::mutex> lk(inst->mu);
  return cg_http_policy_update(inst->engine, eng.data(), eng.size());
}

int cg_proxylib_stats(uint64_t instance, uint64_t* batches, uint64_t* calls) {
  auto inst = find_instance(instance);
  if (!inst) return CG_INVALID_INSTANCE;
  std::lock_guard<std::mutex> lk(inst->qmu);
  if (batches) *batches = inst->batches;
  if (calls) *calls = inst->calls;
  return CG_OK;
}

int cg_proxylib_set_batching(uint64_t instance, uint32_t min_calls, uint32_t max_wait_us) {
  auto inst = find_instance(instance);
  if (!inst) return CG_INVALID_INSTANCE;
  std::lock_guard<std::mutex> lk(inst->qmu);
  inst->min_calls = min_calls ? min_calls : 1;
  inst->max_wait_us = max_wait_us;
  return CG_OK;
}

int cg_proxylib_policy_update_npds(uint64_t instance, const uint8_t* resp, size_t len) {
  std::string json;
  try {
    if (!resp && len) fail(CG_INVALID_ARGUMENT, "NULL DiscoveryResponse");
    json = npds_pb_to_json(resp, len, false);  // golang/protobuf: no UTF-8 check
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (...) {
    set_error("NPDS protobuf decode failed");
    return CG_UNKNOWN_ERROR;
  }
  return cg_proxylib_policy_update(instance, json.data(), json.size());
}

uint64_t OpenModule(GoSlice params, uint8_t debug) {
  std::string key;
  const GoString* kv = static_cast<const GoString*>(params.data);
  for (int64_t i = 0; i < params.len; ++i) {
    const std::string k = gostr(kv[2 * i]), v = gostr(kv[2 * i + 1]);
    if (k != "access-log-path" && k != "xds-path" && k != "node-id") return 0;
    key += k + "=" + v + ";";
  }
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_instance_by_key.find(key);  // same parameters → same instance (libcilium.h:108)
  if (it != g_instance_by_key.end()) return it->second;
  const char* dv = getenv("CILIUM_GPU_DEVICE");
  const std::string dev = dv ? dv : "0";
  cg_kv p{"device", dev.c_str()};
  const uint64_t h = cg_open(&p, 1, debug);
  if (h == 0) return 0;
  auto inst = std::make_shared<Instance>();
  inst->engine = h;
  inst->key = key;
  const uint64_t id = g_next_instance++;
  g_instances[id] = inst;
  g_instance_by_key[key] = id;
  return id;
}

void CloseModule(uint64_t id) {
  std::shared_ptr<Instance> inst;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_instances.find(id);
    if (it == g_instances.end()) return;
    inst = it->second;
    g_instances.erase(it);
    g_instance_by_key.erase(inst->key);
  }
  cg_close(inst->engine);
}

FilterResult OnNewConnection(uint64_t instanceId, GoString proto, uint64_t connectionId, uint8_t ingress,
                             uint32_t srcId, uint32_t dstId, GoString srcAddr, GoString dstAddr,
                             GoString policyName, GoSlice* origBuf, GoSlice* replyBuf) {
  auto inst = find_instance(instanceId);
  if (!inst) return FILTER_INVALID_INSTANCE;
  auto c = std::make_shared<Conn>();
  c->parser = gostr(proto);
  // parser factories implemented here: r2d2, memcache, cassandra
  if (c->parser != "r2d2" && c->parser != "memcache" && c->parser != "cassandra") return FILTER_UNKNOWN_PARSER;
  // net.SplitHostPort + ParseUint(port, 10, 32), port != 0 (connection.go:71-78)
  const std::string da = gostr(dstAddr);
  const size_t colon = da.rfind(':');
  if (colon == std::string::npos || colon + 1 >= da.size()) return FILTER_INVALID_ADDRESS;
  uint64_t port = 0;
  for (size_t i = colon + 1; i < da.size(); ++i) {
    if (da[i] < '0' || da[i] > '9') return FILTER_INVALID_ADDRESS;
    port = port * 10 + (uint64_t)(da[i] - '0');
    if (port > 0xFFFFFFFFull) return FILTER_INVALID_ADDRESS;
  }
  if (port == 0) return FILTER_INVALID_ADDRESS;
  c->inst = inst;
  c->ingress = ingress;
  c->src_id = srcId;
  c->dst_id = dstId;
  c->port = (uint32_t)port;
  c->policy = gostr(policyName);
  c->orig_buf = origBuf;
  c->reply_buf = replyBuf;
  std::lock_guard<std::mutex> lk(g_mu);
  g_conns[connectionId] = c;
  return FILTER_OK;
}

void Close(uint64_t connectionId) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_conns.erase(connectionId);
}

FilterResult OnData(uint64_t connectionId, uint8_t reply, uint8_t endStream, GoSlice* data, GoSlice* filterOps) {
  std::shared_ptr<Conn> c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_conns.find(connectionId);
    if (it == g_conns.end()) return FILTER_UNKNOWN_CONNECTION;
    c = it->second;
  }
  if (!data || !filterOps) return FILTER_UNKNOWN_ERROR;
  if (c->parser == "memcache") return memcache_data(*c, reply != 0, endStream != 0, data, filterOps);
  if (c->parser == "cassandra") return cassandra_data(*c, reply != 0, endStream != 0, data, filterOps);
  // r2d2 reads bytes.Join(dataArray) (r2d2parser.go:151)
  std::string in;
  const GoSlice* parts = static_cast<const GoSlice*>(data->data);
  for (int64_t i = 0; i < data->len; ++i) in.append(static_cast<const char*>(parts[i].data), (size_t)parts[i].len);
  // frames this call will emit ops for (connection.go:141-172: until the ops
  // slice is full or the parser asks for MORE)
  std::vector<Frame> frames;
  bool more = false;
  size_t pos = 0;
  const int64_t room = filterOps->cap - filterOps->len;
  while ((int64_t)frames.size() < room) {
    const size_t e = in.find("\r\n", pos);
    if (e == std::string::npos) {
      more = (int64_t)frames.size() < room;
      break;
    }
    Frame f{e - pos + 2, !reply, "", ""};
    if (f.request) {
      const std::string msg = in.substr(pos, e - pos);
      std::vector<std::string> fields;
      size_t a = 0;
      while (true) {  // strings.Split(msg, " ")
        const size_t b = msg.find(' ', a);
        fields.push_back(msg.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos) break;
        a = b + 1;
      }
      f.cmd = fields[0];
      if (fields.size() == 2) f.file = fields[1];
    }
    frames.push_back(std::move(f));
    pos = e + 2;
  }
  // one GPU batch for the request frames
  std::vector<uint8_t> allow(frames.size(), 1);
  std::vector<size_t> reqs;
  std::vector<std::string> recs;
  for (size_t i = 0; i < frames.size(); ++i)
    if (frames[i].request) {
      reqs.push_back(i);
      recs.push_back(field("cmd", esc(frames[i].cmd)) + field("file", esc(frames[i].file)));
    }
  if (!recs.empty()) {
    std::vector<uint8_t> out;
    if (!decide(*c, recs, &out)) return FILTER_UNKNOWN_ERROR;
    for (size_t k = 0; k < reqs.size(); ++k) allow[reqs[k]] = out[k];
  }
  FilterOp* ops = static_cast<FilterOp*>(filterOps->data);
  for (size_t i = 0; i < frames.size(); ++i) {
    if (!allow[i]) inject(c->reply_buf, "ERROR\r\n", 7);  // r2d2parser.go:197-199
    ops[filterOps->len++] = FilterOp{(uint64_t)(allow[i] ? FILTEROP_PASS : FILTEROP_DROP), (int64_t)frames[i].len};
  }
  if (more) ops[filterOps->len++] = FilterOp{FILTEROP_MORE, 1};
  return FILTER_OK;
}

}  // extern "C"
