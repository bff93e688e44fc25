// http.cc — compile Envoy cilium.NetworkPolicy (NPDS) HTTP rules into
// per-program union DFAs, pack requests, and a host walker for diagnostics.
//
// Reference semantics restated (envoy/cilium_network_policy.h):
//   PolicyInstance::Allowed(ingress, port, remote, headers)          :198-203
//   PortNetworkPolicy::Matches — exact port, then port 0, else allow  :169-192
//     (only TCP port policies are installed, :157-165; duplicate port
//      → EnvoyException rejects the update, :160-162)
//   PortNetworkPolicyRules::Matches — no HTTP rules → allow; empty → allow;
//     else OR over rules                                             :128-146
//   PortNetworkPolicyRule::Matches — remote set (empty = all), then OR over
//     HTTP rules (none = allow)                                      :90-108
//   HttpNetworkPolicyRule::Matches — AND over header matchers        :68-71
//
// Compilation: the header fields referenced by any matcher form a fixed
// field order F (":method", ":path", ":authority", then other names sorted).
// A request becomes the string  v_1 SEP v_2 SEP ... v_F SEP  with SEP = 0x00
// and an absent header encoded as the single byte 0x01; when every field from
// some point on is absent, that tail is the single byte REST = 0x02 instead
// (headers are mostly absent, so strings shrink by ~20%).  None of these
// bytes can occur in a header value Envoy's codec accepts (http_parser
// rejects control bytes other than HTAB), and the packer denies requests
// carrying one as malformed.  Each HTTP rule becomes a
// layered DFA (one deterministic automaton per field, chained by SEP); all
// rules of a program are unioned by subset construction over (rule, state)
// pairs, accepting states labelled with the set of PortNetworkPolicyRules
// (PNPRs) whose HTTP rule matched.  The kernel walks the string once and
// ANDs that label with the remote-identity mask.
#include "http.h"

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <functional>
#include <map>
#include <random>
#include <set>
#include <unordered_map>

#include "clsdfa.h"
#include "comb.h"
#include "json.h"
#include "regex.h"

namespace cg {

namespace {

constexpr uint8_t kSep = 0x00;
constexpr uint8_t kAbsent = 0x01;
constexpr uint8_t kRestAbsent = 0x02;  // every remaining field absent (ends the string)
constexpr int kMaxUnionStates = 400000;  // before minimization, per part
constexpr int kMaxPartStates = 65535;    // u16 transition entries

// ListExact/ListPrefix/ListSearch (proxylib only): the field is a list of
// escaped items, each followed by the pair {0x03, 0x14}, and every item must
// equal / start with / contain a match of the value (memcached keys,
// proxylib/memcached/parser.go:54-97; zero items match)
// Prefix / Suffix / Range: Envoy HeaderMatchType::Prefix / Suffix / Range
// (prefix_match, suffix_match, range_match); `invert` = invert_match.
enum class MKind { Exact, Regex, Present, Search, ListExact, ListPrefix, ListSearch, Prefix, Suffix, Range };
struct MatcherSpec {
  std::string name;  // lowercase
  MKind kind;
  std::string value;
  bool invert = false;
  int64_t range_start = 0, range_end = 0;  // Range: [start, end)
};
struct PnprSpec {
  bool has_remotes = false;
  std::vector<uint64_t> remotes;
  bool has_http = false;
  std::vector<std::vector<MatcherSpec>> http;  // each: AND of matchers
};
struct ScopeSpec {
  std::vector<PnprSpec> rules;
};
struct PolicySpec {
  std::string name;
  // proxylib verdict contract (proxylib/proxylib/policymap.go:208-236): a port
  // with no policy (neither exact nor 0) is denied, where Envoy allows
  bool deny_unlisted = false;
  std::map<uint32_t, ScopeSpec> dir[2];  // [0] egress, [1] ingress
};

std::string lower(const std::string& s) {
  std::string o = s;
  for (auto& c : o)
    if (c >= 'A' && c <= 'Z') c = c - 'A' + 'a';
  return o;
}

MatcherSpec parse_matcher(const Json& h) {
  if (h.type != Json::OBJ) fail(CG_POLICY_REJECTED, "header matcher must be an object");
  MatcherSpec m;
  const Json* name = h.get("name");
  if (!name) fail(CG_POLICY_REJECTED, "header matcher without name");
  m.name = lower(name->as_str("name"));
  const Json* ex = h.get("exact_match");
  const Json* rx = h.get("regex_match");
  const Json* pr = h.get("present_match");
  // engine extension for proxylib parsers: an unanchored Go regexp.MatchString
  // (proxylib/r2d2/r2d2parser.go:80), compiled in MatchMode::Search
  const Json* rs = h.get("regex_search");
  const Json* le = h.get("list_exact");
  const Json* lp = h.get("list_prefix");
  const Json* ls = h.get("list_search");
  const Json* val = h.get("value");
  const Json* inv = h.get("invert_match");
  const Json* px = h.get("prefix_match");
  const Json* sx = h.get("suffix_match");
  const Json* rg = h.get("range_match");
  m.invert = inv && inv->type == Json::BOOL && inv->b;
  if (ex) {
    m.kind = MKind::Exact;
    m.value = ex->as_str("exact_match");
  } else if (px) {
    m.kind = MKind::Prefix;
    m.value = px->as_str("prefix_match");
  } else if (sx) {
    m.kind = MKind::Suffix;
    m.value = sx->as_str("suffix_match");
  } else if (rg) {
    if (rg->type != Json::OBJ) fail(CG_POLICY_REJECTED, "range_match must be an object");
    m.kind = MKind::Range;
    auto num = [&](const char* k) -> int64_t {
      const Json* j = rg->get(k);
      return j ? j->as_i64(k) : 0;
    };
    m.range_start = num("start");
    m.range_end = num("end");
    m.value = std::to_string(m.range_start) + "," + std::to_string(m.range_end);
  } else if (rx) {
    m.kind = MKind::Regex;
    m.value = rx->as_str("regex_match");
  } else if (rs) {
    m.kind = MKind::Search;
    m.value = rs->as_str("regex_search");
  } else if (le) {
    m.kind = MKind::ListExact;
    m.value = le->as_str("list_exact");
  } else if (lp) {
    m.kind = MKind::ListPrefix;
    m.value = lp->as_str("list_prefix");
  } else if (ls) {
    m.kind = MKind::ListSearch;
    m.value = ls->as_str("list_search");
  } else if (pr) {
    m.kind = MKind::Present;
  } else if (val) {
    // deprecated {value, regex} form: empty value = presence check
    m.value = val->as_str("value");
    const Json* isre = h.get("regex");
    bool re = false;
    if (isre) {
      if (isre->type == Json::BOOL) re = isre->b;
      else if (isre->type == Json::OBJ && isre->get("value")) re = isre->get("value")->b;
    }
    m.kind = m.value.empty() ? MKind::Present : (re ? MKind::Regex : MKind::Exact);
  } else {
    m.kind = MKind::Present;
  }
  return m;
}

std::vector<PolicySpec> parse_npds(const char* json, size_t len) {
  Json root = JsonParser(json, len).parse();
  const Json* list = &root;
  if (root.type == Json::OBJ) {
    list = root.get("resources");
    if (!list) fail(CG_POLICY_REJECTED, "expected a list of NetworkPolicy or {resources: [...]}");
  }
  if (list->type != Json::ARR) fail(CG_POLICY_REJECTED, "expected a list of NetworkPolicy");
  std::vector<PolicySpec> out;
  std::set<std::string> names;
  for (const Json& p : list->arr) {
    if (p.type != Json::OBJ) fail(CG_POLICY_REJECTED, "NetworkPolicy must be an object");
    PolicySpec ps;
    const Json* nm = p.get("name");
    if (!nm) fail(CG_POLICY_REJECTED, "NetworkPolicy without name");
    ps.name = nm->as_str("name");
    if (!names.insert(ps.name).second) fail(CG_POLICY_REJECTED, "duplicate NetworkPolicy name " + ps.name);
    if (const Json* pl = p.get("proxylib")) ps.deny_unlisted = pl->type == Json::BOOL && pl->b;
    for (int d = 0; d < 2; ++d) {
      const Json* ports = p.get(d ? "ingress_per_port_policies" : "egress_per_port_policies");
      if (!ports) continue;
      if (ports->type != Json::ARR) fail(CG_POLICY_REJECTED, "per_port_policies must be a list");
      for (const Json& pp : ports->arr) {
        uint32_t port = 0;
        if (const Json* j = pp.get("port")) port = (uint32_t)j->as_u64("port");
        bool tcp = true;
        if (const Json* j = pp.get("protocol")) {
          if (j->type == Json::STR) tcp = j->s == "TCP";
          else tcp = j->as_u64("protocol") == 0;
        }
        if (!tcp) continue;  // "NOT installing non-TCP policy" (cilium_network_policy.h:163-165)
        ScopeSpec sc;
        if (const Json* rules = pp.get("rules")) {
          if (rules->type != Json::ARR) fail(CG_POLICY_REJECTED, "rules must be a list");
          for (const Json& r : rules->arr) {
            PnprSpec pr;
            if (const Json* rp = r.get("remote_policies")) {
              if (rp->type != Json::ARR) fail(CG_POLICY_REJECTED, "remote_policies must be a list");
              for (const Json& id : rp->arr) pr.remotes.push_back(id.as_u64("remote_policies"));
              pr.has_remotes = !pr.remotes.empty();
            }
            if (const Json* hr = r.get("http_rules")) {
              if (hr->type != Json::NUL) {
                pr.has_http = true;
                if (const Json* lst = hr->get("http_rules")) {
                  if (lst->type != Json::ARR) fail(CG_POLICY_REJECTED, "http_rules must be a list");
                  for (const Json& rule : lst->arr) {
                    std::vector<MatcherSpec> ms;
                    if (const Json* hs = rule.get("headers")) {
                      if (hs->type != Json::ARR) fail(CG_POLICY_REJECTED, "headers must be a list");
                      for (const Json& h : hs->arr) ms.push_back(parse_matcher(h));
                    }
                    pr.http.push_back(std::move(ms));
                  }
                }
              }
            }
            sc.rules.push_back(std::move(pr));
          }
        }
        if (!ps.dir[d].emplace(port, std::move(sc)).second)
          fail(CG_POLICY_REJECTED, "PortNetworkPolicy: Duplicate port number");
      }
    }
    out.push_back(std::move(ps));
  }
  return out;
}

// Field-value alphabet: any byte except SEP and the absent markers.
ByteSet value_alphabet() {
  ByteSet s = ByteSet::all();
  s.w[0] &= ~7ULL;
  return s;
}

// One deterministic automaton per (field, conjunction of matchers).
struct FieldDfaCache {
  bool raw = false;  // proxylib snapshot: matchers see arbitrary bytes, escaped (regex.h)
  std::vector<ByteDfa> dfas;
  std::map<std::string, int> by_key;
  int any_id = -1;

  int add(ByteDfa d, const std::string& key) {
    auto it = by_key.find(key);
    if (it != by_key.end()) return it->second;
    dfas.push_back(std::move(d));
    by_key[key] = (int)dfas.size() - 1;
    return (int)dfas.size() - 1;
  }
  int any() {
    if (any_id < 0) {
      ByteSet a = ByteSet::all();
      a.w[0] &= ~5ULL;  // everything but SEP and REST (the absent marker included)
      any_id = add(dfa_star(a), "ANY");
    }
    return any_id;
  }
  int single(const MatcherSpec& m) {
    std::string key = std::string(1, "ERPSLKQXYZ"[(int)m.kind]) + (m.invert ? "!" : "") + ":" + m.value;
    auto it = by_key.find(key);
    if (it != by_key.end()) return it->second;
    // Envoy values never hold 0x00-0x02 (the codec rejects them); proxylib
    // values may hold any byte and arrive escaped (packer), so their
    // matchers are compiled over all bytes and then escaped
    ByteSet va = raw ? ByteSet::all() : value_alphabet();
    ByteDfa d;
    switch (m.kind) {
      // Envoy HeaderMatchType::Value: an empty value matches any present
      // header (HeaderUtility::matchHeaders "value_.empty() ||"); proxylib
      // translations use exact "" for an empty field (proxylib.py cassandra)
      case MKind::Exact: d = (!raw && m.value.empty()) ? dfa_star(va) : dfa_literal(m.value, va); break;
      case MKind::Regex: d = compile_regex(m.value, va, MatchMode::Full); break;
      case MKind::Present: d = dfa_star(va); break;
      case MKind::Search: d = compile_regex(m.value, va, MatchMode::Search); break;
      case MKind::ListExact: d = dfa_literal(m.value, va); break;
      case MKind::ListPrefix: d = dfa_prefix(m.value, va); break;
      case MKind::ListSearch: d = compile_regex(m.value, va, MatchMode::Search); break;
      case MKind::Prefix: d = dfa_prefix(m.value, va); break;
      case MKind::Suffix: d = dfa_suffix(m.value, va); break;
      case MKind::Range: d = dfa_int_range(m.range_start, m.range_end, va); break;
    }
    // invert_match: the header must be present (an absent one never
    // matches: the absent marker is outside the value alphabet) and its
    // value outside the matcher's language
    if (m.invert) d = dfa_complement(d, va);
    const bool list = m.kind == MKind::ListExact || m.kind == MKind::ListPrefix || m.kind == MKind::ListSearch;
    if (list && !raw) fail(CG_POLICY_REJECTED, "list matchers are for proxylib policies");
    if (raw) d = dfa_escape_low(d);
    if (list) d = dfa_list(d);
    return add(std::move(d), key);
  }
  int conj(const std::vector<const MatcherSpec*>& ms) {
    if (ms.empty()) return any();
    std::vector<int> ids;
    for (auto* m : ms) ids.push_back(single(*m));
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    if (ids.size() == 1) return ids[0];
    std::string key = "AND";
    for (int i : ids) key += ":" + std::to_string(i);
    auto it = by_key.find(key);
    if (it != by_key.end()) return it->second;
    ByteDfa d = dfas[ids[0]];
    for (size_t i = 1; i < ids.size(); ++i) d = dfa_intersect(d, dfas[ids[i]]);
    return add(std::move(d), key);
  }
  bool empty_lang(int id) const {
    const ByteDfa& d = dfas[id];
    if (d.accept[d.start]) return false;
    for (int b = 0; b < 256; ++b)
      if (d.next(d.start, b)) return false;
    return true;
  }
};

struct URule {
  std::vector<int> fd;            // field dfa per field
  std::vector<uint32_t> tags;     // PNPR indices
};

struct VecHash64 {
  size_t operator()(const std::vector<uint64_t>& v) const {
    uint64_t h = 0x243f6a8885a308d3ULL ^ v.size();
    for (uint64_t x : v) h = mix64(h ^ x);
    return (size_t)h;
  }
};

struct TooBig {};

// Layered union construction over `rules` (indices into all_rules).
//
// A label keeps, per PortNetworkPolicyRule, only its lowest matched rule bit:
// a remote identity is allowed all of a PNPR's bits or none, so the first
// rule that allows a request is the lowest bit of (label & row) either way,
// and states that differ only in a PNPR's later matches stay merged (the
// union stays as small as with one bit per PNPR).  group[b] = the first bit
// of b's PNPR.
ClsDfa build_union(const FieldDfaCache& fc, const std::vector<URule>& all_rules,
                   const std::vector<int>& rules, int F, uint32_t W, const std::vector<uint32_t>& group,
                   std::vector<std::vector<uint64_t>>& label_masks) {
  // global byte classes: SEP alone, refined by every field DFA's columns
  std::vector<int> cls(256, 1);
  cls[kSep] = 0;
  cls[kRestAbsent] = 2;
  {
    std::set<int> used;
    for (int r : rules)
      for (int id : all_rules[r].fd) used.insert(id);
    for (int id : used) {
      const ByteDfa& d = fc.dfas[id];
      // column signature per byte
      std::map<std::vector<int32_t>, int> colid;
      std::vector<int> dc(256);
      std::vector<int32_t> col(d.size());
      for (int b = 0; b < 256; ++b) {
        for (int s = 0; s < d.size(); ++s) col[s] = d.trans[(size_t)s * 256 + b];
        dc[b] = colid.emplace(col, (int)colid.size()).first->second;
      }
      std::map<std::pair<int, int>, int> nid;
      for (int b = 0; b < 256; ++b) cls[b] = nid.emplace(std::make_pair(cls[b], dc[b]), (int)nid.size()).first->second;
    }
  }
  int ncls = 0;
  for (int b = 0; b < 256; ++b) ncls = std::max(ncls, cls[b] + 1);
  std::vector<int> rep(ncls, -1);
  for (int b = 0; b < 256; ++b)
    if (rep[cls[b]] < 0) rep[cls[b]] = b;

  ClsDfa d;
  d.ncls = ncls;
  for (int b = 0; b < 256; ++b) d.clsmap[b] = (uint8_t)cls[b];
  std::unordered_map<std::vector<uint64_t>, int, VecHash64> ids;
  std::vector<std::vector<uint64_t>> states;  // [0] = layer, then rule<<32|q
  std::map<std::vector<uint64_t>, uint32_t> mask_ids;
  label_masks.clear();

  auto label_of = [&](const std::vector<uint64_t>& st) -> uint32_t {
    if ((int)st[0] != F) return 0;
    std::vector<uint64_t> m(W, 0);
    for (size_t i = 1; i < st.size(); ++i)
      for (uint32_t t : all_rules[(size_t)(st[i] >> 32)].tags) m[t >> 6] |= 1ULL << (t & 63);
    uint32_t kept_group = 0xFFFFFFFFu;  // keep the lowest bit of each PNPR group
    for (uint32_t b = 0; b < 64 * W; ++b) {
      if (!((m[b >> 6] >> (b & 63)) & 1)) continue;
      if (group[b] == kept_group) m[b >> 6] &= ~(1ULL << (b & 63));
      else kept_group = group[b];
    }
    auto it = mask_ids.emplace(m, (uint32_t)mask_ids.size() + 1);
    if (it.second) label_masks.push_back(m);
    return it.first->second;
  };
  auto intern = [&](std::vector<uint64_t>&& st) -> int {
    if (st.size() == 1) return 0;  // no live rule
    auto it = ids.find(st);
    if (it != ids.end()) return it->second;
    int id = (int)states.size();
    if (id >= kMaxUnionStates) throw TooBig{};
    ids.emplace(st, id);
    d.label.push_back(label_of(st));
    states.push_back(std::move(st));
    d.trans.resize((size_t)(id + 1) * ncls, 0);
    return id;
  };
  // dead
  states.push_back({(uint64_t)-1});
  d.label.push_back(0);
  d.trans.assign(ncls, 0);
  // start
  {
    std::vector<uint64_t> st{0};
    for (int r : rules) {
      if (F == 0) {
        st.push_back((uint64_t)r << 32 | 1);
      } else {
        st.push_back((uint64_t)r << 32 | (uint32_t)fc.dfas[all_rules[r].fd[0]].start);
      }
    }
    if (F == 0) st[0] = 0;  // layer 0 == F
    if (st.size() == 1) {
      // no rules: start is a copy of dead
      states.push_back({(uint64_t)-2});
      d.label.push_back(0);
      d.trans.resize(2 * ncls, 0);
    } else {
      int id = (int)states.size();
      ids.emplace(st, id);
      d.label.push_back(label_of(st));
      states.push_back(st);
      d.trans.resize((size_t)(id + 1) * ncls, 0);
    }
  }
  std::vector<uint64_t> nx;
  for (size_t si = 1; si < states.size(); ++si) {
    if (states[si][0] == (uint64_t)-2) break;
    const int f = (int)states[si][0];
    for (int c = 0; c < ncls; ++c) {
      int b = rep[c];
      int target = 0;
      if (f < F) {
        const std::vector<uint64_t>& cur = states[si];
        nx.clear();
        if (b == kRestAbsent) {
          // fields f..F-1 all absent: a rule survives iff each of its
          // remaining field automata accepts the absent marker (from its
          // current state for field f, which the packer only leaves at the
          // field's start)
          nx.push_back((uint64_t)F);
          for (size_t i = 1; i < cur.size(); ++i) {
            uint32_t r = (uint32_t)(cur[i] >> 32), q = (uint32_t)cur[i];
            bool ok = true;
            for (int g = f; g < F && ok; ++g) {
              const ByteDfa& fd = fc.dfas[all_rules[r].fd[g]];
              const int s1 = fd.next(g == f ? (int)q : fd.start, kAbsent);
              ok = s1 != 0 && fd.accept[s1];
            }
            if (ok) nx.push_back((uint64_t)r << 32 | 1u);
          }
        } else if (b == kSep) {
          nx.push_back((uint64_t)(f + 1));
          for (size_t i = 1; i < cur.size(); ++i) {
            uint32_t r = (uint32_t)(cur[i] >> 32), q = (uint32_t)cur[i];
            const ByteDfa& fd = fc.dfas[all_rules[r].fd[f]];
            if (!fd.accept[q]) continue;
            uint32_t nq = (f + 1 < F) ? (uint32_t)fc.dfas[all_rules[r].fd[f + 1]].start : 1u;
            nx.push_back((uint64_t)r << 32 | nq);
          }
        } else {
          nx.push_back((uint64_t)f);
          for (size_t i = 1; i < cur.size(); ++i) {
            uint32_t r = (uint32_t)(cur[i] >> 32), q = (uint32_t)cur[i];
            int nq = fc.dfas[all_rules[r].fd[f]].next((int)q, b);
            if (nq) nx.push_back((uint64_t)r << 32 | (uint32_t)nq);
          }
        }
        target = intern(std::vector<uint64_t>(nx));
      }
      d.trans[si * ncls + c] = target;
    }
  }
  return d;
}

struct PartOut {
  ClsDfa dfa;
  CombTable comb;
  std::vector<std::vector<uint64_t>> label_masks;
};

void build_parts(const FieldDfaCache& fc, const std::vector<URule>& all_rules, std::vector<int> rules,
                 int F, uint32_t W, const std::vector<uint32_t>& group, std::vector<PartOut>& out) {
  if (rules.empty()) return;
  PartOut p;
  bool ok = true;
  try {
    ClsDfa raw = build_union(fc, all_rules, rules, F, W, group, p.label_masks);
    p.dfa = minimize_cls(raw);
    std::vector<uint32_t> labels(p.dfa.size(), kCombNoLabel);
    for (int s = 0; s < p.dfa.size(); ++s)
      if (p.dfa.label[s]) labels[s] = p.dfa.label[s] - 1;
    if (p.dfa.size() > kMaxPartStates || p.label_masks.size() >= kCombNoLabel ||
        !build_comb(p.dfa, labels, &p.comb))
      ok = false;
  } catch (const TooBig&) {
    ok = false;
  }
  if (ok) {
    if (getenv("CILIUM_GPU_DEBUG"))
      fprintf(stderr, "[cilium-gpu] http part: %zu rules, %d states, %d byte classes, %zu comb cells\n", rules.size(),
              p.dfa.size(), p.dfa.ncls, p.comb.cells.size());
    out.push_back(std::move(p));
    return;
  }
  if (rules.size() == 1) fail(CG_UNSUPPORTED, "a single HTTP rule exceeds the DFA state budget");
  std::vector<int> a(rules.begin(), rules.begin() + rules.size() / 2);
  std::vector<int> b(rules.begin() + rules.size() / 2, rules.end());
  build_parts(fc, all_rules, a, F, W, group, out);
  build_parts(fc, all_rules, b, F, W, group, out);
}

}  // namespace

uint32_t http_next_epoch() {
  static std::atomic<uint32_t> g_epoch{0};
  return ++g_epoch;
}

std::shared_ptr<HttpSnapshot> http_compile(const char* json, size_t len) {
  std::vector<PolicySpec> pols = parse_npds(json, len);
  auto snap = std::make_shared<HttpSnapshot>();
  HttpSnapshot& S = *snap;
  S.epoch = http_next_epoch();
  if (pols.size() >= 0x7FFF) fail(CG_POLICY_REJECTED, "too many policies");

  // ---- field order
  std::set<std::string> names;
  for (const auto& p : pols)
    for (int d = 0; d < 2; ++d)
      for (const auto& [port, sc] : p.dir[d])
        for (const auto& pr : sc.rules)
          for (const auto& hr : pr.http)
            for (const auto& m : hr) names.insert(m.name);
  for (const char* pseudo : {":method", ":path", ":authority"})
    if (names.count(pseudo)) {
      S.fields.push_back(pseudo);
      names.erase(pseudo);
    }
  for (const auto& n : names) S.fields.push_back(n);
  const int F = (int)S.fields.size();
  std::map<std::string, int> field_idx;
  for (int i = 0; i < F; ++i) field_idx[S.fields[i]] = i;

  FieldDfaCache fc;
  {
    size_t nraw = 0;
    for (const auto& p : pols) nraw += p.deny_unlisted;
    if (nraw && nraw != pols.size())
      fail(CG_POLICY_REJECTED, "proxylib and Envoy HTTP policies cannot share one snapshot");
    S.raw_values = fc.raw = nraw != 0;
  }
  S.npolicies = (uint32_t)pols.size();
  S.dflt.assign((size_t)S.npolicies * 2, kProgAllow);
  std::vector<std::pair<uint32_t, uint32_t>> phash;  // key → prog


  // Build one program from the merged PNPR list; returns program id.
  //
  // Mask bits are rules in Envoy's evaluation order: the exact port's
  // PortNetworkPolicyRules, then port 0's; within a PNPR one bit per
  // HttpNetworkPolicyRule (one bit for a PNPR without HTTP rules).  A
  // request's first matching rule is then the lowest bit of (its accept
  // label | the "always" bits) & its remote row, and its per-rule hit counter
  // is rule_base + that bit.  A scope without HTTP rules allows everything
  // (:129-138): first in the order it decides the program alone (allow-all,
  // nothing attributed); after the exact port's rules it is one more
  // always-matching bit whose counter records "allowed by the wildcard
  // scope" (rule_info http = CG_HTTP_RULE_SCOPE_ALLOW).
  auto build_prog = [&](const std::vector<const ScopeSpec*>& scopes, uint32_t key, uint32_t pol_idx,
                        uint32_t ingress, uint32_t port) -> uint32_t {
    HttpProg pg{};
    uint32_t pid = (uint32_t)S.progs.size();
    struct Bit {
      const PnprSpec* pnpr;  // nullptr: an allow-all scope
      uint32_t scope, pnpr_idx, http_idx;
    };
    std::vector<Bit> bits;
    std::vector<uint32_t> pnpr_first;  // first bit of each entry of pnprs
    std::vector<const PnprSpec*> pnprs;
    for (uint32_t si = 0; si < scopes.size(); ++si) {
      const ScopeSpec* sc = scopes[si];
      bool have_http = false;
      for (const auto& r : sc->rules) have_http |= r.has_http;
      if (!have_http || sc->rules.empty()) {  // :129-138
        if (si == 0) {
          pg.flags = kProgAllowAll;
          S.progs.push_back(pg);
          S.prog_key.push_back(key);
          return pid;
        }
        bits.push_back({nullptr, si, 0, CG_HTTP_RULE_SCOPE_ALLOW});
        break;  // rules after an allow-all scope are never reached
      }
      for (uint32_t ri = 0; ri < sc->rules.size(); ++ri) {
        const PnprSpec& r = sc->rules[ri];
        pnprs.push_back(&r);
        pnpr_first.push_back((uint32_t)bits.size());
        if (r.http.empty()) bits.push_back({&r, si, ri, CG_HTTP_RULE_NO_HTTP});
        for (uint32_t hi = 0; hi < r.http.size(); ++hi) bits.push_back({&r, si, ri, hi});
      }
    }
    const uint32_t R = (uint32_t)bits.size();
    const uint32_t W = (R + 63) / 64;
    pg.mask_words = W;
    pg.rule_base = (uint32_t)S.rule_info.size();
    pg.nrules = R;
    for (const Bit& b : bits) S.rule_info.push_back({pol_idx, ingress, port, b.scope, b.pnpr_idx, b.http_idx});
    // always: PNPRs with no HTTP rules (and an allow-all scope) match any
    // payload (:98-107); open: bits of PNPRs without a remote set
    std::vector<uint64_t> always(W, 0), open(W, 0);
    std::map<uint32_t, std::vector<uint64_t>> by_remote;
    for (uint32_t j = 0; j < R; ++j) {
      const Bit& b = bits[j];
      if (!b.pnpr || b.pnpr->http.empty()) always[j >> 6] |= 1ULL << (j & 63);
      if (!b.pnpr || !b.pnpr->has_remotes) open[j >> 6] |= 1ULL << (j & 63);
    }
    for (uint32_t j = 0; j < R; ++j) {
      const Bit& b = bits[j];
      if (!b.pnpr || !b.pnpr->has_remotes) continue;
      for (uint64_t rid : b.pnpr->remotes) {
        if (rid > 0xFFFFFFFFULL) continue;  // can never equal a u32 identity
        auto it = by_remote.find((uint32_t)rid);
        if (it == by_remote.end()) it = by_remote.emplace((uint32_t)rid, open).first;
        it->second[j >> 6] |= 1ULL << (j & 63);
      }
    }
    for (uint64_t w : always)
      if (w) pg.flags |= kProgHasAlways;
    // union rules: each HTTP rule tags its own bit
    std::vector<URule> urules;
    std::map<std::vector<int>, size_t> dedupe;
    for (uint32_t j = 0; j < (uint32_t)pnprs.size(); ++j) {
      uint32_t bit = pnpr_first[j];
      for (const auto& hr : pnprs[j]->http) {
        const uint32_t tag = bit++;
        std::vector<std::vector<const MatcherSpec*>> per_field(F);
        for (const auto& m : hr) per_field[field_idx[m.name]].push_back(&m);
        std::vector<int> fd(F);
        bool empty = false;
        for (int f = 0; f < F; ++f) {
          fd[f] = fc.conj(per_field[f]);
          if (fc.empty_lang(fd[f])) empty = true;
        }
        if (empty) continue;
        auto it = dedupe.find(fd);
        if (it == dedupe.end()) {
          dedupe[fd] = urules.size();
          urules.push_back({fd, {tag}});
        } else {
          urules[it->second].tags.push_back(tag);
        }
      }
    }
    S.total_rules += urules.size();
    std::vector<int> idx(urules.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int)i;
    std::vector<PartOut> parts;
    std::vector<uint32_t> group(64 * (size_t)W, 0xFFFFFFFEu);
    for (uint32_t j = 0; j < R; ++j) group[j] = (j && bits[j].pnpr == bits[j - 1].pnpr) ? group[j - 1] : j;
    build_parts(fc, urules, idx, F, W, group, parts);
    // one part over at most 64 byte classes: class-indexed rows with states
    // as byte offsets (comb.h), the strings packed as class codes
    std::array<uint8_t, 256> code{};
    if (parts.size() == 1 && parts[0].dfa.ncls <= 64) {
      ClsDfa z = zero_class_first(parts[0].dfa);
      std::vector<uint32_t> labels(z.size(), kCombNoLabel);
      for (int st = 0; st < z.size(); ++st)
        if (z.label[st]) labels[st] = z.label[st] - 1;
      CombTable cc;
      if (build_comb(z, labels, &cc, kCombMaxBase, true) && scale_comb(&cc)) {
        parts[0].dfa = std::move(z);
        parts[0].comb = std::move(cc);
        pg.flags |= kProgClass;
        for (int b = 0; b < 256; ++b) code[b] = (uint8_t)(4 * parts[0].dfa.clsmap[b]);
      }
    }
    if (pg.flags & kProgClass) {
      S.prog_code.resize(pid + 1);
      S.prog_code[pid] = code;
    }
    pg.part_begin = (uint32_t)S.parts.size();
    pg.part_count = (uint32_t)parts.size();
    while (S.cells.size() & 3) S.cells.push_back(kCombEmpty);  // blocks start 16-byte aligned
    pg.cell_begin = (uint32_t)S.cells.size();
    size_t block = 0;
    for (const auto& po : parts) block += po.comb.cells.size();
    const bool rebase = block <= kCombMaxBase;
    if (rebase) pg.flags |= kProgRebased;
    for (auto& po : parts) {
      HttpPart hp{};
      const ClsDfa& d = po.dfa;
      CombTable& cb = po.comb;
      hp.cell_off = (uint32_t)S.cells.size();
      if (rebase) rebase_comb(&cb, hp.cell_off - pg.cell_begin);
      hp.walk_off = rebase ? pg.cell_begin : hp.cell_off;
      hp.nstates = (uint32_t)d.size();
      hp.start = cb.start;
      hp.dead = cb.dead;
      hp.ncells = (uint32_t)cb.cells.size();
      hp.mode = cb.scaled ? kPartClass : 0;
      S.cells.insert(S.cells.end(), cb.cells.begin(), cb.cells.end());
      S.total_states += d.size();
      S.total_exceptions += cb.exceptions;
      S.parts.push_back(hp);
    }
    // The block continues with each part's label masks (indexed by accept
    // label) and the "always" mask, masks as 8-byte-aligned u64 pairs at
    // block-relative u32 offsets: the kernel stages the whole block into LDS
    // with the DFA.
    auto put_mask = [&](const std::vector<uint64_t>& m) -> uint32_t {
      if (S.cells.size() & 1) S.cells.push_back(0);
      const uint32_t off = (uint32_t)S.cells.size() - pg.cell_begin;
      for (uint64_t w : m) {
        S.cells.push_back((uint32_t)w);
        S.cells.push_back((uint32_t)(w >> 32));
      }
      return off;
    };
    // each part's label masks back to back (stride 2W u32): accept label l of
    // part i has its PNPR mask at block offset acc_off + l * 2W
    for (size_t i = 0; i < parts.size(); ++i) {
      HttpPart& hp = S.parts[pg.part_begin + i];
      if (S.cells.size() & 1) S.cells.push_back(0);
      hp.acc_off = (uint32_t)S.cells.size() - pg.cell_begin;
      for (size_t l = 0; l < parts[i].label_masks.size(); ++l) put_mask(parts[i].label_masks[l]);
    }
    pg.always_off = put_mask(always);
    // remote-identity table (PortNetworkPolicyRule remote sets, :90-97):
    // identity → block offset of its rule mask row (rows deduplicated;
    // dev_types.h rtab_b1/rtab_b2 buckets); unlisted identities get the row
    // of the rules without a remote set
    {
      std::map<std::vector<uint64_t>, uint32_t> rows;
      auto row_of = [&](const std::vector<uint64_t>& m) {
        auto it = rows.find(m);
        if (it == rows.end()) it = rows.emplace(m, put_mask(m)).first;
        return it->second;
      };
      pg.default_remote = row_of(open);
      std::vector<std::pair<uint32_t, uint32_t>> ent;
      for (auto& [rid, m] : by_remote) ent.push_back({rid, row_of(m)});
      // 2-choice cuckoo placement into the fewest buckets that take it
      uint32_t nb = (uint32_t)std::max<size_t>((ent.size() * 10 / 9 + 3) / 4, 1);
      std::vector<std::pair<uint32_t, uint32_t>> slots;  // (identity, row) per slot, row kNoRow = empty
      for (;; nb += nb / 8 + 1) {
        if (nb >= 65536) fail(CG_POLICY_REJECTED, "too many remote identities in one HTTP policy scope");
        slots.assign((size_t)nb * 4, {0u, kNoRow});
        std::mt19937 rng(0xC111A);
        auto put = [&](uint32_t bk, const std::pair<uint32_t, uint32_t>& e) {
          for (int sl = 0; sl < 4; ++sl)
            if (slots[(size_t)bk * 4 + sl].second == kNoRow) {
              slots[(size_t)bk * 4 + sl] = e;
              return true;
            }
          return false;
        };
        bool ok = true;
        for (const auto& e : ent) {
          auto cur = e;
          uint32_t from = 0xFFFFFFFFu;
          bool placed = false;
          for (int kick = 0; kick < 500 && !placed; ++kick) {
            const uint32_t c1 = rtab_b1(cur.first, nb), c2 = rtab_b2(cur.first, nb);
            if (put(c1, cur) || put(c2, cur)) {
              placed = true;
              break;
            }
            // evict from the bucket the current entry did not come from
            const uint32_t vb = c1 == from ? c2 : c2 == from ? c1 : (rng() & 1) ? c1 : c2;
            std::swap(cur, slots[(size_t)vb * 4 + (rng() & 3)]);
            from = vb;
          }
          if (!placed) {
            ok = false;
            break;
          }
        }
        if (ok) break;
      }
      while ((S.cells.size() - pg.cell_begin) & 3) S.cells.push_back(0);  // buckets 16-byte aligned

      pg.rtab_off = (uint32_t)S.cells.size() - pg.cell_begin;
      pg.rtab_nb = nb;
      // empty slots: an identity the table does not hold, with the default row
      uint32_t empty_id = 0;
      while (by_remote.count(empty_id)) ++empty_id;
      const size_t at = S.cells.size();
      S.cells.resize(at + kRtabBucketCells * (size_t)nb, 0);
      for (uint32_t k = 0; k < nb; ++k)
        for (int sl = 0; sl < 4; ++sl) {
          const auto& e = slots[(size_t)k * 4 + sl];
          const bool empty = e.second == kNoRow;
          S.cells[at + kRtabBucketCells * k + sl] = empty ? empty_id : e.first;
          S.cells[at + kRtabBucketCells * k + 4 + sl] = empty ? pg.default_remote : e.second;
        }
      const uint32_t cap = 4 * nb;
      S.total_remote_slots += cap;
      // identities over a short span (identities are allocated densely): a
      // direct u16 row array as well, which the kernel prefers
      if (!ent.empty()) {
        uint32_t lo = ent[0].first, hi = ent[0].first;
        bool rows16 = pg.default_remote < 0x10000;
        for (const auto& e : ent) {
          lo = std::min(lo, e.first);
          hi = std::max(hi, e.first);
          rows16 &= e.second < 0x10000;
        }
        if (rows16 && hi - lo < kRdirMaxSpan) {
          const uint32_t len = hi - lo + 1;
          std::vector<uint16_t> t(len + 1, (uint16_t)pg.default_remote);
          for (const auto& e : ent) t[e.first - lo] = (uint16_t)e.second;
          pg.rdir_base = lo;
          pg.rdir_len = len;
          pg.rdir_off = (uint32_t)S.cells.size() - pg.cell_begin;
          for (uint32_t k = 0; k < len; k += 2) S.cells.push_back((uint32_t)t[k] | (uint32_t)t[k + 1] << 16);
          pg.flags |= kProgRemoteDirect;
        }
      }
    }
    S.cells.push_back(0);  // spare words: the kernel reads two mask words whatever the width
    S.cells.push_back(0);
    pg.cell_count = (uint32_t)S.cells.size() - pg.cell_begin;
    if (getenv("CILIUM_GPU_DEBUG")) {
      size_t comb = 0, labels = 0;
      for (uint32_t i = 0; i < pg.part_count; ++i) {
        comb += S.parts[pg.part_begin + i].ncells;
        labels += parts[i].label_masks.size();
      }
      fprintf(stderr, "[cilium-gpu] http program %u: block %u cells (comb %zu, %zu labels x %u words, remote table %u "
              "buckets, direct %u)\n", pid, pg.cell_count, comb, labels, 2 * pg.mask_words, pg.rtab_nb, pg.rdir_len);
    }
    S.progs.push_back(pg);
    S.prog_key.push_back(key);
    return pid;
  };

  for (uint32_t pi = 0; pi < pols.size(); ++pi) {
    const PolicySpec& p = pols[pi];
    S.policy_index[p.name] = pi;
    for (int d = 0; d < 2; ++d) {
      const auto& ports = p.dir[d];
      const ScopeSpec* wild = nullptr;
      auto w = ports.find(0);
      if (w != ports.end()) wild = &w->second;
      if (p.deny_unlisted) S.dflt[pi * 2 + d] = kProgDeny;
      if (wild) S.dflt[pi * 2 + d] = build_prog({wild}, (pi << 17) | ((uint32_t)d << 16), pi, d, 0);
      for (const auto& [port, sc] : ports) {
        if (port == 0) continue;
        if (port > 0xFFFF) continue;  // can never equal a 16-bit destination port
        std::vector<const ScopeSpec*> scs{&sc};
        if (wild) scs.push_back(wild);
        uint32_t key = (pi << 17) | ((uint32_t)d << 16) | port;
        phash.push_back({key, build_prog(scs, key, pi, d, port)});
      }
    }
  }

  // ---- hash tables
  {
    uint32_t cap = next_pow2(std::max<size_t>(2 * phash.size(), 16));
    S.phash_keys.assign(cap, 0xFFFFFFFFu);
    S.phash_vals.assign(cap, 0);
    S.phash_mask = cap - 1;
    for (auto [k, v] : phash) {
      uint32_t h = hash32(k) & S.phash_mask;
      while (S.phash_keys[h] != 0xFFFFFFFFu) h = (h + 1) & S.phash_mask;
      S.phash_keys[h] = k;
      S.phash_vals[h] = v;
    }
  }
  if (S.cells.empty()) S.cells.push_back(kCombEmpty);
  if (S.progs.empty()) S.progs.push_back(HttpProg{});
  S.prog_code.resize(S.progs.size());
  if (S.parts.empty()) S.parts.push_back(HttpPart{});
  if (S.dflt.empty()) S.dflt.push_back(kProgDeny);
  return snap;
}

uint32_t HttpSnapshot::lookup_prog(uint32_t policy, bool ingress, uint32_t port) const {
  if (policy >= npolicies) return kProgDeny;
  uint32_t key = (policy << 17) | ((uint32_t)ingress << 16) | (port & 0xFFFF);
  uint32_t h = hash32(key) & phash_mask;
  while (phash_keys[h] != 0xFFFFFFFFu) {
    if (phash_keys[h] == key) return phash_vals[h];
    h = (h + 1) & phash_mask;
  }
  return dflt[policy * 2 + (ingress ? 1 : 0)];
}

void HttpSnapshot::upload(Engine& e) {
  if (!e.has_gpu()) return;
  d_progs.upload_vec(progs);
  d_parts.upload_vec(parts);
  d_cells.upload_vec(cells);
  d_dflt.upload_vec(dflt);
  // [2 * prog] allowed, [2 * prog + 1] denied, [2 * nprogs] stale batches,
  // then one hit counter per rule (rule_info order): the all-reduce vector
  d_counters.alloc((std::max<size_t>(progs.size(), 1) * 2 + 1 + rule_info.size()) * sizeof(uint64_t));
  d_counters.zero();
  dev.progs = d_progs.as<HttpProg>();
  dev.parts = d_parts.as<HttpPart>();
  dev.cells = d_cells.as<uint32_t>();
  dev.dflt = d_dflt.as<uint32_t>();
  dev.npolicies = npolicies;
  dev.nprogs = (uint32_t)progs.size();
  dev.nparts = (uint32_t)parts.size();
  dev.epoch = epoch;
  // LDS per workgroup = the largest rebased program table (so 160 KiB / that
  // many workgroups share a CU); larger programs walk from global memory
  uint32_t max_cells = 0;
  for (const auto& pg : progs)
    if (!(pg.flags & kProgAllowAll) && (pg.flags & kProgRebased) && pg.cell_count <= kMaxLdsCells)
      max_cells = std::max(max_cells, pg.cell_count);
  dev.lds_cells = std::min((max_cells + 255) & ~255u, kMaxLdsCells);
  dev.n_global_progs = 0;
  for (const auto& pg : progs)
    if (!(pg.flags & kProgAllowAll) && !((pg.flags & kProgRebased) && pg.cell_count <= dev.lds_cells))
      dev.n_global_progs++;
  dev.counters = d_counters.as<unsigned long long>();
  dev.rule_hits = dev.counters + 2 * (size_t)dev.nprogs + 1;
  http_raw_upload(*this);
}

}  // namespace cg
