// kafka.cc — compile Kafka L7 rule sets.
//
// Reference: kafkaRedirect.canAccess (pkg/proxy/kafka.go:117-153) gathers
// L7DataMap.GetRelevantRules(identity) (pkg/policy/l4.go:118-141: rules of
// every selector matching the identity, plus the wildcard selector's) and
// denies when none exist; otherwise RequestMessage.MatchesRule
// (pkg/kafka/policy.go:200-225).  Rules are Sanitize()d as at policy import
// (pkg/policy/api/rule_validation.go:232-275).
//
// MatchesRule is order-independent: it returns true iff some rule with an
// empty Topic (or any rule, when the request has no topics) matches, or
// every distinct request topic is the Topic of some matching rule.  The
// device evaluation computes exactly that.
#include "kafka.h"

#include <algorithm>
#include <set>

#include "json.h"

namespace cg {

namespace {

// KafkaAPIKeyMap, pkg/policy/api/kafka.go:153-188
const std::map<std::string, int> kApiKeys = {
    {"produce", 0},        {"fetch", 1},           {"offsets", 2},        {"metadata", 3},
    {"leaderandisr", 4},   {"stopreplica", 5},     {"updatemetadata", 6}, {"controlledshutdown", 7},
    {"offsetcommit", 8},   {"offsetfetch", 9},     {"findcoordinator", 10}, {"joingroup", 11},
    {"heartbeat", 12},     {"leavegroup", 13},     {"syncgroup", 14},     {"describegroups", 15},
    {"listgroups", 16},    {"saslhandshake", 17},  {"apiversions", 18},   {"createtopics", 19},
    {"deletetopics", 20},  {"deleterecords", 21},  {"initproducerid", 22}, {"offsetforleaderepoch", 23},
    {"addpartitionstotxn", 24}, {"addoffsetstotxn", 25}, {"endtxn", 26}, {"writetxnmarkers", 27},
    {"txnoffsetcommit", 28}, {"describeacls", 29}, {"createacls", 30},   {"deleteacls", 31},
    {"describeconfigs", 32}, {"alterconfigs", 33}};

std::string lower(std::string s) {
  for (auto& c : s)
    if (c >= 'A' && c <= 'Z') c = c - 'A' + 'a';
  return s;
}

struct RuleSpec {
  uint64_t keys = 0;
  bool key_wild = true;
  bool ver_wild = true;
  int16_t version = 0;
  std::string client, topic;
};

// PortRuleKafka.Sanitize (rule_validation.go:232-275) + MapRoleToAPIKey
// (api/kafka.go:274-293).
RuleSpec sanitize(const Json& r) {
  auto str = [&](const char* k) -> std::string {
    const Json* j = r.get(k);
    return j && j->type == Json::STR ? j->s : std::string();
  };
  std::string role = str("role"), apikey = str("apiKey"), ver = str("apiVersion");
  RuleSpec s;
  s.client = str("clientID");
  s.topic = str("topic");
  if (!apikey.empty() && !role.empty())
    fail(CG_POLICY_REJECTED, "Cannot set both Role:\"" + role + "\" and APIKey :\"" + apikey + "\" together");
  if (!apikey.empty()) {
    auto it = kApiKeys.find(lower(apikey));
    if (it == kApiKeys.end()) fail(CG_POLICY_REJECTED, "invalid Kafka APIKey :\"" + apikey + "\"");
    s.key_wild = false;
    s.keys |= 1ULL << it->second;
  }
  if (!role.empty()) {
    std::string lr = lower(role);
    s.key_wild = false;
    if (lr == "produce") {
      for (int k : {0, 3, 18}) s.keys |= 1ULL << k;
    } else if (lr == "consume") {
      for (int k : {1, 2, 3, 8, 9, 10, 11, 12, 13, 14, 18}) s.keys |= 1ULL << k;
    } else {
      fail(CG_POLICY_REJECTED, "invalid Kafka APIRole :\"" + role + "\"");
    }
  }
  if (!ver.empty()) {
    // strconv.ParseInt(ver, 10, 16)
    size_t i = 0;
    bool neg = false;
    if (ver[0] == '+' || ver[0] == '-') {
      neg = ver[0] == '-';
      i = 1;
    }
    if (i >= ver.size()) fail(CG_POLICY_REJECTED, "invalid Kafka APIVersion :\"" + ver + "\"");
    long v = 0;
    for (; i < ver.size(); ++i) {
      if (ver[i] < '0' || ver[i] > '9') fail(CG_POLICY_REJECTED, "invalid Kafka APIVersion :\"" + ver + "\"");
      v = v * 10 + (ver[i] - '0');
      if (v > 40000) fail(CG_POLICY_REJECTED, "invalid Kafka APIVersion :\"" + ver + "\"");
    }
    if (neg) v = -v;
    if (v < -32768 || v > 32767) fail(CG_POLICY_REJECTED, "invalid Kafka APIVersion :\"" + ver + "\"");
    s.ver_wild = false;
    s.version = (int16_t)v;
  }
  if (!s.topic.empty()) {
    if (s.topic.size() > 255) fail(CG_POLICY_REJECTED, "kafka topic exceeds maximum len of 255");
    // KafkaTopicValidChar `^[a-zA-Z0-9\\._\\-]+$` (api/kafka.go:244): the Go raw
    // string's "\\" is a literal backslash inside the class.
    for (unsigned char c : s.topic) {
      bool ok = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '\\' ||
                c == '.' || c == '_' || c == '-';
      if (!ok) fail(CG_POLICY_REJECTED, "invalid Kafka Topic name \"" + s.topic + "\"");
    }
  }
  return s;
}

}  // namespace

std::shared_ptr<KafkaSnapshot> kafka_compile(const char* json, size_t len) {
  Json root = JsonParser(json, len).parse();
  if (root.type != Json::ARR) fail(CG_POLICY_REJECTED, "expected a list of Kafka redirects");
  auto snap = std::make_shared<KafkaSnapshot>();
  KafkaSnapshot& S = *snap;
  auto intern = [](std::unordered_map<std::string, uint32_t>& m, const std::string& s) -> uint32_t {
    auto it = m.find(s);
    if (it != m.end()) return it->second;
    uint32_t id = (uint32_t)m.size();
    m.emplace(s, id);
    return id;
  };
  std::map<std::vector<int>, uint32_t> group_ids;  // selector set → group
  std::vector<std::pair<uint64_t, uint32_t>> gh;
  uint32_t ri = 0;
  for (const Json& red : root.arr) {
    const Json* nm = red.get("name");
    if (!nm) fail(CG_POLICY_REJECTED, "Kafka redirect without name");
    if (!S.redirect_index.emplace(nm->as_str("name"), ri).second)
      fail(CG_POLICY_REJECTED, "duplicate Kafka redirect name");
    struct Sel {
      bool wildcard;
      std::set<uint32_t> ids;
      std::vector<RuleSpec> rules;
      bool has_rules;
    };
    std::vector<Sel> sels;
    if (const Json* ss = red.get("selectors")) {
      if (ss->type != Json::ARR) fail(CG_POLICY_REJECTED, "selectors must be a list");
      for (const Json& sj : ss->arr) {
        Sel sel;
        const Json* ids = sj.get("identities");
        sel.wildcard = !ids || ids->type == Json::NUL;
        if (!sel.wildcard) {
          if (ids->type != Json::ARR) fail(CG_POLICY_REJECTED, "identities must be a list or null");
          for (const Json& id : ids->arr) {
            uint64_t v = id.as_u64("identities");
            if (v <= 0xFFFFFFFFULL) sel.ids.insert((uint32_t)v);
          }
        }
        sel.has_rules = false;
        if (const Json* rs = sj.get("rules")) {
          if (rs->type != Json::ARR) fail(CG_POLICY_REJECTED, "rules must be a list");
          for (const Json& r : rs->arr) sel.rules.push_back(sanitize(r));
          sel.has_rules = !sel.rules.empty();
        }
        sels.push_back(std::move(sel));
      }
    }
    // Identity 0 resolves to no labels (kafka.go:121-128): wildcard selectors only.
    auto make_group = [&](const std::vector<int>& selset) -> uint32_t {
      auto it = group_ids.find(selset);
      // group ids are global; the selector indices are made global by
      // prefixing the redirect index
      if (it != group_ids.end()) return it->second;
      KafkaGroupDev g{};
      std::vector<RuleSpec> wr, tr;
      for (size_t i = 1; i < selset.size(); ++i)
        for (const auto& r : sels[selset[i]].rules) (r.topic.empty() ? wr : tr).push_back(r);
      g.any_rules = (wr.size() + tr.size()) > 0;
      auto dev_rule = [&](const RuleSpec& r) {
        KafkaRuleDev d{};
        d.keys = r.keys;
        d.flags = (r.key_wild ? kKfKeyWild : 0) | (r.ver_wild ? kKfVerWild : 0) |
                  (!r.client.empty() ? kKfHasClient : 0);
        d.version = r.version;
        d.client_id = r.client.empty() ? 0 : intern(S.client_ids, r.client);
        return d;
      };
      g.wild_off = (uint32_t)S.rules.size();
      for (const auto& r : wr) {
        S.rules.push_back(dev_rule(r));
        S.topic_of.push_back(0xFFFFFFFFu);
      }
      g.wild_cnt = (uint32_t)wr.size();
      std::vector<std::pair<uint32_t, KafkaRuleDev>> trd;
      for (const auto& r : tr) trd.push_back({intern(S.topic_ids, r.topic), dev_rule(r)});
      std::stable_sort(trd.begin(), trd.end(),
                       [](const auto& a, const auto& b) { return a.first < b.first; });
      g.tr_off = (uint32_t)S.rules.size();
      for (auto& [t, d] : trd) {
        S.rules.push_back(d);
        S.topic_of.push_back(t);
      }
      g.tr_cnt = (uint32_t)trd.size();
      uint32_t gid = (uint32_t)S.groups.size();
      S.groups.push_back(g);
      group_ids[selset] = gid;
      return gid;
    };
    std::vector<int> wild;
    wild.push_back(-(int)ri - 1);  // redirect tag keeps groups per redirect
    for (size_t i = 0; i < sels.size(); ++i)
      if (sels[i].wildcard) wild.push_back((int)i);
    S.dflt_group.push_back(make_group(wild));
    std::set<uint32_t> all_ids;
    for (const auto& s : sels)
      for (uint32_t id : s.ids) all_ids.insert(id);
    for (uint32_t id : all_ids) {
      if (id == 0) continue;
      std::vector<int> set{-(int)ri - 1};
      for (size_t i = 0; i < sels.size(); ++i)
        if (!sels[i].wildcard && sels[i].ids.count(id)) set.push_back((int)i);
      for (size_t i = 0; i < sels.size(); ++i)
        if (sels[i].wildcard) set.push_back((int)i);
      gh.push_back({((uint64_t)ri << 32) | id, make_group(set)});
    }
    ++ri;
  }
  uint32_t cap = next_pow2(std::max<size_t>(gh.size() * 2, 16));
  S.ghash_keys.assign(cap, ~0ULL);
  S.ghash_vals.assign(cap, 0);
  S.ghash_mask = cap - 1;
  for (auto [k, v] : gh) {
    uint32_t h = hash64to32(k) & S.ghash_mask;
    while (S.ghash_keys[h] != ~0ULL) h = (h + 1) & S.ghash_mask;
    S.ghash_keys[h] = k;
    S.ghash_vals[h] = v;
  }
  if (S.rules.empty()) {
    S.rules.push_back(KafkaRuleDev{});
    S.topic_of.push_back(0xFFFFFFFFu);
  }
  if (S.groups.empty()) S.groups.push_back(KafkaGroupDev{});
  if (S.dflt_group.empty()) S.dflt_group.push_back(0);
  return snap;
}

// isTopicAPIKey, pkg/kafka/policy.go:27-52
static inline bool is_topic_api_key(int k) {
  switch (k) {
    case 0: case 1: case 2: case 3: case 4: case 5: case 6: case 8: case 9:
    case 19: case 20: case 21: case 23: case 24: case 27: case 28: case 34: case 35: case 37:
      return true;
  }
  return false;
}

static inline bool rule_matches(const KafkaRuleDev& r, bool has_topic, const cg_kafka_request& q) {
  // ruleMatches, pkg/kafka/policy.go:144-195
  if (!(r.flags & kKfKeyWild)) {
    if (q.api_key < 0 || q.api_key >= 64 || !((r.keys >> q.api_key) & 1)) return false;
  }
  if (!(r.flags & kKfVerWild) && r.version != q.api_version) return false;
  bool has_client = r.flags & kKfHasClient;
  if (!has_topic && !has_client) return true;
  switch (q.kind) {
    case CG_KAFKA_K_TYPED: return !has_client || r.client_id == q.client_id;
    case CG_KAFKA_K_CONSUMER_METADATA: return true;
    default: return !(has_topic && is_topic_api_key(q.api_key));  // matchNonTopicRequests
  }
}

uint8_t kafka_eval_host(const KafkaSnapshot& s, const cg_kafka_request& q, const uint32_t* arena,
                        size_t arena_len) {
  if (q.policy >= s.dflt_group.size()) return 0;
  uint32_t g = s.dflt_group[q.policy];
  if (q.remote != 0) {
    uint64_t key = ((uint64_t)q.policy << 32) | q.remote;
    uint32_t h = hash64to32(key) & s.ghash_mask;
    while (s.ghash_keys[h] != ~0ULL) {
      if (s.ghash_keys[h] == key) {
        g = s.ghash_vals[h];
        break;
      }
      h = (h + 1) & s.ghash_mask;
    }
  }
  const KafkaGroupDev& G = s.groups[g];
  if (!G.any_rules) return 0;  // "No Kafka rules matching identity, rejecting"
  for (uint32_t i = 0; i < G.wild_cnt; ++i)
    if (rule_matches(s.rules[G.wild_off + i], false, q)) return 1;
  const uint32_t* topics = q.topic_ids;
  uint32_t nt = q.n_topics;
  if (nt > CG_KAFKA_MAX_TOPICS) {
    if ((size_t)q.topic_ids[0] + nt > arena_len) return 0;
    topics = arena + q.topic_ids[0];
  }
  if (nt == 0) {
    for (uint32_t i = 0; i < G.tr_cnt; ++i)
      if (rule_matches(s.rules[G.tr_off + i], true, q)) return 1;
    return 0;
  }
  for (uint32_t t = 0; t < nt; ++t) {
    uint32_t tid = topics[t];
    bool cov = false;
    for (uint32_t i = 0; i < G.tr_cnt && !cov; ++i)
      if (s.topic_of[G.tr_off + i] == tid && rule_matches(s.rules[G.tr_off + i], true, q)) cov = true;
    if (!cov) return 0;
  }
  return 1;
}

void KafkaSnapshot::upload(Engine& e) {
  if (!e.has_gpu()) return;
  e.set_device();
  d_rules.upload_vec(rules);
  d_topic_of.upload_vec(topic_of);
  d_groups.upload_vec(groups);
  d_ghk.upload_vec(ghash_keys);
  d_ghv.upload_vec(ghash_vals);
  d_dflt.upload_vec(dflt_group);
  d_counters.alloc(std::max<size_t>(dflt_group.size(), 1) * 2 * sizeof(uint64_t));
  d_counters.zero();
  dev.rules = d_rules.as<KafkaRuleDev>();
  dev.topic_of = d_topic_of.as<uint32_t>();
  dev.groups = d_groups.as<KafkaGroupDev>();
  dev.ghash_keys = d_ghk.as<unsigned long long>();
  dev.ghash_vals = d_ghv.as<uint32_t>();
  dev.ghash_mask = ghash_mask;
  dev.dflt_group = d_dflt.as<uint32_t>();
  dev.nredirects = (uint32_t)dflt_group.size();
  dev.counters = d_counters.as<unsigned long long>();
}

}  // namespace cg
