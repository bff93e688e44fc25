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
// device evaluation computes exactly that, from per-group decision summaries
// (dev_types.h KafkaSumDev): the topic-less half of the rule set becomes a few
// bit tests per request instead of a loop over every rule of the group.
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

// isTopicAPIKey, pkg/kafka/policy.go:27-52
inline bool is_topic_api_key(int k) {
  switch (k) {
    case 0: case 1: case 2: case 3: case 4: case 5: case 6: case 8: case 9:
    case 19: case 20: case 21: case 23: case 24: case 27: case 28: case 34: case 35: case 37:
      return true;
  }
  return false;
}

inline bool rule_matches(const KafkaRuleDev& r, const cg_kafka_request& q) {
  // ruleMatches, pkg/kafka/policy.go:144-195
  const bool has_topic = r.flags & kKfHasTopic;
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

uint32_t intern(std::unordered_map<std::string, uint32_t>& m, const std::string& s) {
  auto it = m.find(s);
  if (it != m.end()) return it->second;
  uint32_t id = (uint32_t)m.size();
  m.emplace(s, id);
  return id;
}

// Fold one rule into the summaries of one context (65 buckets).  `xs` collects
// the exception rules per bucket.  Per request class the rule's ruleMatches
// outcome (given key and version match) is fixed, except for a typed request
// against a clientID rule, which needs the comparison.
using ClientMap = std::map<uint64_t, KafkaClientDev>;

void fold_rule(KafkaSumDev* sums, uint32_t sum_base, std::vector<std::vector<KafkaRuleDev>>& xs, ClientMap& cm,
               const KafkaRuleDev& d) {
  const bool has_topic = d.flags & kKfHasTopic, has_client = d.flags & kKfHasClient;
  for (uint32_t b = 0; b < kKfBuckets; ++b) {
    if (!(d.flags & kKfKeyWild) && (b == 64 || !((d.keys >> b) & 1))) continue;
    bool exception = false;
    for (int c = 0; c < 3; ++c) {
      // class 0 typed, 1 consumer-metadata, 2 nil (ruleMatches switch)
      bool match = true, needs_client = false;
      if (has_topic || has_client) {
        if (c == 0) needs_client = has_client;
        else if (c == 2) match = !(has_topic && b < 64 && is_topic_api_key((int)b));
      }
      if (!match) continue;
      if (needs_client) {
        if (!(d.flags & kKfVerWild) && (d.version < 0 || d.version >= 64)) {
          exception = true;
          continue;
        }
        const uint64_t key = ((uint64_t)(sum_base + b) << 32) | d.client_id;
        KafkaClientDev& e = cm.emplace(key, KafkaClientDev{key, 0, 0, {0, 0, 0}}).first->second;
        if (d.flags & kKfVerWild) e.any = 1;
        else e.vm |= 1ULL << d.version;
        sums[b].any |= kKfSumHasClients;
      } else if (d.flags & kKfVerWild) {
        sums[b].any |= 1u << c;
      } else if (d.version >= 0 && d.version < 64) {
        sums[b].vm[c] |= 1ULL << d.version;
      } else {
        exception = true;
      }
    }
    if (exception) xs[b].push_back(d);
  }
}

KafkaRuleDev dev_rule(KafkaSnapshot& S, const RuleSpec& r) {
  KafkaRuleDev d{};
  d.keys = r.keys;
  d.flags = (r.key_wild ? kKfKeyWild : 0) | (r.ver_wild ? kKfVerWild : 0) | (!r.client.empty() ? kKfHasClient : 0) |
            (!r.topic.empty() ? kKfHasTopic : 0);
  d.version = r.version;
  d.client_id = r.client.empty() ? 0 : intern(S.client_ids, r.client);
  return d;
}

// One identity group's rules (GetRelevantRules result) → its 130 summaries,
// exception rules and (group, topic) rule lists.
void add_group(KafkaSnapshot& S, uint32_t gid, const std::vector<RuleSpec>& rs,
               std::vector<KafkaTopicDev>& tentries, ClientMap& cm) {
  S.sums.resize((size_t)(gid + 1) * kKfSumsPerGroup, KafkaSumDev{});
  KafkaSumDev* sums = S.sums.data() + (size_t)gid * kKfSumsPerGroup;
  std::vector<std::vector<KafkaRuleDev>> xs[2] = {std::vector<std::vector<KafkaRuleDev>>(kKfBuckets),
                                                  std::vector<std::vector<KafkaRuleDev>>(kKfBuckets)};
  std::map<uint32_t, std::vector<KafkaRuleDev>> by_topic;
  for (const auto& r : rs) {
    KafkaRuleDev d = dev_rule(S, r);
    // request without topics: every rule is tried (MatchesRule, policy.go:211)
    const uint32_t base = gid * kKfSumsPerGroup;
    fold_rule(sums + kKfBuckets, base + kKfBuckets, xs[1], cm, d);
    if (r.topic.empty()) fold_rule(sums, base, xs[0], cm, d);
    else by_topic[intern(S.topic_ids, r.topic)].push_back(d);
  }
  for (int ctx = 0; ctx < 2; ++ctx)
    for (uint32_t b = 0; b < kKfBuckets; ++b) {
      KafkaSumDev& su = sums[ctx * kKfBuckets + b];
      su.x_off = (uint32_t)S.rules.size();
      su.x_cnt = (uint32_t)xs[ctx][b].size();
      S.rules.insert(S.rules.end(), xs[ctx][b].begin(), xs[ctx][b].end());
    }
  for (auto& [t, v] : by_topic) {
    tentries.push_back(KafkaTopicDev{((uint64_t)gid << 32) | t, (uint32_t)S.rules.size(), (uint32_t)v.size()});
    S.rules.insert(S.rules.end(), v.begin(), v.end());
  }
}

}  // namespace

namespace {

void build_dict(const std::unordered_map<std::string, uint32_t>& m, std::vector<uint32_t>* slots,
                std::vector<uint8_t>* blob, uint32_t* mask) {
  uint32_t cap = 16;
  while (cap < 2 * m.size()) cap <<= 1;
  *mask = cap - 1;
  constexpr uint32_t W = kKfDictSlotWords;
  slots->assign((size_t)cap * W, 0);
  for (uint32_t i = 0; i < cap; ++i) (*slots)[i * W + 1] = kKfDictEmpty;
  blob->clear();
  for (const auto& [str, id] : m) {
    const uint8_t* p = (const uint8_t*)str.data();
    const uint32_t h = kf_fnv1a(p, (uint32_t)str.size());
    uint32_t s = h & *mask;
    while ((*slots)[s * W + 1] != kKfDictEmpty) s = (s + 1) & *mask;
    uint32_t* e = slots->data() + (size_t)s * W;
    e[0] = h;
    e[1] = (uint32_t)str.size();
    e[2] = id;
    e[3] = (uint32_t)blob->size();
    for (size_t k = 0; k < str.size() && k < 16; ++k) e[4 + k / 4] |= (uint32_t)p[k] << (8 * (k % 4));
    if (str.size() > 16) blob->insert(blob->end(), p + 16, p + str.size());
  }
  if (blob->empty()) blob->push_back(0);
}

}  // namespace

std::shared_ptr<KafkaSnapshot> kafka_compile(const char* json, size_t len) {
  Json root = JsonParser(json, len).parse();
  if (root.type != Json::ARR) fail(CG_POLICY_REJECTED, "expected a list of Kafka redirects");
  auto snap = std::make_shared<KafkaSnapshot>();
  KafkaSnapshot& S = *snap;
  std::map<std::vector<int>, uint32_t> group_ids;  // selector set → group
  std::vector<std::pair<uint64_t, uint32_t>> gh;
  std::vector<KafkaTopicDev> tentries;
  ClientMap cmap;
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
      std::vector<RuleSpec> rs;
      for (size_t i = 1; i < selset.size(); ++i)
        for (const auto& r : sels[selset[i]].rules) rs.push_back(r);
      const uint32_t gid = S.ngroups++;
      add_group(S, gid, rs, tentries, cmap);
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
  uint32_t cap = next_pow2(std::max<size_t>(gh.size() * 4, 16));  // load <= 1/4: ~1.1 probes
  S.ghash.assign(cap, KafkaGroupSlot{~0ULL, 0, 0});
  S.ghash_mask = cap - 1;
  for (auto [k, v] : gh) {
    uint32_t h = kf_hash(k) & S.ghash_mask;
    while (S.ghash[h].key != ~0ULL) h = (h + 1) & S.ghash_mask;
    S.ghash[h] = KafkaGroupSlot{k, v, 0};
  }
  cap = next_pow2(std::max<size_t>(cmap.size() * 4, 16));
  S.chash.assign(cap, KafkaClientDev{~0ULL, 0, 0, {0, 0, 0}});
  S.chash_mask = cap - 1;
  for (const auto& [k, e] : cmap) {
    uint32_t h = kf_hash(k) & S.chash_mask;
    while (S.chash[h].key != ~0ULL) h = (h + 1) & S.chash_mask;
    S.chash[h] = e;
  }
  cap = next_pow2(std::max<size_t>(tentries.size() * 4, 16));
  S.thash.assign(cap, KafkaTopicDev{~0ULL, 0, 0});
  S.thash_mask = cap - 1;
  for (const auto& t : tentries) {
    uint32_t h = kf_hash(t.key) & S.thash_mask;
    while (S.thash[h].key != ~0ULL) h = (h + 1) & S.thash_mask;
    S.thash[h] = t;
  }
  if (S.rules.empty()) S.rules.push_back(KafkaRuleDev{});
  if (S.ngroups == 0) {
    S.sums.assign(kKfSumsPerGroup, KafkaSumDev{});
    S.ngroups = 1;
  }
  if (S.dflt_group.empty()) S.dflt_group.push_back(0);
  for (int w = 0; w < 2; ++w) build_dict(w == 0 ? S.topic_ids : S.client_ids, &S.dict_slots[w], &S.dict_blob[w],
                                        &S.dict_mask[w]);
  return snap;
}

// Mirrors kafka_kernel (kernels.hip) step for step, so the compiler can be
// checked against the oracle without a GPU.
uint8_t kafka_eval_host(const KafkaSnapshot& s, const cg_kafka_request& q, const uint32_t* arena,
                        size_t arena_len) {
  if (q.policy >= s.dflt_group.size()) return 0;
  uint32_t g = s.dflt_group[q.policy];
  if (q.remote != 0) {
    uint64_t key = ((uint64_t)q.policy << 32) | q.remote;
    uint32_t h = kf_hash(key) & s.ghash_mask;
    while (s.ghash[h].key != ~0ULL) {
      if (s.ghash[h].key == key) {
        g = s.ghash[h].group;
        break;
      }
      h = (h + 1) & s.ghash_mask;
    }
  }
  const uint32_t nt = q.n_topics;
  const uint32_t b = (q.api_key >= 0 && q.api_key < 64) ? (uint32_t)q.api_key : 64;
  const uint32_t si = g * kKfSumsPerGroup + (nt == 0 ? kKfBuckets : 0) + b;
  const KafkaSumDev& su = s.sums[si];
  const int c = q.kind == CG_KAFKA_K_TYPED ? 0 : q.kind == CG_KAFKA_K_CONSUMER_METADATA ? 1 : 2;
  const bool vin = q.api_version >= 0 && q.api_version < 64;
  if ((su.any >> c) & 1) return 1;
  if (vin && ((su.vm[c] >> q.api_version) & 1)) return 1;
  if (c == 0 && (su.any & kKfSumHasClients)) {
    const uint64_t key = ((uint64_t)si << 32) | q.client_id;
    uint32_t h = kf_hash(key) & s.chash_mask;
    while (s.chash[h].key != ~0ULL) {
      if (s.chash[h].key == key) {
        if (s.chash[h].any || (vin && ((s.chash[h].vm >> q.api_version) & 1))) return 1;
        break;
      }
      h = (h + 1) & s.chash_mask;
    }
  }
  for (uint32_t i = 0; i < su.x_cnt; ++i)
    if (rule_matches(s.rules[su.x_off + i], q)) return 1;
  if (nt == 0) return 0;
  const uint32_t* topics = q.topic_ids;
  uint32_t ntot = nt;
  if (nt > CG_KAFKA_MAX_TOPICS) {
    if (nt == CG_KAFKA_TOPICS_IN_ARENA) ntot = q.topic_ids[1];
    if ((size_t)q.topic_ids[0] + ntot > arena_len) return 0;
    topics = arena + q.topic_ids[0];
  }
  for (uint32_t t = 0; t < ntot; ++t) {
    const uint64_t key = ((uint64_t)g << 32) | topics[t];
    uint32_t h = kf_hash(key) & s.thash_mask;
    bool cov = false;
    while (s.thash[h].key != ~0ULL) {
      if (s.thash[h].key == key) {
        for (uint32_t i = 0; i < s.thash[h].cnt && !cov; ++i)
          cov = rule_matches(s.rules[s.thash[h].off + i], q);
        break;
      }
      h = (h + 1) & s.thash_mask;
    }
    if (!cov) return 0;
  }
  return 1;
}

void KafkaSnapshot::upload(Engine& e) {
  if (!e.has_gpu()) return;
  e.set_device();
  d_rules.upload_vec(rules);
  d_sums.upload_vec(sums);
  d_thash.upload_vec(thash);
  d_chash.upload_vec(chash);
  d_ghash.upload_vec(ghash);
  d_dflt.upload_vec(dflt_group);
  d_counters.alloc(std::max<size_t>(dflt_group.size(), 1) * 2 * sizeof(uint64_t));
  d_counters.zero();
  dev.sums = d_sums.as<KafkaSumDev>();
  dev.rules = d_rules.as<KafkaRuleDev>();
  dev.thash = d_thash.as<KafkaTopicDev>();
  dev.thash_mask = thash_mask;
  dev.chash = d_chash.as<KafkaClientDev>();
  dev.chash_mask = chash_mask;
  dev.ghash = d_ghash.as<KafkaGroupSlot>();
  dev.ghash_mask = ghash_mask;
  dev.dflt_group = d_dflt.as<uint32_t>();
  dev.nredirects = (uint32_t)dflt_group.size();
  dev.counters = d_counters.as<unsigned long long>();
  for (int w = 0; w < 2; ++w) {
    d_dslots[w].upload_vec(dict_slots[w]);
    d_dblob[w].upload_vec(dict_blob[w]);
    ddict[w] = KafkaDictDev{d_dslots[w].as<uint32_t>(), d_dblob[w].as<uint8_t>(), dict_mask[w], 0};
  }
}

}  // namespace cg
