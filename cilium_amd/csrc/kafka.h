// kafka.h — Kafka L7 policy snapshot (per-redirect L7DataMap rule sets).
#pragma once

#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "dev_types.h"
#include "engine.h"

namespace cg {

struct KafkaSnapshot {
  std::map<std::string, uint32_t> redirect_index;
  std::unordered_map<std::string, uint32_t> topic_ids, client_ids;
  std::vector<KafkaRuleDev> rules;   // exception rules and topic rules
  std::vector<KafkaSumDev> sums;     // kKfSumsPerGroup per group
  std::vector<KafkaTopicDev> thash;
  uint32_t thash_mask = 0;
  uint32_t ngroups = 0;
  std::vector<KafkaClientDev> chash;
  uint32_t chash_mask = 0;
  std::vector<KafkaGroupSlot> ghash;
  uint32_t ghash_mask = 0;
  std::vector<uint32_t> dflt_group;

  DevMem d_rules, d_sums, d_thash, d_chash, d_ghash, d_dflt, d_counters;
  KafkaDev dev{};
  void upload(Engine& e);
};

std::shared_ptr<KafkaSnapshot> kafka_compile(const char* json, size_t len);
uint8_t kafka_eval_host(const KafkaSnapshot& s, const cg_kafka_request& r, const uint32_t* arena,
                        size_t arena_len);

}  // namespace cg
