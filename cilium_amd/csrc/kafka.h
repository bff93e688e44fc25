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

  // device dictionaries of the rule strings (0 topics, 1 clientIDs)
  std::vector<uint32_t> dict_slots[2];  // kKfDictSlotWords u32 per slot (KafkaDictDev)
  std::vector<uint8_t> dict_blob[2];
  uint32_t dict_mask[2] = {0, 0};

  DevMem d_rules, d_sums, d_thash, d_chash, d_ghash, d_dflt, d_counters, d_dslots[2], d_dblob[2];
  KafkaDev dev{};
  KafkaDictDev ddict[2] = {};
  LaunchFence fence;  // last member: queued kernels finish before the buffers go (engine.h)
  void upload(Engine& e);
};

std::shared_ptr<KafkaSnapshot> kafka_compile(const char* json, size_t len);
// Decode one request's bytes on the host (kafka_wire.cc): the record,
// topics beyond CG_KAFKA_MAX_TOPICS appended to *spill (record offset
// relative to spill's start); returns CG_KAFKA_DECODE_OK / _ERROR.
uint8_t kafka_decode_host_one(const KafkaSnapshot& s, const uint8_t* raw, uint64_t len, uint16_t redirect,
                              uint32_t remote, cg_kafka_request* q, std::vector<uint32_t>* spill);
uint8_t kafka_eval_host(const KafkaSnapshot& s, const cg_kafka_request& r, const uint32_t* arena,
                        size_t arena_len);

}  // namespace cg
