// l4.h — policy map state (host mirror + device cuckoo table).
#pragma once

#include <memory>
#include <unordered_map>
#include <vector>

#include "dev_types.h"
#include "engine.h"

namespace cg {

inline uint64_t l4_key(const cg_policy_key& k) {
  return (uint64_t)k.sec_label | ((uint64_t)k.dport << 32) | ((uint64_t)k.protocol << 48) |
         ((uint64_t)k.egress << 56);
}
inline cg_policy_key l4_unkey(uint64_t v) {
  cg_policy_key k;
  k.sec_label = (uint32_t)v;
  k.dport = (uint16_t)(v >> 32);
  k.protocol = (uint8_t)(v >> 48);
  k.egress = (uint8_t)(v >> 56);
  return k;
}

struct PolicyMapState {
  uint32_t max_entries = 16384;
  struct Entry {
    uint16_t proxy_port_be;
    uint32_t id;  // counter slot
  };
  std::unordered_map<uint64_t, Entry> entries;  // insertion-ordered dump via `order`
  std::vector<uint64_t> order;                  // keys in insertion order
  std::vector<uint32_t> free_ids;
  uint32_t next_id = 0;
  bool dirty = true;

  // device
  std::vector<L4Slot> slots;
  std::vector<uint32_t> fp;  // per bucket: 4 x 8-bit slot fingerprints
  uint32_t bucket_mask = 0;
  std::shared_ptr<DevMem> d_counters;  // [id] packets, bytes: kept across rebuilds
  std::shared_ptr<DevTables> tab;      // the published device tables (engine.h)
  L4Dev dev{};                         // view of tab; copy it together with tab
  std::vector<uint64_t> host_counters;  // for handles without a GPU (always 0)

  void rebuild(Engine& e);  // cuckoo build + upload (counters preserved by id)
  void read_counters(Engine& e, uint32_t id, uint64_t* pk, uint64_t* by);
  void zero_counter(Engine& e, uint32_t id);
};

}  // namespace cg
