// lpm.h — PreFilter state: the four CIDR maps of
// pkg/datapath/prefilter/prefilter.go and the device LPM structures.
#pragma once

#include <array>
#include <memory>
#include <set>
#include <vector>

#include "dev_types.h"
#include "engine.h"

namespace cg {

struct CidrKey {
  uint8_t family;
  uint8_t plen;
  std::array<uint8_t, 16> net;  // masked to plen bits
  bool operator<(const CidrKey& o) const {
    if (family != o.family) return family < o.family;
    if (plen != o.plen) return plen < o.plen;
    return net < o.net;
  }
  bool operator==(const CidrKey& o) const { return family == o.family && plen == o.plen && net == o.net; }
};

struct PrefilterState {
  uint32_t config = CG_PF_FIX4 | CG_PF_FIX6;
  uint32_t max_lpm = 65536;
  uint32_t max_hash = 20u << 20;
  int64_t revision = 1;
  // map index as preFilterMapType (prefilter.go:33-37): 0 v4dyn, 1 v4fix, 2 v6dyn, 3 v6fix
  std::set<CidrKey> maps[4];
  std::vector<uint32_t> ep4;
  std::vector<std::array<uint8_t, 16>> ep6;
  bool dirty = true;

  bool enabled(int which) const;
  // device structures
  std::vector<uint32_t> top, top_rank, mid, leaf_base;
  std::vector<uint64_t> leaves;
  std::vector<uint64_t> v6_code;  // 16 bucket codes | mixed buckets before the word << 32
  std::vector<uint32_t> v6_mix;   // per mixed bucket: R << 4 | min(R - L, 15)
  std::vector<uint64_t> v6_iv;
  uint32_t v6_bits = 16;
  std::vector<uint32_t> ep4_keys;
  bool ep4_zero = false, ep6_zero = false;
  std::vector<uint64_t> ep6_keys;
  std::shared_ptr<DevMem> d_counters;  // {drop, pass}: kept across rebuilds
  std::shared_ptr<DevTables> tab;      // the published device tables (engine.h)
  LpmDev dev{};                        // view of tab; copy it together with tab
  bool v4_filter = false, v6_filter = false;

  void rebuild(Engine& e);
};

}  // namespace cg
