// ipcache.h — the IP → security-identity map (cilium_ipcache,
// bpf/lib/maps.h:135-159; Go side pkg/maps/ipcache/ipcache.go:36-130) and its
// device longest-prefix structures (dev_types.h IpcacheDev).
#pragma once

#include <map>
#include <memory>
#include <vector>

#include "dev_types.h"
#include "engine.h"
#include "lpm.h"

namespace cg {

struct IpcacheState {
  uint32_t max_entries = 512000;  // ipcache.go:36 MaxEntries, node_config.h:61
  // key {family, prefixlen, masked address} → RemoteEndpointInfo {sec_label, tunnel_endpoint}
  std::map<CidrKey, IpcVal> entries;
  bool dirty = true;

  // host copies of the device tables (also walked by cg_diag_ipcache_eval_host)
  std::vector<uint64_t> l16, chunks, runs6, code6;  // l16: the /16 level while building
  std::vector<uint32_t> l16x, ent6;
  std::vector<uint8_t> crowd6;
  std::vector<uint32_t> ex4;  // exact /32 slots (dev_types.h IpcacheDev)
  std::vector<uint64_t> ex6;  // exact /128 slots
  uint32_t ex4_mask = 0, ex6_mask = 0, ex4_probes = 0, ex6_probes = 0;
  uint32_t v6_bits = 16;
  std::shared_ptr<DevTables> tab;  // the published device tables (engine.h)
  IpcacheDev dev{};                // view of tab; copy it together with tab

  void build_tables();
  IpcacheDev host_view() const;
  void rebuild(Engine& e);
};

}  // namespace cg
