// capi.cc — the extern "C" boundary (include/cilium_gpu.h).  Every entry
// point catches internal errors and returns a cg_result code.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <exception>
#include <chrono>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "engine.h"
#include "http.h"
#include "kafka.h"
#include "kafka_wire.h"
#include "kernels.h"
#include "l4.h"
#include "ipcache.h"
#include "lpm.h"
#include "regex.h"
#include "ring.h"

using namespace cg;

namespace {

std::mutex g_handles_mu;
std::map<uint64_t, std::shared_ptr<Engine>> g_handles;
uint64_t g_next_handle = 1;
// Bumped (after the change is published) by everything that changes what a
// ring call resolves to: cg_close, ring open / close, an HTTP policy publish.
// cg_http_ring_verdicts keeps its handle, ring and snapshot per calling thread
// while this is unchanged, so Envoy's workers take no lock and touch no
// shared reference count per request.
std::atomic<uint64_t> g_epoch{1};
void bump_epoch() { g_epoch.fetch_add(1, std::memory_order_acq_rel); }

std::shared_ptr<Engine> get(uint64_t h) {
  std::lock_guard<std::mutex> lk(g_handles_mu);
  auto it = g_handles.find(h);
  if (it == g_handles.end()) fail(CG_INVALID_INSTANCE, "unknown handle");
  return it->second;
}

template <class F>
int guarded(F&& f) {
  try {
    f();
    return CG_OK;
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("out of host memory");
    return CG_UNKNOWN_ERROR;
  } catch (const std::exception& e) {
    set_error(e.what());
    return CG_UNKNOWN_ERROR;
  } catch (...) {
    set_error("unknown error");
    return CG_UNKNOWN_ERROR;
  }
}

PolicyMapState& get_map(Engine& e, uint32_t id) {
  auto it = e.maps.find(id);
  if (it == e.maps.end()) fail(CG_NOT_FOUND, "unknown policy map id");
  return *it->second;
}

IpcacheState& get_ipc(Engine& e, uint32_t id) {
  auto it = e.ipcaches.find(id);
  if (it == e.ipcaches.end()) fail(CG_NOT_FOUND, "unknown ipcache id");
  return *it->second;
}

PrefilterState& get_pf(Engine& e, uint32_t id) {
  auto it = e.prefilters.find(id);
  if (it == e.prefilters.end()) fail(CG_NOT_FOUND, "unknown prefilter id");
  return *it->second;
}

void* stream_of(Engine& e, void* s) { return s ? s : e.stream; }

void check_launch(int err, const char* what) { hip_check(err, what); }

// A queued launch on `stream` reads this table set: record it on the set's
// retirement fence (engine.h LaunchFence).
void fence(const std::shared_ptr<DevTables>& t, void* stream) {
  if (t) t->fence.record(stream);
}

CidrKey make_cidr(const cg_cidr& c) {
  CidrKey k;
  if (c.family != 4 && c.family != 6) fail(CG_INVALID_ADDRESS, "cidr family must be 4 or 6");
  int bits = c.family == 4 ? 32 : 128;
  if (c.prefixlen > bits) fail(CG_INVALID_ADDRESS, "prefix length out of range");
  k.family = c.family;
  k.plen = c.prefixlen;
  k.net.fill(0);
  int bytes = bits / 8;
  for (int i = 0; i < bytes; ++i) {
    int keep = std::max(0, std::min(8, (int)c.prefixlen - 8 * i));
    uint8_t mask = keep == 0 ? 0 : (uint8_t)(0xFF << (8 - keep));
    k.net[i] = c.addr[i] & mask;  // net.ParseCIDR returns the masked network
  }
  return k;
}

// selectMap (prefilter.go:108-122)
int select_map(const CidrKey& k) {
  if (k.family == 4) return k.plen == 32 ? 1 : 0;
  return k.plen == 128 ? 3 : 2;
}

}  // namespace

extern "C" {

const char* cg_last_error(void) { return get_error().c_str(); }

const char* cg_version(void) { return "libciliumgpu gfx950 r1"; }

uint64_t cg_open(const cg_kv* params, size_t n, uint8_t debug) {
  uint64_t out = 0;
  int rc = guarded([&] {
    auto e = std::make_shared<Engine>();
    e->debug = debug;
    int dev = 0;
    for (size_t i = 0; i < n; ++i)
      if (params[i].key && params[i].value && strcmp(params[i].key, "device") == 0) dev = atoi(params[i].value);
    e->device = dev;
    if (dev >= 0) {
      int count = 0;
      if (hipGetDeviceCount(&count) != hipSuccess || dev >= count)
        fail(CG_NO_DEVICE, "no HIP device " + std::to_string(dev));
      hipDeviceProp_t prop;
      hip_check(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
      if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        fail(CG_NO_DEVICE, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950 only");
      e->cus = prop.multiProcessorCount;
      hip_check(hipSetDevice(dev), "hipSetDevice");
      hipStream_t s;
      hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
      e->stream = s;
    }
    std::lock_guard<std::mutex> lk(g_handles_mu);
    out = g_next_handle++;
    g_handles[out] = e;
  });
  return rc == CG_OK ? out : 0;
}

void cg_close(uint64_t h) {
  std::shared_ptr<Engine> e;
  {
    std::lock_guard<std::mutex> lk(g_handles_mu);
    auto it = g_handles.find(h);
    if (it == g_handles.end()) return;
    e = it->second;
    g_handles.erase(it);
  }
  bump_epoch();
  if (e->has_gpu()) {
    (void)hipSetDevice(e->device);
    {
      std::shared_ptr<HttpRing> r;
      {
        std::lock_guard<std::mutex> lk(e->ring_mu);
        r = std::move(e->ring);
      }
      if (r) r->close();
    }
    (void)hipStreamSynchronize((hipStream_t)e->stream);
    e->maps.clear();
    e->prefilters.clear();
    e->ipcaches.clear();
    e->http.reset();
    e->kafka.reset();
    (void)hipStreamDestroy((hipStream_t)e->stream);
  }
}

int cg_sync(uint64_t h) {
  return guarded([&] {
    auto e = get(h);
    if (e->has_gpu()) dev_sync(*e, nullptr);
  });
}

// ------------------------------------------------------------------ L4 ----
int cg_policymap_create(uint64_t h, uint32_t max_entries, uint32_t* map_id) {
  return guarded([&] {
    auto e = get(h);
    if (!map_id) fail(CG_INVALID_ARGUMENT, "map_id is NULL");
    if (max_entries == 0) max_entries = 16384;  // policymap.go:37 MaxEntries
    if (max_entries > 65536) fail(CG_INVALID_ARGUMENT, "max_entries > 65536");
    std::lock_guard<std::mutex> lk(e->mu);
    auto m = std::make_unique<PolicyMapState>();
    m->max_entries = max_entries;
    uint32_t id = e->next_id++;
    e->maps[id] = std::move(m);
    *map_id = id;
  });
}

int cg_policymap_destroy(uint64_t h, uint32_t map_id) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    get_map(*e, map_id);
    if (e->has_gpu()) dev_sync(*e, nullptr);
    e->maps.erase(map_id);
  });
}

int cg_policymap_allow(uint64_t h, uint32_t map_id, const cg_policy_key* keys, const uint16_t* ports_be,
                       size_t n) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PolicyMapState& m = get_map(*e, map_id);
    if (n && (!keys || !ports_be)) fail(CG_INVALID_ARGUMENT, "NULL keys/ports");
    size_t fresh = 0;
    std::map<uint64_t, int> seen;
    for (size_t i = 0; i < n; ++i) {
      uint64_t k = l4_key(keys[i]);
      if (k == kL4EmptyKey) fail(CG_INVALID_ARGUMENT, "reserved all-ones policy key");
      if (!m.entries.count(k) && seen.emplace(k, 1).second) ++fresh;
    }
    if (m.entries.size() + fresh > m.max_entries) fail(CG_MAP_FULL, "policy map full (E2BIG)");
    for (size_t i = 0; i < n; ++i) {
      uint64_t k = l4_key(keys[i]);
      auto it = m.entries.find(k);
      if (it != m.entries.end()) {
        it->second.proxy_port_be = ports_be[i];
      } else {
        uint32_t id;
        if (!m.free_ids.empty()) {
          id = m.free_ids.back();
          m.free_ids.pop_back();
        } else {
          id = m.next_id++;
        }
        m.zero_counter(*e, id);
        m.entries[k] = {ports_be[i], id};
        m.order.push_back(k);
      }
    }
    m.dirty = true;
  });
}

int cg_policymap_delete(uint64_t h, uint32_t map_id, const cg_policy_key* keys, size_t n) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PolicyMapState& m = get_map(*e, map_id);
    for (size_t i = 0; i < n; ++i)
      if (!m.entries.count(l4_key(keys[i]))) fail(CG_NOT_FOUND, "policy key not found (ENOENT)");
    for (size_t i = 0; i < n; ++i) {
      uint64_t k = l4_key(keys[i]);
      auto it = m.entries.find(k);
      if (it == m.entries.end()) continue;  // duplicate in the batch
      m.free_ids.push_back(it->second.id);
      m.entries.erase(it);
      m.order.erase(std::find(m.order.begin(), m.order.end(), k));
    }
    m.dirty = true;
  });
}

int cg_policymap_lookup(uint64_t h, uint32_t map_id, const cg_policy_key* key, cg_policy_entry* entry) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PolicyMapState& m = get_map(*e, map_id);
    auto it = m.entries.find(l4_key(*key));
    if (it == m.entries.end()) fail(CG_NOT_FOUND, "policy key not found");
    if (entry) {
      memset(entry, 0, sizeof(*entry));
      entry->proxy_port = it->second.proxy_port_be;
      // counters include every verdict call queued on this device so far
      if (e->has_gpu()) {
        e->set_device();
        hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      }
      m.read_counters(*e, it->second.id, &entry->packets, &entry->bytes);
    }
  });
}

int cg_policymap_dump(uint64_t h, uint32_t map_id, cg_policy_key* keys, cg_policy_entry* entries, size_t cap,
                      size_t* n) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PolicyMapState& m = get_map(*e, map_id);
    if (n) *n = m.order.size();
    std::vector<uint64_t> ctr;
    if (e->has_gpu() && m.d_counters) {
      e->set_device();
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      ctr.resize((size_t)m.max_entries * 2);
      hip_check(hipMemcpy(ctr.data(), m.d_counters->get(), ctr.size() * 8, hipMemcpyDeviceToHost), "D2H counters");
    }
    size_t i = 0;
    for (uint64_t k : m.order) {
      if (i >= cap) break;
      if (keys) keys[i] = l4_unkey(k);
      if (entries) {
        memset(&entries[i], 0, sizeof(cg_policy_entry));
        const auto& en = m.entries[k];
        entries[i].proxy_port = en.proxy_port_be;
        if (!ctr.empty()) {
          entries[i].packets = ctr[(size_t)en.id * 2];
          entries[i].bytes = ctr[(size_t)en.id * 2 + 1];
        }
      }
      ++i;
    }
  });
}

int cg_policymap_flush(uint64_t h, uint32_t map_id) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PolicyMapState& m = get_map(*e, map_id);
    for (auto& [k, en] : m.entries) m.free_ids.push_back(en.id);
    m.entries.clear();
    m.order.clear();
    m.dirty = true;
  });
}

// A map's published tables, copied under the handle lock and held while the
// launch is enqueued (engine.h DevTables).
struct L4View {
  std::shared_ptr<DevTables> keep;
  L4Dev dev;
};
static L4View l4_view(Engine& e, uint32_t map_id) {
  std::lock_guard<std::mutex> lk(e.mu);
  PolicyMapState& m = get_map(e, map_id);
  if (m.dirty) m.rebuild(e);
  return {m.tab, m.dev};
}
struct IpcView {
  std::shared_ptr<DevTables> keep;
  IpcacheDev dev;
};
static IpcView ipc_view(Engine& e, uint32_t ipc_id) {
  std::lock_guard<std::mutex> lk(e.mu);
  IpcacheState& p = get_ipc(e, ipc_id);
  if (p.dirty) p.rebuild(e);
  return {p.tab, p.dev};
}

static uint32_t check_l4_mode(uint32_t mode) {
  if ((mode & ~(3u | CG_L4_IGNORE_DROP)) || (mode & 3u) == 3u) fail(CG_INVALID_ARGUMENT, "unknown L4 verdict mode");
  return mode;
}

static void l4_dev(Engine& e, uint32_t map_id, uint32_t mode, const cg_l4_tuple* d_t, size_t n, int32_t* d_out,
                   void* s) {
  e.require_gpu();
  const L4View v = l4_view(e, map_id);
  e.set_device();
  check_launch(launch_l4(v.dev, d_t, n, d_out, mode, stream_of(e, s), e.cus), "l4 kernel launch");
  fence(v.keep, stream_of(e, s));
}

static void l4_host(Engine& e, uint32_t map_id, uint32_t mode, const cg_l4_tuple* t, size_t n, int32_t* out) {
  e.require_gpu();
  if (n && (!t || !out)) fail(CG_INVALID_ARGUMENT, "NULL tuples/verdicts");
  const L4View v = l4_view(e, map_id);
  host_pipeline(e, n, {{t, sizeof(cg_l4_tuple)}}, {{out, sizeof(int32_t)}},
                [&](void* const* din, void* const* dout, size_t cnt, void* st) {
                  check_launch(launch_l4(v.dev, din[0], cnt, (int32_t*)dout[0], mode, st, e.cus), "l4 kernel launch");
                });
}

int cg_l4_verdicts_dev(uint64_t h, uint32_t map_id, const cg_l4_tuple* d_tuples, size_t n, int32_t* d_verdicts,
                       void* stream) {
  return guarded([&] { l4_dev(*get(h), map_id, CG_L4_CAN_ACCESS, d_tuples, n, d_verdicts, stream); });
}

int cg_l4_verdicts_host(uint64_t h, uint32_t map_id, const cg_l4_tuple* tuples, size_t n, int32_t* verdicts) {
  return guarded([&] { l4_host(*get(h), map_id, CG_L4_CAN_ACCESS, tuples, n, verdicts); });
}

int cg_l4_policy_verdicts_dev(uint64_t h, uint32_t map_id, uint32_t mode, const cg_l4_tuple* d_tuples, size_t n,
                              int32_t* d_verdicts, void* stream) {
  return guarded([&] { l4_dev(*get(h), map_id, check_l4_mode(mode), d_tuples, n, d_verdicts, stream); });
}

int cg_l4_policy_verdicts_host(uint64_t h, uint32_t map_id, uint32_t mode, const cg_l4_tuple* tuples, size_t n,
                               int32_t* verdicts) {
  return guarded([&] { l4_host(*get(h), map_id, check_l4_mode(mode), tuples, n, verdicts); });
}

// The egress flow with identities from the ipcache (bpf_lxc.c:509-527 v4,
// :205-220 v6): policy_can_egress{4,6} semantics.
static void l4_ipc_dev(Engine& e, uint32_t map_id, uint32_t ipc_id, int family, const void* d_addr,
                       const cg_l4_tuple* d_t, size_t n, int32_t* d_out, void* s) {
  e.require_gpu();
  const L4View v = l4_view(e, map_id);
  const IpcView iv = ipc_view(e, ipc_id);
  e.set_device();
  check_launch(launch_l4_ipcache(v.dev, iv.dev, family, d_addr, d_t, n, d_out, CG_L4_EGRESS, stream_of(e, s), e.cus),
               "l4 (ipcache) kernel launch");
  fence(v.keep, stream_of(e, s));
  fence(iv.keep, stream_of(e, s));
}

static void l4_ipc_host(Engine& e, uint32_t map_id, uint32_t ipc_id, int family, const void* addr,
                        const cg_l4_tuple* t, size_t n, int32_t* out) {
  e.require_gpu();
  if (n && (!addr || !t || !out)) fail(CG_INVALID_ARGUMENT, "NULL addresses/tuples/verdicts");
  const L4View v = l4_view(e, map_id);
  const IpcView iv = ipc_view(e, ipc_id);
  host_pipeline(e, n, {{addr, family == 6 ? 16u : 4u}, {t, sizeof(cg_l4_tuple)}}, {{out, sizeof(int32_t)}},
                [&](void* const* din, void* const* dout, size_t cnt, void* st) {
                  check_launch(launch_l4_ipcache(v.dev, iv.dev, family, din[0], din[1], cnt, (int32_t*)dout[0],
                                                 CG_L4_EGRESS, st, e.cus),
                               "l4 (ipcache) kernel launch");
                });
}

int cg_l4_verdicts_ipcache_dev(uint64_t h, uint32_t map_id, uint32_t ipc_id, const uint32_t* d_remote_v4,
                               const cg_l4_tuple* d_tuples, size_t n, int32_t* d_verdicts, void* stream) {
  return guarded([&] { l4_ipc_dev(*get(h), map_id, ipc_id, 4, d_remote_v4, d_tuples, n, d_verdicts, stream); });
}

int cg_l4_verdicts_ipcache_host(uint64_t h, uint32_t map_id, uint32_t ipc_id, const uint32_t* remote_v4,
                                const cg_l4_tuple* tuples, size_t n, int32_t* verdicts) {
  return guarded([&] { l4_ipc_host(*get(h), map_id, ipc_id, 4, remote_v4, tuples, n, verdicts); });
}

int cg_l4_verdicts_ipcache6_dev(uint64_t h, uint32_t map_id, uint32_t ipc_id, const uint8_t* d_remote_v6,
                                const cg_l4_tuple* d_tuples, size_t n, int32_t* d_verdicts, void* stream) {
  return guarded([&] { l4_ipc_dev(*get(h), map_id, ipc_id, 6, d_remote_v6, d_tuples, n, d_verdicts, stream); });
}

int cg_l4_verdicts_ipcache6_host(uint64_t h, uint32_t map_id, uint32_t ipc_id, const uint8_t* remote_v6,
                                 const cg_l4_tuple* tuples, size_t n, int32_t* verdicts) {
  return guarded([&] { l4_ipc_host(*get(h), map_id, ipc_id, 6, remote_v6, tuples, n, verdicts); });
}

// ----------------------------------------------------------------- LPM ----
int cg_prefilter_create(uint64_t h, uint32_t config, uint32_t max_lpm, uint32_t max_hash, uint32_t* pf_id) {
  return guarded([&] {
    auto e = get(h);
    if (!pf_id) fail(CG_INVALID_ARGUMENT, "pf_id is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    auto p = std::make_unique<PrefilterState>();
    p->config = config;
    if (max_lpm) p->max_lpm = max_lpm;
    if (max_hash) p->max_hash = max_hash;
    uint32_t id = e->next_id++;
    e->prefilters[id] = std::move(p);
    *pf_id = id;
  });
}

int cg_prefilter_destroy(uint64_t h, uint32_t pf_id) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    get_pf(*e, pf_id);
    if (e->has_gpu()) dev_sync(*e, nullptr);
    e->prefilters.erase(pf_id);
  });
}

int cg_prefilter_insert(uint64_t h, uint32_t pf_id, int64_t revision, const cg_cidr* cidrs, size_t n,
                        int64_t* revision_out) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PrefilterState& p = get_pf(*e, pf_id);
    if (revision != 0 && p.revision != revision)
      fail(CG_REVISION_MISMATCH,
           "Latest revision is " + std::to_string(p.revision) + " not " + std::to_string(revision));
    std::vector<std::pair<int, CidrKey>> undo;
    int err = 0;
    std::string msg;
    for (size_t i = 0; i < n && !err; ++i) {
      CidrKey k = make_cidr(cidrs[i]);
      int which = select_map(k);
      if (!p.enabled(which)) {
        err = CG_NO_MAP;
        msg = "No map enabled for CIDR string";
        break;
      }
      uint32_t cap = (which == 0 || which == 2) ? p.max_lpm : p.max_hash;
      if (p.maps[which].count(k)) {
        // BPF_ANY update of an existing key succeeds, and Insert still queues
        // it for undo: a later failure deletes it (prefilter.go:141-158).
        undo.push_back({which, k});
        continue;
      }
      if (p.maps[which].size() >= cap) {
        err = CG_MAP_FULL;
        msg = "Error inserting CIDR string: map full";
        break;
      }
      p.maps[which].insert(k);
      undo.push_back({which, k});
    }
    if (err) {
      for (auto& [w, k] : undo) p.maps[w].erase(k);
      fail(err, msg);
    }
    p.revision++;
    p.dirty = true;
    if (revision_out) *revision_out = p.revision;
  });
}

int cg_prefilter_delete(uint64_t h, uint32_t pf_id, int64_t revision, const cg_cidr* cidrs, size_t n,
                        int64_t* revision_out) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PrefilterState& p = get_pf(*e, pf_id);
    if (revision != 0 && p.revision != revision)
      fail(CG_REVISION_MISMATCH,
           "Latest revision is " + std::to_string(p.revision) + " not " + std::to_string(revision));
    std::vector<CidrKey> ks;
    for (size_t i = 0; i < n; ++i) {
      CidrKey k = make_cidr(cidrs[i]);
      int which = select_map(k);
      if (!p.enabled(which)) fail(CG_NO_MAP, "No map enabled for CIDR string");
      if (!p.maps[which].count(k)) fail(CG_NOT_FOUND, "No map entry for CIDR string");
      ks.push_back(k);
    }
    for (auto& k : ks) p.maps[select_map(k)].erase(k);
    p.revision++;
    p.dirty = true;
    if (revision_out) *revision_out = p.revision;
  });
}

int cg_prefilter_dump(uint64_t h, uint32_t pf_id, cg_cidr* out, size_t cap, size_t* n, int64_t* revision) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PrefilterState& p = get_pf(*e, pf_id);
    size_t i = 0, total = 0;
    for (int w = 0; w < 4; ++w) {  // prefixesV4Dyn .. prefixesV6Fix order (prefilter.go:102)
      for (const auto& k : p.maps[w]) {
        if (out && i < cap) {
          memset(&out[i], 0, sizeof(cg_cidr));
          out[i].family = k.family;
          out[i].prefixlen = k.plen;
          memcpy(out[i].addr, k.net.data(), 16);
          ++i;
        }
        ++total;
      }
    }
    if (n) *n = total;
    if (revision) *revision = p.revision;
  });
}

int cg_prefilter_set_endpoints(uint64_t h, uint32_t pf_id, const uint32_t* v4, size_t n4, const uint8_t* v6,
                               size_t n6) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PrefilterState& p = get_pf(*e, pf_id);
    p.ep4.assign(v4, v4 + n4);
    p.ep6.resize(n6);
    for (size_t i = 0; i < n6; ++i) memcpy(p.ep6[i].data(), v6 + 16 * i, 16);
    p.dirty = true;
  });
}

struct LpmView {
  std::shared_ptr<DevTables> keep;
  LpmDev dev;
  bool v4f, v6f;
};
static LpmView lpm_view(Engine& e, uint32_t pf_id) {
  std::lock_guard<std::mutex> lk(e.mu);
  PrefilterState& p = get_pf(e, pf_id);
  if (p.dirty) p.rebuild(e);
  return {p.tab, p.dev, p.v4_filter, p.v6_filter};
}

int cg_prefilter_verdicts_dev(uint64_t h, uint32_t pf_id, const uint32_t* d_v4, size_t n4, uint8_t* d_out4,
                              const uint8_t* d_v6, size_t n6, uint8_t* d_out6, void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    const LpmView v = lpm_view(*e, pf_id);
    e->set_device();
    check_launch(launch_lpm(v.dev, v.v4f, v.v6f, d_v4, n4, d_out4, d_v6, n6, d_out6, stream_of(*e, stream), e->cus),
                 "lpm kernel launch");
    fence(v.keep, stream_of(*e, stream));
  });
}

int cg_prefilter_verdicts_host(uint64_t h, uint32_t pf_id, const uint32_t* v4, size_t n4, uint8_t* out4,
                               const uint8_t* v6, size_t n6, uint8_t* out6) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    if ((n4 && (!v4 || !out4)) || (n6 && (!v6 || !out6))) fail(CG_INVALID_ARGUMENT, "NULL address/verdict arrays");
    const LpmView v = lpm_view(*e, pf_id);
    host_pipeline(*e, n4, {{v4, 8}}, {{out4, 1}}, [&](void* const* din, void* const* dout, size_t cnt, void* st) {
      check_launch(launch_lpm(v.dev, v.v4f, v.v6f, (const uint32_t*)din[0], cnt, (uint8_t*)dout[0], nullptr, 0,
                              nullptr, st, e->cus),
                   "lpm kernel launch");
    });
    host_pipeline(*e, n6, {{v6, 32}}, {{out6, 1}}, [&](void* const* din, void* const* dout, size_t cnt, void* st) {
      check_launch(launch_lpm(v.dev, v.v4f, v.v6f, nullptr, 0, nullptr, (const uint8_t*)din[0], cnt,
                              (uint8_t*)dout[0], st, e->cus),
                   "lpm kernel launch");
    });
  });
}

// ------------------------------------------------------------- ipcache ----
int cg_ipcache_create(uint64_t h, uint32_t max_entries, uint32_t* ipc_id) {
  return guarded([&] {
    auto e = get(h);
    if (!ipc_id) fail(CG_INVALID_ARGUMENT, "ipc_id is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    auto p = std::make_unique<IpcacheState>();
    if (max_entries) p->max_entries = max_entries;
    uint32_t id = e->next_id++;
    e->ipcaches[id] = std::move(p);
    *ipc_id = id;
  });
}

int cg_ipcache_destroy(uint64_t h, uint32_t ipc_id) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    get_ipc(*e, ipc_id);
    if (e->has_gpu()) dev_sync(*e, nullptr);
    e->ipcaches.erase(ipc_id);
  });
}

int cg_ipcache_update(uint64_t h, uint32_t ipc_id, const cg_cidr* keys, const cg_remote_endpoint_info* values,
                      size_t n) {
  return guarded([&] {
    auto e = get(h);
    if (n && (!keys || !values)) fail(CG_INVALID_ARGUMENT, "NULL keys/values");
    std::lock_guard<std::mutex> lk(e->mu);
    IpcacheState& p = get_ipc(*e, ipc_id);
    std::map<CidrKey, IpcVal> batch;
    for (size_t i = 0; i < n; ++i) batch[make_cidr(keys[i])] = IpcVal{values[i].sec_label, values[i].tunnel_endpoint};
    size_t fresh = 0;
    for (const auto& kv : batch) fresh += !p.entries.count(kv.first);
    if (p.entries.size() + fresh > p.max_entries) fail(CG_MAP_FULL, "ipcache: map full (max_entries)");
    // a key given twice in one batch keeps its last value, as sequential updates would
    for (size_t i = 0; i < n; ++i) p.entries[make_cidr(keys[i])] = IpcVal{values[i].sec_label, values[i].tunnel_endpoint};
    p.dirty = true;
  });
}

int cg_ipcache_delete(uint64_t h, uint32_t ipc_id, const cg_cidr* keys, size_t n) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    IpcacheState& p = get_ipc(*e, ipc_id);
    std::vector<CidrKey> ks;
    for (size_t i = 0; i < n; ++i) {
      CidrKey k = make_cidr(keys[i]);
      if (!p.entries.count(k)) fail(CG_NOT_FOUND, "ipcache: no entry for key");
      ks.push_back(k);
    }
    for (auto& k : ks) p.entries.erase(k);
    p.dirty = true;
  });
}

int cg_ipcache_lookup(uint64_t h, uint32_t ipc_id, const cg_cidr* key, cg_remote_endpoint_info* value) {
  return guarded([&] {
    auto e = get(h);
    if (!key || !value) fail(CG_INVALID_ARGUMENT, "NULL key/value");
    std::lock_guard<std::mutex> lk(e->mu);
    IpcacheState& p = get_ipc(*e, ipc_id);
    auto it = p.entries.find(make_cidr(*key));
    if (it == p.entries.end()) fail(CG_NOT_FOUND, "ipcache: no entry for key");
    value->sec_label = it->second.identity;
    value->tunnel_endpoint = it->second.tunnel;
  });
}

int cg_ipcache_dump(uint64_t h, uint32_t ipc_id, cg_cidr* keys, cg_remote_endpoint_info* values, size_t cap,
                    size_t* n) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    IpcacheState& p = get_ipc(*e, ipc_id);
    size_t i = 0;
    for (const auto& [k, v] : p.entries) {
      if (i >= cap) break;
      if (keys) {
        memset(&keys[i], 0, sizeof(cg_cidr));
        keys[i].family = k.family;
        keys[i].prefixlen = k.plen;
        memcpy(keys[i].addr, k.net.data(), 16);
      }
      if (values) values[i] = cg_remote_endpoint_info{v.identity, v.tunnel};
      ++i;
    }
    if (n) *n = p.entries.size();
  });
}

int cg_ipcache_resolve_dev(uint64_t h, uint32_t ipc_id, const uint32_t* d_v4, size_t n4,
                           cg_remote_endpoint_info* d_out4, const uint8_t* d_v6, size_t n6,
                           cg_remote_endpoint_info* d_out6, void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    const IpcView v = ipc_view(*e, ipc_id);
    e->set_device();
    check_launch(launch_ipcache(v.dev, d_v4, n4, (IpcVal*)d_out4, d_v6, n6, (IpcVal*)d_out6, stream_of(*e, stream),
                                e->cus),
                 "ipcache kernel launch");
    fence(v.keep, stream_of(*e, stream));
  });
}

int cg_ipcache_resolve_host(uint64_t h, uint32_t ipc_id, const uint32_t* v4, size_t n4,
                            cg_remote_endpoint_info* out4, const uint8_t* v6, size_t n6,
                            cg_remote_endpoint_info* out6) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    if ((n4 && (!v4 || !out4)) || (n6 && (!v6 || !out6))) fail(CG_INVALID_ARGUMENT, "NULL address/result arrays");
    const IpcView v = ipc_view(*e, ipc_id);
    host_pipeline(*e, n4, {{v4, 4}}, {{out4, 8}}, [&](void* const* din, void* const* dout, size_t cnt, void* st) {
      check_launch(launch_ipcache(v.dev, (const uint32_t*)din[0], cnt, (IpcVal*)dout[0], nullptr, 0, nullptr, st,
                                  e->cus),
                   "ipcache kernel launch");
    });
    host_pipeline(*e, n6, {{v6, 16}}, {{out6, 8}}, [&](void* const* din, void* const* dout, size_t cnt, void* st) {
      check_launch(launch_ipcache(v.dev, nullptr, 0, nullptr, (const uint8_t*)din[0], cnt, (IpcVal*)dout[0], st,
                                  e->cus),
                   "ipcache kernel launch");
    });
  });
}

// The ipcache tables walked on the host exactly as ipcache_kernel does.
int cg_diag_ipcache_eval_host(uint64_t h, uint32_t ipc_id, const uint32_t* v4, size_t n4,
                              cg_remote_endpoint_info* out4, const uint8_t* v6, size_t n6,
                              cg_remote_endpoint_info* out6) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    IpcacheState& p = get_ipc(*e, ipc_id);
    if (p.dirty) p.rebuild(*e);
    const IpcacheDev t = p.host_view();
    for (size_t i = 0; i < n4; ++i) {
      const uint64_t v = ipc_v4_value(t, __builtin_bswap32(v4[i]));
      out4[i] = cg_remote_endpoint_info{(uint32_t)v, (uint32_t)(v >> 32)};
    }
    for (size_t i = 0; i < n6; ++i) {
      uint64_t hi = 0, lo = 0;
      for (int k = 0; k < 8; ++k) hi = hi << 8 | v6[16 * i + k];
      for (int k = 8; k < 16; ++k) lo = lo << 8 | v6[16 * i + k];
      const uint32_t tb = (uint32_t)(hi >> (64 - t.v6_bits));
      uint32_t k, L, R;
      uint64_t v = kIpcMiss;
      if (ipc_v6_bucket(t.code6[tb >> 5], tb, &k)) {
        L = t.ent6[4 * (size_t)k];
        R = t.ent6[4 * (size_t)k + 1];
        const uint32_t crowd = t.ent6[4 * (size_t)k + 2];
        uint64_t xv;
        if (t.ent6[4 * (size_t)k + 3] && ipc_ex6_find(t, hi, lo, ipc_ex6_hash(hi, lo) & t.ex6_mask, &xv)) {
          v = xv;  // a /128 entry
        } else {
          v = t.runs6[4 * (size_t)R + 2];
          if (!ipc_le128(t.runs6[4 * (size_t)R], t.runs6[4 * (size_t)R + 1], hi, lo))
            v = ipc_v6_search_value(t, hi, lo, L, R, crowd);
        }
      }
      out6[i] = cg_remote_endpoint_info{(uint32_t)v, (uint32_t)(v >> 32)};
    }
  });
}

// ---------------------------------------------------------------- HTTP ----
int cg_http_policy_update(uint64_t h, const char* json, size_t len) {
  return guarded([&] {
    auto e = get(h);
    if (!json) fail(CG_INVALID_ARGUMENT, "NULL policy");
    std::shared_ptr<HttpSnapshot> snap = http_compile(json, len);
    if (e->has_gpu()) {
      e->set_device();
      snap->upload(*e);
    }
    {
      std::lock_guard<std::mutex> lk(e->mu);
      e->http = snap;  // publish
    }
    bump_epoch();
  });
}

int cg_http_policy_update_npds(uint64_t h, const uint8_t* resp, size_t len) {
  std::string json;
  const int rc = guarded([&] {
    if (!resp && len) fail(CG_INVALID_ARGUMENT, "NULL DiscoveryResponse");
    json = npds_pb_to_json(resp, len, true);  // Envoy: proto3 strings must be UTF-8
  });
  if (rc != CG_OK) return rc;
  return cg_http_policy_update(h, json.data(), json.size());
}

static std::shared_ptr<HttpSnapshot> http_snap(Engine& e);

int cg_http_policy_export(uint64_t h, void* buf, size_t cap, size_t* len) {
  return guarded([&] {
    auto e = get(h);
    const std::vector<uint8_t> img = http_image_export(*http_snap(*e));
    if (len) *len = img.size();
    if (buf && cap >= img.size()) memcpy(buf, img.data(), img.size());
    else if (buf) fail(CG_INVALID_ARGUMENT, "policy image buffer too small");
  });
}

int cg_http_policy_import(uint64_t h, const void* buf, size_t len) {
  return guarded([&] {
    auto e = get(h);
    std::shared_ptr<HttpSnapshot> snap = http_image_import(static_cast<const uint8_t*>(buf), len);
    if (e->has_gpu()) {
      e->set_device();
      snap->upload(*e);
    }
    {
      std::lock_guard<std::mutex> lk(e->mu);
      e->http = snap;  // publish
    }
    bump_epoch();
  });
}

static std::shared_ptr<HttpSnapshot> http_snap(Engine& e) {
  std::lock_guard<std::mutex> lk(e.mu);
  if (!e.http) fail(CG_NOT_FOUND, "no HTTP policy installed");
  return e.http;
}

int cg_http_policy_index(uint64_t h, const char* name, uint32_t* index) {
  return guarded([&] {
    auto e = get(h);
    auto s = http_snap(*e);
    auto it = s->policy_index.find(name ? name : "");
    if (it == s->policy_index.end()) fail(CG_NOT_FOUND, "no policy named " + std::string(name ? name : ""));
    *index = it->second;
  });
}

int cg_http_rule_info_get(uint64_t h, cg_http_rule_info* out, size_t cap, size_t* n) {
  return guarded([&] {
    auto e = get(h);
    auto s = http_snap(*e);
    if (n) *n = s->rule_info.size();
    if (out) memcpy(out, s->rule_info.data(), std::min(cap, s->rule_info.size()) * sizeof(cg_http_rule_info));
  });
}

int cg_http_policy_stats(uint64_t h, uint64_t* out, size_t n) {
  return guarded([&] {
    auto e = get(h);
    auto s = http_snap(*e);
    uint64_t max_prog_cells = 0, lds_progs = 0;
    for (const auto& pg : s->progs) {
      if (pg.flags & kProgAllowAll) continue;
      max_prog_cells = std::max<uint64_t>(max_prog_cells, pg.cell_count);
      lds_progs += (pg.flags & kProgRebased) && pg.cell_count <= kMaxLdsCells;
    }
    uint64_t v[12] = {s->progs.size(),
                     s->parts.size(),
                     s->total_states,
                     s->cells.size() * 4,
                     s->fields.size(),
                     s->total_rules,
                     s->npolicies,
                     s->total_remote_slots,
                     s->total_exceptions,
                     s->cells.size(),
                     max_prog_cells,
                     lds_progs};
    for (size_t i = 0; i < n && i < 12; ++i) out[i] = v[i];
  });
}

size_t cg_http_batch_bytes(uint64_t h, size_t n) {
  size_t v = 0;
  guarded([&] {
    auto e = get(h);
    v = http_batch_bytes(*http_snap(*e), n);
  });
  return v;
}

size_t cg_http_batch_slots(uint64_t h, size_t n) {
  size_t v = 0;
  guarded([&] {
    auto e = get(h);
    v = http_batch_slots(*http_snap(*e), n);
  });
  return v;
}

int cg_http_pack(uint64_t h, size_t n, const uint32_t* policy, const uint8_t* ingress, const uint16_t* port,
                 const uint32_t* remote, const uint8_t* hdr_blob, const uint64_t* hdr_off, void* batch,
                 size_t batch_cap, uint32_t* order, size_t* nslots, uint8_t* arena, size_t arena_cap,
                 size_t* arena_used) {
  return guarded([&] {
    auto e = get(h);
    auto s = http_snap(*e);
    http_pack(*s, n, policy, ingress, port, remote, hdr_blob, hdr_off, batch, batch_cap, order, nslots, arena,
              arena_cap, arena_used);
  });
}

static size_t batch_used_bytes(const void* batch) {
  HttpBatchHeader hdr;
  memcpy(&hdr, batch, sizeof(hdr));
  if (hdr.magic != kBatchMagic) fail(CG_INVALID_ARGUMENT, "not a packed HTTP batch");
  return hdr.total_bytes;
}

int cg_http_verdicts_dev(uint64_t h, const void* d_batch, size_t nslots, const uint8_t* d_arena, uint8_t* d_out,
                         void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = http_snap(*e);
    e->set_device();
    check_launch(launch_http(s->dev, d_batch, nslots, d_arena, d_out, stream_of(*e, stream), e->cus),
                 "http kernel launch");
    s->fence.record(stream_of(*e, stream));
  });
}

int cg_http_verdicts_rules_dev(uint64_t h, const void* d_batch, size_t nslots, const uint8_t* d_arena, uint8_t* d_out,
                               uint32_t* d_rule, void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = http_snap(*e);
    if (nslots && !d_rule) fail(CG_INVALID_ARGUMENT, "NULL rule array");
    e->set_device();
    check_launch(launch_http(s->dev, d_batch, nslots, d_arena, d_out, stream_of(*e, stream), e->cus, nullptr, d_rule),
                 "http kernel launch");
    s->fence.record(stream_of(*e, stream));
  });
}

int cg_http_verdicts_raw_dev(uint64_t h, const uint8_t* d_raw, const uint64_t* d_raw_off, size_t n,
                             const uint32_t* d_policy, const uint8_t* d_ingress, const uint16_t* d_port,
                             const uint32_t* d_remote, uint8_t* d_out, void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = http_snap(*e);
    if (n && (!d_raw_off || !d_policy || !d_ingress || !d_port || !d_remote || !d_out))
      fail(CG_INVALID_ARGUMENT, "NULL device array");
    e->set_device();
    auto lease = e->staging.acquire(e->device);
    http_verdicts_raw_on(*s, *lease, e->cus, RawInput::Heads, d_raw, d_raw_off, n, d_policy, d_ingress, d_port,
                         d_remote, d_out, stream_of(*e, stream));
    // the device-layout sequence returns with its kernels still queued on
    // the stream, reading the snapshot's tables: keep the snapshot alive
    s->fence.record(stream_of(*e, stream));
    // no stream given: the handle's, waited for (a caller that wants the
    // call asynchronous names its stream)
    if (!stream) hip_check(hipStreamSynchronize((hipStream_t)stream_of(*e, stream)), "hipStreamSynchronize");
  });
}

int cg_http_verdicts_fields_dev(uint64_t h, const uint8_t* d_hdr_blob, const uint64_t* d_hdr_off, size_t n,
                                const uint32_t* d_policy, const uint8_t* d_ingress, const uint16_t* d_port,
                                const uint32_t* d_remote, uint8_t* d_out, void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = http_snap(*e);
    if (n && (!d_hdr_off || !d_policy || !d_ingress || !d_port || !d_remote || !d_out))
      fail(CG_INVALID_ARGUMENT, "NULL device array");
    e->set_device();
    auto lease = e->staging.acquire(e->device);
    http_verdicts_raw_on(*s, *lease, e->cus, RawInput::Lists, d_hdr_blob, d_hdr_off, n, d_policy, d_ingress, d_port,
                         d_remote, d_out, stream_of(*e, stream));
    s->fence.record(stream_of(*e, stream));  // as cg_http_verdicts_raw_dev
    if (!stream) hip_check(hipStreamSynchronize((hipStream_t)stream_of(*e, stream)), "hipStreamSynchronize");
  });
}

// Copy a host array into the lease's pinned buffer i and DMA it to its
// device buffer i (async on the lease's stream).
static void* stage_in(StagingSlot& sl, int i, const void* src, size_t bytes) {
  void* d = sl.dev_buf(i, bytes);
  if (!bytes) return d;
  void* hb = sl.host_buf(i, bytes);
  memcpy(hb, src, bytes);
  hip_check(hipMemcpyAsync(d, hb, bytes, hipMemcpyHostToDevice, (hipStream_t)sl.stream), "H2D");
  return d;
}

static void http_verdicts_host_impl(uint64_t h, const void* batch, size_t nslots, const uint32_t* order,
                                    size_t n, const uint8_t* arena, size_t arena_len, uint8_t* out, uint32_t* rule);

int cg_http_verdicts_host(uint64_t h, const void* batch, size_t nslots, const uint32_t* order, size_t n,
                          const uint8_t* arena, size_t arena_len, uint8_t* out) {
  return guarded([&] { http_verdicts_host_impl(h, batch, nslots, order, n, arena, arena_len, out, nullptr); });
}

int cg_http_verdicts_rules_host(uint64_t h, const void* batch, size_t nslots, const uint32_t* order, size_t n,
                                const uint8_t* arena, size_t arena_len, uint8_t* out, uint32_t* rule) {
  return guarded([&] {
    if (n && !rule) fail(CG_INVALID_ARGUMENT, "NULL rule array");
    http_verdicts_host_impl(h, batch, nslots, order, n, arena, arena_len, out, rule);
  });
}

static void http_verdicts_host_impl(uint64_t h, const void* batch, size_t nslots, const uint32_t* order,
                                    size_t n, const uint8_t* arena, size_t arena_len, uint8_t* out, uint32_t* rule) {
  {
    auto e = get(h);
    e->require_gpu();
    auto s = http_snap(*e);
    if (!batch || (n && (!order || !out))) fail(CG_INVALID_ARGUMENT, "NULL batch/order/out");
    HttpBatchHeader hdr;
    memcpy(&hdr, batch, sizeof(hdr));
    if (hdr.magic != kBatchMagic || hdr.epoch != s->epoch)
      fail(CG_INVALID_ARGUMENT, "batch was packed against another policy snapshot");
    if (hdr.nslots != nslots) fail(CG_INVALID_ARGUMENT, "nslots differs from the packed batch");
    if (hdr.arena_bytes && (!arena || arena_len < hdr.arena_bytes))
      fail(CG_INVALID_ARGUMENT, "overflow arena shorter than the packed batch needs");
    e->set_device();
    auto lease = e->staging.acquire(e->device);
    void* dr = stage_in(*lease, 0, batch, batch_used_bytes(batch));
    void* da = stage_in(*lease, 1, arena, hdr.arena_bytes);
    void* dout = lease->dev_buf(2, nslots + 1);
    uint32_t* drule = rule ? (uint32_t*)lease->dev_buf(3, (nslots + 1) * 4) : nullptr;
    check_launch(launch_http(s->dev, dr, nslots, (const uint8_t*)da, (uint8_t*)dout, lease->stream, e->cus, nullptr,
                             drule),
                 "http kernel launch");
    uint8_t* slots = (uint8_t*)lease->host_buf(2, nslots + 1);
    uint32_t* rslots = rule ? (uint32_t*)lease->host_buf(3, (nslots + 1) * 4) : nullptr;
    if (nslots)
      hip_check(hipMemcpyAsync(slots, dout, nslots, hipMemcpyDeviceToHost, (hipStream_t)lease->stream), "D2H");
    if (nslots && rule)
      hip_check(hipMemcpyAsync(rslots, drule, nslots * 4, hipMemcpyDeviceToHost, (hipStream_t)lease->stream), "D2H");
    hip_check(hipStreamSynchronize((hipStream_t)lease->stream), "hipStreamSynchronize");
    for (size_t i = 0; i < nslots; ++i)
      if (order[i] < n) {
        out[order[i]] = slots[i];
        if (rule) rule[order[i]] = rslots[i];
      }
  }
}

// --------------------------------------------------------------- Kafka ----
int cg_kafka_policy_update(uint64_t h, const char* json, size_t len) {
  return guarded([&] {
    auto e = get(h);
    if (!json) fail(CG_INVALID_ARGUMENT, "NULL policy");
    auto snap = kafka_compile(json, len);
    if (e->has_gpu()) {
      e->set_device();
      snap->upload(*e);
    }
    std::lock_guard<std::mutex> lk(e->mu);
    e->kafka = snap;
  });
}

static std::shared_ptr<KafkaSnapshot> kafka_snap(Engine& e) {
  std::lock_guard<std::mutex> lk(e.mu);
  if (!e.kafka) fail(CG_NOT_FOUND, "no Kafka policy installed");
  return e.kafka;
}

int cg_kafka_policy_index(uint64_t h, const char* name, uint32_t* index) {
  return guarded([&] {
    auto e = get(h);
    auto s = kafka_snap(*e);
    auto it = s->redirect_index.find(name ? name : "");
    if (it == s->redirect_index.end()) fail(CG_NOT_FOUND, "no Kafka redirect named " + std::string(name ? name : ""));
    *index = it->second;
  });
}

int cg_kafka_intern(uint64_t h, uint32_t what, const char* str, size_t len, uint32_t* id) {
  return guarded([&] {
    auto e = get(h);
    auto s = kafka_snap(*e);
    const auto& m = what == 0 ? s->topic_ids : s->client_ids;
    auto it = m.find(std::string(str ? str : "", len));
    *id = it == m.end() ? CG_KAFKA_UNKNOWN_STR : it->second;
  });
}

int cg_kafka_verdicts_dev(uint64_t h, const cg_kafka_request* d_reqs, size_t n, const uint32_t* d_arena,
                          uint8_t* d_out, void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = kafka_snap(*e);
    e->set_device();
    check_launch(launch_kafka(s->dev, d_reqs, n, d_arena, d_out, stream_of(*e, stream), e->cus),
                 "kafka kernel launch");
    s->fence.record(stream_of(*e, stream));
  });
}

int cg_kafka_verdicts_split_dev(uint64_t h, const cg_kafka_request_head* d_heads, const uint32_t* d_topics,
                                size_t n, const uint32_t* d_arena, uint8_t* d_out, void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = kafka_snap(*e);
    if (n && (!d_heads || !d_topics || !d_out)) fail(CG_INVALID_ARGUMENT, "NULL heads/topics/out");
    e->set_device();
    check_launch(launch_kafka(s->dev, d_heads, n, d_arena, d_out, stream_of(*e, stream), e->cus, d_topics),
                 "kafka kernel launch");
    s->fence.record(stream_of(*e, stream));
  });
}

int cg_kafka_verdicts_host(uint64_t h, const cg_kafka_request* reqs, size_t n, const uint32_t* arena,
                           size_t arena_len, uint8_t* out) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = kafka_snap(*e);
    if (n && (!reqs || !out)) fail(CG_INVALID_ARGUMENT, "NULL requests/out");
    e->set_device();
    // the topic arena is shared by every chunk: one copy on its own lease
    auto lease = e->staging.acquire(e->device);
    const uint32_t* da = (const uint32_t*)stage_in(*lease, 0, arena, arena ? arena_len * 4 : 0);
    hip_check(hipStreamSynchronize((hipStream_t)lease->stream), "hipStreamSynchronize");
    host_pipeline(*e, n, {{reqs, sizeof(cg_kafka_request)}}, {{out, 1}},
                  [&](void* const* din, void* const* dout, size_t cnt, void* st) {
                    check_launch(launch_kafka(s->dev, din[0], cnt, da, (uint8_t*)dout[0], st, e->cus),
                                 "kafka kernel launch");
                  });
  });
}

// ------------------------------------------------------- Kafka decode ----
// The GPU decode of n staged requests on `st`, then the host decode of the
// requests the device deferred (gzip / snappy message payloads): their bytes
// come back, kafka_decode_host_one rewrites their record and status, and
// their long topic lists go after the device's arena entries.  Returns the
// arena entries used (may exceed arena_cap: nothing written beyond it).
static size_t kafka_decode_on(Engine& e, const KafkaSnapshot& s, StagingSlot& sl, const uint8_t* d_raw,
                              const uint64_t* d_off, size_t n, const uint16_t* d_red, const uint32_t* d_rem,
                              cg_kafka_request* d_reqs, uint32_t* d_arena, size_t arena_cap, uint8_t* d_status,
                              hipStream_t st) {
  // counters: topic arena entries, requests the decode kernel deferred,
  // inflate bytes reserved, payloads inflated on the device, requests the
  // inflate kernel deferred (to the host), payloads it deferred without a
  // reservation (arena full, impossible size)
  auto* ctr = (unsigned long long*)sl.dev_buf(7, 48);
  hip_check(hipMemsetAsync(ctr, 0, 48, st), "hipMemsetAsync");
  // the decode kernel's deferred requests (compressed sets) and the
  // payloads' decoded bytes (grow-only; a payload past it goes to the host)
  auto* dlist = (uint32_t*)sl.dev_buf(28, n * 4);
  uint8_t* zarena = (uint8_t*)sl.dev_buf(27, kKafkaInflateArena);
  check_launch(launch_kafka_decode(s.ddict[0], s.ddict[1], d_raw, d_off, n, d_red, d_rem, d_reqs, d_arena,
                                   arena_cap, ctr, d_status, st, e.cus, dlist, zarena, kKafkaInflateArena),
               "kafka decode kernel launch");
  auto* hc = (unsigned long long*)sl.host_buf(7, 48);
  hip_check(hipMemcpyAsync(hc, ctr, 48, hipMemcpyDeviceToHost, st), "D2H");
  hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  size_t used = (size_t)hc[0];
  e.kafka_inflated.fetch_add(hc[3]);
  e.kafka_deferred.fetch_add(hc[4]);
  e.kafka_arena_full.fetch_add(hc[5]);
  if (hc[4] == 0) return used;
  std::vector<uint8_t> status(n);
  std::vector<uint64_t> off(n + 1);
  hip_check(hipMemcpy(status.data(), d_status, n, hipMemcpyDeviceToHost), "D2H");
  hip_check(hipMemcpy(off.data(), d_off, (n + 1) * 8, hipMemcpyDeviceToHost), "D2H");
  std::vector<uint8_t> bytes;
  std::vector<uint32_t> spill;
  for (size_t i = 0; i < n; ++i) {
    if (status[i] != 2) continue;  // kKwDefer
    const uint64_t len = off[i + 1] > off[i] ? off[i + 1] - off[i] : 0;
    bytes.resize(len);
    if (len) hip_check(hipMemcpy(bytes.data(), d_raw + off[i], len, hipMemcpyDeviceToHost), "D2H");
    cg_kafka_request q;
    hip_check(hipMemcpy(&q, d_reqs + i, sizeof(q), hipMemcpyDeviceToHost), "D2H");
    const size_t base = spill.size();
    const uint8_t rc = kafka_decode_host_one(s, bytes.data(), len, q.policy, q.remote, &q, &spill);
    if (rc == CG_KAFKA_DECODE_OK && q.n_topics > CG_KAFKA_MAX_TOPICS) q.topic_ids[0] = (uint32_t)(used + base);
    hip_check(hipMemcpy(d_reqs + i, &q, sizeof(q), hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_status + i, &rc, 1, hipMemcpyHostToDevice), "H2D");
  }
  if (!spill.empty() && used + spill.size() <= arena_cap)
    hip_check(hipMemcpy(d_arena + used, spill.data(), spill.size() * 4, hipMemcpyHostToDevice), "H2D");
  return used + spill.size();
}

static void check_offsets(const uint64_t* off, size_t n) {
  if (!off) fail(CG_INVALID_ARGUMENT, "NULL raw_off");
  for (size_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) fail(CG_INVALID_ARGUMENT, "raw_off must be non-decreasing");
}

int cg_kafka_decode_stats(uint64_t h, uint64_t* device_inflated, uint64_t* host_deferred) {
  return guarded([&] {
    auto e = get(h);
    if (device_inflated) *device_inflated = e->kafka_inflated.load();
    if (host_deferred) *host_deferred = e->kafka_deferred.load();
  });
}

int cg_kafka_inflate_stats(uint64_t h, uint64_t* unreserved) {
  return guarded([&] {
    auto e = get(h);
    if (unreserved) *unreserved = e->kafka_arena_full.load();
  });
}

int cg_kafka_decode_dev(uint64_t h, const uint8_t* d_raw, const uint64_t* d_raw_off, size_t n,
                        const uint16_t* d_redirect, const uint32_t* d_remote, cg_kafka_request* d_reqs,
                        uint32_t* d_arena, size_t arena_cap, size_t* arena_used, uint8_t* d_status, void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = kafka_snap(*e);
    if (!arena_used) fail(CG_INVALID_ARGUMENT, "NULL arena_used");
    *arena_used = 0;
    if (!n) return;
    e->set_device();
    auto lease = e->staging.acquire(e->device);
    const size_t used = kafka_decode_on(*e, *s, *lease, d_raw, d_raw_off, n, d_redirect, d_remote, d_reqs, d_arena,
                                        d_arena ? arena_cap : 0, d_status, (hipStream_t)stream_of(*e, stream));
    *arena_used = used;
    if (used > (d_arena ? arena_cap : 0)) fail(CG_MAP_FULL, "Kafka topic arena too small");
  });
}

// Stage raw requests, offsets, redirects and remotes on a lease (buffers
// 0..3) and decode them into lease buffers 4 (records), 5 (statuses), 6 (arena).
struct KafkaStaged {
  cg_kafka_request* reqs;
  uint8_t* status;
  uint32_t* arena;
  size_t used;
};
static KafkaStaged kafka_stage_decode(Engine& e, const KafkaSnapshot& s, StagingSlot& sl, const uint8_t* raw,
                                      const uint64_t* raw_off, size_t n, const uint16_t* redirect,
                                      const uint32_t* remote, size_t arena_cap) {
  check_offsets(raw_off, n);
  if (!redirect || !remote || (raw_off[n] && !raw)) fail(CG_INVALID_ARGUMENT, "NULL raw/redirect/remote");
  const auto st = (hipStream_t)sl.stream;
  const uint8_t* d_raw = (const uint8_t*)stage_in(sl, 0, raw, raw_off[n]);
  const uint64_t* d_off = (const uint64_t*)stage_in(sl, 1, raw_off, (n + 1) * 8);
  const uint16_t* d_red = (const uint16_t*)stage_in(sl, 2, redirect, n * 2);
  const uint32_t* d_rem = (const uint32_t*)stage_in(sl, 3, remote, n * 4);
  KafkaStaged k;
  k.reqs = (cg_kafka_request*)sl.dev_buf(4, n * sizeof(cg_kafka_request));
  k.status = (uint8_t*)sl.dev_buf(5, n);
  k.arena = (uint32_t*)sl.dev_buf(6, std::max<size_t>(arena_cap, 1) * 4);
  k.used = kafka_decode_on(e, s, sl, d_raw, d_off, n, d_red, d_rem, k.reqs, k.arena, arena_cap, k.status, st);
  return k;
}

int cg_kafka_decode_host(uint64_t h, const uint8_t* raw, const uint64_t* raw_off, size_t n, const uint16_t* redirect,
                         const uint32_t* remote, cg_kafka_request* reqs, uint32_t* arena, size_t arena_cap,
                         size_t* arena_used, uint8_t* status) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = kafka_snap(*e);
    if (!arena_used || (n && (!reqs || !status))) fail(CG_INVALID_ARGUMENT, "NULL reqs/status/arena_used");
    *arena_used = 0;
    if (!n) return;
    if (!arena) arena_cap = 0;
    e->set_device();
    auto lease = e->staging.acquire(e->device);
    const KafkaStaged k = kafka_stage_decode(*e, *s, *lease, raw, raw_off, n, redirect, remote, arena_cap);
    *arena_used = k.used;
    if (k.used > arena_cap) fail(CG_MAP_FULL, "Kafka topic arena too small");
    const auto st = (hipStream_t)lease->stream;
    hip_check(hipMemcpyAsync(reqs, k.reqs, n * sizeof(cg_kafka_request), hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipMemcpyAsync(status, k.status, n, hipMemcpyDeviceToHost, st), "D2H");
    if (k.used) hip_check(hipMemcpyAsync(arena, k.arena, k.used * 4, hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  });
}

int cg_kafka_verdicts_raw_host(uint64_t h, const uint8_t* raw, const uint64_t* raw_off, size_t n,
                               const uint16_t* redirect, const uint32_t* remote, uint8_t* out) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    auto s = kafka_snap(*e);
    if (n && !out) fail(CG_INVALID_ARGUMENT, "NULL out");
    if (!n) return;
    check_offsets(raw_off, n);
    e->set_device();
    auto lease = e->staging.acquire(e->device);
    // a request's topic list needs at least 2 bytes per topic
    const size_t cap = (size_t)(raw_off[n] - raw_off[0]) / 2 + 16;
    const KafkaStaged k = kafka_stage_decode(*e, *s, *lease, raw, raw_off, n, redirect, remote, cap);
    if (k.used > cap) fail(CG_UNKNOWN_ERROR, "Kafka topic arena bound exceeded");
    const auto st = (hipStream_t)lease->stream;
    uint8_t* d_v = (uint8_t*)lease->dev_buf(0, n + 16);  // the raw bytes are no longer needed
    check_launch(launch_kafka(s->dev, k.reqs, n, k.arena, d_v, st, e->cus), "kafka kernel launch");
    uint8_t* hv = (uint8_t*)lease->host_buf(4, 2 * n);
    hip_check(hipMemcpyAsync(hv, d_v, n, hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipMemcpyAsync(hv + n, k.status, n, hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
    for (size_t i = 0; i < n; ++i) out[i] = hv[n + i] == CG_KAFKA_DECODE_OK ? hv[i] : CG_KAFKA_V_CLOSE;
  });
}

// Requests from host memory through the device path.  A large call runs in
// chunks of ~kHostChunkBytes on two workers, each with its own lease
// (pinned buffers + stream): while one worker copies its chunk into pinned
// memory (several threads) the other's chunk is on the bus or the GPU.
// 32 MiB: 0.351 / 0.340 G requests/s on config 5's 8M header lists against
// 0.299 / 0.331 at 160 MiB and 0.280 / 0.262 at 16 (profiles/r05aa_host_chunks.txt)
constexpr size_t kHostChunkBytes = (size_t)32 << 20;

static void run_host_chunk(const HttpSnapshot& s, Engine& e, StagingSlot& sl, RawInput in, const uint8_t* raw,
                           const uint64_t* raw_off, size_t a, size_t b, const uint32_t* policy,
                           const uint8_t* ingress, const uint16_t* port, const uint32_t* remote, uint8_t* out,
                           unsigned copy_threads) {
  const size_t m = b - a;
  const uint64_t base = raw_off[a], bytes = raw_off[b] - base;
  const auto st = (hipStream_t)sl.stream;
  uint8_t* h_raw = (uint8_t*)sl.host_buf(0, bytes);
  uint64_t* h_off = (uint64_t*)sl.host_buf(1, (m + 1) * 8);
  uint32_t* h_pol = (uint32_t*)sl.host_buf(2, m * 4);
  uint8_t* h_ing = (uint8_t*)sl.host_buf(3, m);
  uint16_t* h_port = (uint16_t*)sl.host_buf(4, m * 2);
  uint32_t* h_rem = (uint32_t*)sl.host_buf(5, m * 4);
  // the copies, split over threads by request ranges
  auto copy = [&](size_t i0, size_t i1) {
    const uint64_t b0 = raw_off[a + i0] - base, b1 = raw_off[a + i1] - base;
    if (b1 > b0) memcpy(h_raw + b0, raw + base + b0, b1 - b0);
    for (size_t i = i0; i < i1; ++i) h_off[i] = raw_off[a + i] - base;  // rebased to the staged bytes
    memcpy(h_pol + i0, policy + a + i0, (i1 - i0) * 4);
    memcpy(h_ing + i0, ingress + a + i0, i1 - i0);
    memcpy(h_port + i0, port + a + i0, (i1 - i0) * 2);
    memcpy(h_rem + i0, remote + a + i0, (i1 - i0) * 4);
  };
  const unsigned nt = m < 65536 ? 1u : copy_threads;
  if (nt <= 1) {
    copy(0, m);
  } else {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back(copy, m * t / nt, m * (t + 1) / nt);
    for (auto& x : th) x.join();
  }
  h_off[m] = bytes;
  auto h2d = [&](int i, const void* hsrc, size_t nb) {
    void* d = sl.dev_buf(i, nb);
    if (nb) hip_check(hipMemcpyAsync(d, hsrc, nb, hipMemcpyHostToDevice, st), "H2D");
    return d;
  };
  const uint8_t* d_raw = (const uint8_t*)h2d(0, h_raw, bytes);
  const uint64_t* d_off = (const uint64_t*)h2d(1, h_off, (m + 1) * 8);
  const uint32_t* d_pol = (const uint32_t*)h2d(2, h_pol, m * 4);
  const uint8_t* d_ing = (const uint8_t*)h2d(3, h_ing, m);
  const uint16_t* d_port = (const uint16_t*)h2d(4, h_port, m * 2);
  const uint32_t* d_rem = (const uint32_t*)h2d(5, h_rem, m * 4);
  uint8_t* d_out = (uint8_t*)sl.dev_buf(6, m);
  http_verdicts_raw_on(s, sl, e.cus, in, d_raw, d_off, m, d_pol, d_ing, d_port, d_rem, d_out, st);
  uint8_t* ho = (uint8_t*)sl.host_buf(6, m);
  hip_check(hipMemcpyAsync(ho, d_out, m, hipMemcpyDeviceToHost, st), "D2H");
  hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  memcpy(out + a, ho, m);
}

static void verdicts_raw_from_host(uint64_t h, RawInput in, const uint8_t* raw, const uint64_t* raw_off, size_t n,
                                   const uint32_t* policy, const uint8_t* ingress, const uint16_t* port,
                                   const uint32_t* remote, uint8_t* out) {
  auto e = get(h);
  e->require_gpu();
  auto s = http_snap(*e);
  if (!n) return;
  check_offsets(raw_off, n);
  if (!policy || !ingress || !port || !remote || !out || (raw_off[n] != raw_off[0] && !raw))
    fail(CG_INVALID_ARGUMENT, "NULL raw/policy/ingress/port/remote/out");
  if (in == RawInput::Lists)  // the 16-bit value spans (the device path would deny it)
    for (size_t i = 0; i < n; ++i)
      if (raw_off[i + 1] - raw_off[i] > 0xFFFFu) fail(CG_INVALID_ARGUMENT, "header list longer than 64 KiB");
  const uint64_t total = raw_off[n] - raw_off[0] + 19 * (uint64_t)n;
  // (CILIUM_GPU_HOST_CHUNK_MB: another chunk size, for measurements)
  size_t chunk_bytes = kHostChunkBytes;
  if (const char* v = getenv("CILIUM_GPU_HOST_CHUNK_MB")) chunk_bytes = std::max<size_t>(1, strtoull(v, nullptr, 10)) << 20;
  const size_t nchunks = (size_t)std::max<uint64_t>(1, std::min<uint64_t>(n / 4096 + 1, total / chunk_bytes + 1));
  const unsigned nw = nchunks > 1 ? 2u : 1u;
  const unsigned copy_threads = std::max(1u, cg_http_pack_threads() / nw);
  std::exception_ptr err;
  std::mutex mu;
  auto worker = [&](unsigned w) {
    try {
      e->set_device();
      auto lease = e->staging.acquire(e->device);
      for (size_t k = w; k < nchunks; k += nw) {
        {
          std::lock_guard<std::mutex> lk(mu);
          if (err) return;
        }
        run_host_chunk(*s, *e, *lease, in, raw, raw_off, n * k / nchunks, n * (k + 1) / nchunks, policy, ingress,
                       port, remote, out, copy_threads);
      }
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu);
      if (!err) err = std::current_exception();
    }
  };
  if (nw == 1) {
    worker(0);
  } else {
    std::thread t1(worker, 1u);
    worker(0);
    t1.join();
  }
  if (err) std::rethrow_exception(err);
}

int cg_http_verdicts_raw_host(uint64_t h, const uint8_t* raw, const uint64_t* raw_off, size_t n,
                              const uint32_t* policy, const uint8_t* ingress, const uint16_t* port,
                              const uint32_t* remote, uint8_t* out) {
  return guarded([&] { verdicts_raw_from_host(h, RawInput::Heads, raw, raw_off, n, policy, ingress, port, remote, out); });
}

// ---- small header-list calls: the host packer on the calling thread ----
// Envoy decides one request per decodeHeaders (cilium_l7policy.cc:127-182),
// from many worker threads at once.  For a call of at most kSmallLists lists
// the host packer (one pass, no device layout step) + one staged copy in +
// one http_kernel launch + one copy out is the fastest sequence: 29.5 us per
// single-request call, 90K calls/s from 16 threads, each call on its own
// staging lease (profiles/r05g_http_latency.jsonl).  Combining concurrent
// calls into one batch was measured and lost (80K calls/s at 8 calls per
// batch: the flusher serializes the packing and the wake-ups).
constexpr size_t kSmallLists = 1024;

static void small_lists_host(Engine& e, const uint8_t* blob, const uint64_t* off, size_t n, const uint32_t* pol,
                             const uint8_t* ing, const uint16_t* port, const uint32_t* rem, uint8_t* out) {
  auto s = http_snap(e);
  const size_t bytes = off[n] - off[0];
  // the overflow arena holds the strings past a slot: bounded by the list
  // bytes plus each request's separators
  const size_t arena_cap = bytes + n * (2 * s->fields.size() + 24) + 64;
  e.set_device();
  auto lease = e.staging.acquire(e.device);
  const size_t bcap = http_batch_bytes(*s, n), scap = http_batch_slots(*s, n) + 1;
  uint8_t* hb = (uint8_t*)lease->host_buf(0, bcap);
  uint8_t* ha = (uint8_t*)lease->host_buf(1, arena_cap);
  std::vector<uint32_t> order(scap);
  size_t nslots = 0, aused = 0;
  http_pack(*s, n, pol, ing, port, rem, blob, off, hb, bcap, order.data(), &nslots, ha, arena_cap, &aused);
  HttpBatchHeader hdr;
  memcpy(&hdr, hb, sizeof(hdr));
  const hipStream_t st = (hipStream_t)lease->stream;
  void* dr = lease->dev_buf(0, bcap);
  void* da = lease->dev_buf(1, arena_cap);
  hip_check(hipMemcpyAsync(dr, hb, hdr.total_bytes, hipMemcpyHostToDevice, st), "H2D");
  if (hdr.arena_bytes) hip_check(hipMemcpyAsync(da, ha, hdr.arena_bytes, hipMemcpyHostToDevice, st), "H2D");
  void* dout = lease->dev_buf(2, nslots + 1);
  check_launch(launch_http(s->dev, dr, nslots, (const uint8_t*)da, (uint8_t*)dout, st, e.cus), "http kernel launch");
  uint8_t* slots = (uint8_t*)lease->host_buf(2, nslots + 1);
  if (nslots) hip_check(hipMemcpyAsync(slots, dout, nslots, hipMemcpyDeviceToHost, st), "D2H");
  hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  memset(out, 0, n);
  for (size_t i = 0; i < nslots; ++i)
    if (order[i] < n) out[order[i]] = slots[i];
}

int cg_http_verdicts_fields_host(uint64_t h, const uint8_t* hdr_blob, const uint64_t* hdr_off, size_t n,
                                 const uint32_t* policy, const uint8_t* ingress, const uint16_t* port,
                                 const uint32_t* remote, uint8_t* out) {
  return guarded([&] {
    // small calls, and any call on a snapshot the device packer does not
    // take (more than kRawMaxFields header fields): the host packer, in
    // pieces of kHostPackLists, so a snapshot works or fails the same way
    // whatever the batch size
    bool host_pack = n && n <= kSmallLists;
    if (n && !host_pack) {
      auto e = get(h);
      host_pack = !http_snap(*e)->lists_ok;
    }
    if (host_pack) {
      auto e = get(h);
      e->require_gpu();
      (void)http_snap(*e);  // CG_NOT_FOUND first
      check_offsets(hdr_off, n);
      if (!policy || !ingress || !port || !remote || !out || (hdr_off[n] != hdr_off[0] && !hdr_blob))
        fail(CG_INVALID_ARGUMENT, "NULL hdr_blob/policy/ingress/port/remote/out");
      for (size_t i = 0; i < n; ++i)  // the packer's limit (16-bit value spans), before the batch is shared
        if (hdr_off[i + 1] - hdr_off[i] > 0xFFFFu) fail(CG_INVALID_ARGUMENT, "header list longer than 64 KiB");
      constexpr size_t kHostPackLists = (size_t)1 << 20;
      for (size_t a = 0; a < n; a += kHostPackLists) {
        const size_t m = std::min(kHostPackLists, n - a);
        small_lists_host(*e, hdr_blob, hdr_off + a, m, policy + a, ingress + a, port + a, remote + a, out + a);
      }
      return;
    }
    verdicts_raw_from_host(h, RawInput::Lists, hdr_blob, hdr_off, n, policy, ingress, port, remote, out);
  });
}

// ------------------------------------------------------ verdict ring ----
int cg_http_ring_open(uint64_t h, uint32_t workgroups, uint32_t slots) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    std::lock_guard<std::mutex> lk(e->ring_mu);
    if (e->ring) fail(CG_INVALID_ARGUMENT, "the handle's ring is open");
    auto r = std::make_shared<HttpRing>();
    r->open(*e, workgroups, slots);
    e->ring = std::move(r);
    bump_epoch();
  });
}

// A calling thread's handle, ring and snapshot as of epoch `epoch` (g_epoch).
struct RingCallCache {
  uint64_t h = 0, epoch = 0;
  std::shared_ptr<Engine> e;
  std::shared_ptr<HttpRing> r;
  std::shared_ptr<HttpSnapshot> s;
};
thread_local RingCallCache t_ring_call;

int cg_http_ring_verdicts(uint64_t h, const uint8_t* hdr_blob, const uint64_t* hdr_off, size_t n,
                          const uint32_t* policy, const uint8_t* ingress, const uint16_t* port,
                          const uint32_t* remote, uint8_t* out) {
  bool other = false;
  const int rc = guarded([&] {
    RingCallCache& c = t_ring_call;
    const uint64_t ep = g_epoch.load(std::memory_order_acquire);
    if (c.h != h || c.epoch != ep || !c.e) {  // the locked lookups, once per thread and epoch
      c = RingCallCache{};
      auto e = get(h);
      e->require_gpu();
      std::shared_ptr<HttpRing> r;
      {
        std::lock_guard<std::mutex> lk(e->ring_mu);
        r = e->ring;
      }
      if (!r) fail(CG_NOT_FOUND, "no ring open (cg_http_ring_open)");
      auto s = http_snap(*e);
      c = RingCallCache{h, ep, std::move(e), std::move(r), std::move(s)};
    }
    Engine* e = c.e.get();
    HttpRing* r = c.r.get();
    const std::shared_ptr<HttpSnapshot>& s = c.s;
    if (!n) return;
    check_offsets(hdr_off, n);
    if (!policy || !ingress || !port || !remote || !out || (hdr_off[n] != hdr_off[0] && !hdr_blob))
      fail(CG_INVALID_ARGUMENT, "NULL hdr_blob/policy/ingress/port/remote/out");
    for (size_t i = 0; i < n; ++i)  // the packer's limit (16-bit value spans)
      if (hdr_off[i + 1] - hdr_off[i] > 0xFFFFu) fail(CG_INVALID_ARGUMENT, "header list longer than 64 KiB");
    if (n > kRingReqs || hdr_off[n] - hdr_off[0] > kRingBlob || !s->lists_ok) {
      other = true;  // past a slot: the staged entry
      return;
    }
    r->verdicts(*e, s, hdr_blob, hdr_off, n, policy, ingress, port, remote, out);
  });
  if (rc == CG_OK && other)
    return cg_http_verdicts_fields_host(h, hdr_blob, hdr_off, n, policy, ingress, port, remote, out);
  return rc;
}

int cg_http_ring_stats(uint64_t h, uint64_t* served, uint64_t* launches) {
  return guarded([&] {
    auto e = get(h);
    std::shared_ptr<HttpRing> r;
    {
      std::lock_guard<std::mutex> lk(e->ring_mu);
      r = e->ring;
    }
    if (!r) fail(CG_NOT_FOUND, "no ring open (cg_http_ring_open)");
    r->stats(served, launches);
  });
}

int cg_http_ring_close(uint64_t h) {
  return guarded([&] {
    auto e = get(h);
    std::shared_ptr<HttpRing> r;
    {
      std::lock_guard<std::mutex> lk(e->ring_mu);
      r = std::move(e->ring);
    }
    bump_epoch();
    if (!r) fail(CG_NOT_FOUND, "no ring open (cg_http_ring_open)");
    r->close();
  });
}

// ------------------------------------------------------------ counters ----
static void counters_loc(Engine& e, uint32_t what, uint32_t id, void** p, size_t* n) {
  *p = nullptr;
  *n = 0;
  if (what == CG_CTR_HTTP_PROGRAMS || what == CG_CTR_HTTP_RULES || what == CG_CTR_HTTP_ALLREDUCE) {
    auto s = http_snap(e);
    uint64_t* base = s->d_counters.as<uint64_t>();
    const size_t np = s->progs.size() * 2, nr = s->rule_info.size();
    if (what == CG_CTR_HTTP_PROGRAMS) {
      *p = base;
      *n = np;
    } else if (what == CG_CTR_HTTP_RULES) {
      *p = base ? base + np + 1 : nullptr;
      *n = nr;
    } else {
      *p = base;
      *n = np + 1 + nr;
    }
  } else if (what == 1) {
    auto s = kafka_snap(e);
    *p = s->d_counters.get();
    *n = s->dflt_group.size() * 2;
  } else if (what == 2) {
    std::lock_guard<std::mutex> lk(e.mu);
    PrefilterState& pf = get_pf(e, id);
    *p = pf.d_counters ? pf.d_counters->get() : nullptr;
    *n = pf.d_counters ? 2 : 0;
  } else {
    fail(CG_INVALID_ARGUMENT, "unknown counter set");
  }
}

int cg_read_counters(uint64_t h, uint32_t what, uint32_t id, uint64_t* out, size_t cap, size_t* n) {
  return guarded([&] {
    auto e = get(h);
    void* p;
    size_t cnt;
    counters_loc(*e, what, id, &p, &cnt);
    if (n) *n = cnt;
    size_t k = std::min(cap, cnt);
    if (k && p && e->has_gpu()) {
      e->set_device();
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      hip_check(hipMemcpy(out, p, k * 8, hipMemcpyDeviceToHost), "D2H counters");
    } else if (k) {
      memset(out, 0, k * 8);
    }
  });
}

int cg_counters_device_ptr(uint64_t h, uint32_t what, uint32_t id, void** d_ptr, size_t* n) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    counters_loc(*e, what, id, d_ptr, n);
  });
}

int cg_counters_copy_dev(uint64_t h, uint32_t what, uint32_t id, void* d_dst, size_t n, void* stream) {
  return guarded([&] {
    auto e = get(h);
    e->require_gpu();
    void* p;
    size_t cnt;
    counters_loc(*e, what, id, &p, &cnt);
    size_t k = std::min(n, cnt);
    e->set_device();
    if (k)
      hip_check(hipMemcpyAsync(d_dst, p, k * 8, hipMemcpyDeviceToDevice, (hipStream_t)stream_of(*e, stream)),
                "D2D counters");
  });
}

int cg_reset_counters(uint64_t h) {
  return guarded([&] {
    auto e = get(h);
    if (!e->has_gpu()) return;
    e->set_device();
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->http) e->http->d_counters.zero();
    if (e->kafka) e->kafka->d_counters.zero();
    for (auto& [id, p] : e->prefilters)
      if (p->d_counters) p->d_counters->zero();
    for (auto& [id, m] : e->maps)
      if (m->d_counters) m->d_counters->zero();
  });
}

// ------------------------------------------------------ regex syntax ----
int cg_regex_validate(const char* re, size_t re_len, uint32_t flavour) {
  return guarded([&] {
    std::string err;
    const RegexFlavour f = flavour == CG_REGEX_GO ? RegexFlavour::Go : RegexFlavour::Ecma;
    if (flavour > CG_REGEX_GO) fail(CG_INVALID_ARGUMENT, "unknown regex flavour");
    if (!regex_syntax_ok(std::string(re, re_len), &err, f)) fail(CG_POLICY_REJECTED, err);
  });
}

// ------------------------------------------------------- diagnostics ----
// Host-side walkers of the compiled tables and the regex compiler, for the
// CPU test-suite only.  No verdict entry point calls them.
int cg_diag_regex_match(const char* re, size_t re_len, const uint8_t* s, size_t len, uint32_t search,
                        uint8_t* result) {
  return guarded([&] {
    // the last compiled patterns are kept: tests run one pattern on many strings
    static std::mutex mu;
    static std::map<std::pair<std::string, bool>, std::shared_ptr<const ByteDfa>> cache;
    const auto key = std::make_pair(std::string(re, re_len), search != 0);
    std::shared_ptr<const ByteDfa> d;
    {
      std::lock_guard<std::mutex> g(mu);
      auto it = cache.find(key);
      if (it != cache.end()) d = it->second;
    }
    if (!d) {
      d = std::make_shared<const ByteDfa>(
          compile_regex(key.first, ByteSet::all(), search ? MatchMode::Search : MatchMode::Full));
      std::lock_guard<std::mutex> g(mu);
      if (cache.size() >= 64) cache.clear();
      cache.emplace(key, d);
    }
    *result = dfa_run(*d, std::string((const char*)s, len)) ? 1 : 0;
  });
}

int cg_diag_http_rules_host(uint64_t h, const void* batch, size_t nslots, const uint32_t* order, size_t n,
                            const uint8_t* arena, size_t arena_len, uint32_t* rule) {
  return guarded([&] {
    auto e = get(h);
    auto s = http_snap(*e);
    std::vector<uint8_t> slots(nslots);
    std::vector<uint32_t> r(nslots);
    http_eval_host(*s, (const uint8_t*)batch, arena, arena_len, slots.data(), r.data());
    for (size_t i = 0; i < nslots; ++i)
      if (order[i] < n) rule[order[i]] = r[i];
  });
}

int cg_diag_http_eval_host(uint64_t h, const void* batch, size_t nslots, const uint32_t* order, size_t n,
                           const uint8_t* arena, size_t arena_len, uint8_t* out) {
  return guarded([&] {
    auto e = get(h);
    auto s = http_snap(*e);
    std::vector<uint8_t> slots(nslots);
    http_eval_host(*s, (const uint8_t*)batch, arena, arena_len, slots.data());
    for (size_t i = 0; i < nslots; ++i)
      if (order[i] < n) out[order[i]] = slots[i];
  });
}

// Cuckoo lookup as the L4 kernels do it: fingerprint screen, then the slot.
static bool l4_lookup_host(const PolicyMapState& m, uint64_t key, uint32_t* val) {
  uint32_t b1, b2, fp;
  l4_place(key, m.bucket_mask, &b1, &b2, &fp);
  for (uint32_t bk : {b1, b2}) {
    const L4Slot* b = m.slots.data() + (size_t)bk * 4;
    for (int s = 0; s < 4; ++s)
      if (((m.fp[bk] >> (8 * s)) & 0xFF) == fp && b[s].key == key) {
        *val = b[s].val;
        return true;
      }
  }
  return false;
}

int cg_diag_l4_eval_host(uint64_t h, uint32_t map_id, const cg_l4_tuple* t, size_t n, int32_t* out) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PolicyMapState& m = get_map(*e, map_id);
    if (m.dirty) m.rebuild(*e);
    for (size_t i = 0; i < n; ++i) {
      const bool frag = t[i].flags & CG_L4_F_FRAGMENT;
      const uint64_t eg = (t[i].flags & CG_L4_F_INGRESS) ? 0 : 1;
      uint32_t val = 0;
      int which = 0;
      if (!frag && l4_lookup_host(m, (uint64_t)t[i].identity | ((uint64_t)t[i].dport << 32) |
                                         ((uint64_t)t[i].proto << 48) | (eg << 56), &val))
        which = 1;
      else if (l4_lookup_host(m, (uint64_t)t[i].identity | (eg << 56), &val))
        which = 2;
      else if (!frag && l4_lookup_host(m, ((uint64_t)t[i].dport << 32) | ((uint64_t)t[i].proto << 48) | (eg << 56),
                                       &val))
        which = 3;
      if (which == 1 || which == 3) out[i] = (int32_t)(val >> 16);
      else if (which == 2 || (t[i].flags & CG_L4_F_CB_POLICY)) out[i] = 0;
      else out[i] = frag ? CG_DROP_FRAG_NOSUPPORT : CG_DROP_POLICY;
    }
  });
}

// The prefilter tables walked exactly as lpm_kernel does.
int cg_diag_prefilter_eval_host(uint64_t h, uint32_t pf_id, const uint32_t* v4, size_t n4, uint8_t* out4,
                                const uint8_t* v6, size_t n6, uint8_t* out6) {
  return guarded([&] {
    auto e = get(h);
    std::lock_guard<std::mutex> lk(e->mu);
    PrefilterState& p = get_pf(*e, pf_id);
    if (p.dirty) p.rebuild(*e);
    auto ep4 = [&](uint32_t a) {
      if (a == 0) return p.ep4_zero;
      uint32_t mask = (uint32_t)p.ep4_keys.size() - 1, hh = ep_hash32(a) & mask;
      for (uint32_t k = 0; k <= mask; ++k, hh = (hh + 1) & mask) {
        if (p.ep4_keys[hh] == a) return true;
        if (p.ep4_keys[hh] == 0) return false;
      }
      return false;
    };
    auto ep6 = [&](uint64_t hi, uint64_t lo) {
      if ((hi | lo) == 0) return p.ep6_zero;
      uint32_t mask = (uint32_t)(p.ep6_keys.size() / 2) - 1, hh = ep_hash128(hi, lo) & mask;
      for (uint32_t k = 0; k <= mask; ++k, hh = (hh + 1) & mask) {
        if (p.ep6_keys[2 * hh] == hi && p.ep6_keys[2 * hh + 1] == lo) return true;
        if ((p.ep6_keys[2 * hh] | p.ep6_keys[2 * hh + 1]) == 0) return false;
      }
      return false;
    };
    auto be64 = [](const uint8_t* a) {
      uint64_t x = 0;
      for (int i = 0; i < 8; ++i) x = x << 8 | a[i];
      return x;
    };
    for (size_t i = 0; i < n4; ++i) {
      uint32_t s = __builtin_bswap32(v4[2 * i]);
      bool drop = false;
      if (p.v4_filter) {
        const uint32_t q = s >> 16, tw = p.top[q >> 4], tc = (tw >> (2 * (q & 15))) & 3;
        if (tc == kLpmPartial) {
          const uint32_t m = p.top_rank[q >> 4] + __builtin_popcount(lpm_partials(tw) & ((1u << (2 * (q & 15))) - 1));
          const uint32_t k = (s >> 8) & 255, w = p.mid[(size_t)m * 16 + (k >> 4)], c = (w >> (2 * (k & 15))) & 3;
          if (c == kLpmPartial) {
            uint32_t rank = p.leaf_base[m];
            for (uint32_t j = 0; j < (k >> 4); ++j) rank += __builtin_popcount(lpm_partials(p.mid[(size_t)m * 16 + j]));
            rank += __builtin_popcount(lpm_partials(w) & ((1u << (2 * (k & 15))) - 1));
            drop = (p.leaves[(size_t)rank * 4 + ((s & 0xFF) >> 6)] >> (s & 63)) & 1;
          } else {
            drop = c == 1;
          }
        } else {
          drop = tc == 1;
        }
      }
      if (!drop) drop = !ep4(v4[2 * i + 1]);
      out4[i] = drop ? CG_XDP_DROP : CG_XDP_PASS;
    }
    for (size_t i = 0; i < n6; ++i) {
      uint64_t hi = be64(v6 + 32 * i), lo = be64(v6 + 32 * i + 8);
      bool drop = false;
      if (p.v6_filter) {
        const uint32_t t = (uint32_t)(hi >> (64 - p.v6_bits));
        uint32_t m;
        const uint32_t code = v6_code_of(p.v6_code[t >> 4], t, &m);
        drop = code == 1;
        if (code == kLpmPartial) {
          const uint32_t e = p.v6_mix[m], span = e & 15;
          int64_t R = e >> 4, L = span == 15 ? 0 : R - span;
          int64_t ans = -1;
          while (L <= R) {
            int64_t mid = (L + R) >> 1;
            std::pair<uint64_t, uint64_t> lo_m{p.v6_iv[4 * mid], p.v6_iv[4 * mid + 1]};
            if (!(std::make_pair(hi, lo) < lo_m)) ans = mid, L = mid + 1;
            else R = mid - 1;
          }
          drop = ans >= 0 && !(std::make_pair(p.v6_iv[4 * ans + 2], p.v6_iv[4 * ans + 3]) < std::make_pair(hi, lo));
        }
      }
      if (!drop) drop = !ep6(be64(v6 + 32 * i + 16), be64(v6 + 32 * i + 24));
      out6[i] = drop ? CG_XDP_DROP : CG_XDP_PASS;
    }
  });
}

int cg_diag_kafka_eval_host(uint64_t h, const cg_kafka_request* reqs, size_t n, const uint32_t* arena,
                            size_t arena_len, uint8_t* out) {
  return guarded([&] {
    auto e = get(h);
    auto s = kafka_snap(*e);
    for (size_t i = 0; i < n; ++i) out[i] = kafka_eval_host(*s, reqs[i], arena, arena_len);
  });
}

int cg_diag_kafka_decode_host(uint64_t h, const uint8_t* raw, const uint64_t* raw_off, size_t n,
                              const uint16_t* redirect, const uint32_t* remote, cg_kafka_request* reqs,
                              uint32_t* arena, size_t arena_cap, size_t* arena_used, uint8_t* status) {
  return guarded([&] {
    auto e = get(h);
    auto s = kafka_snap(*e);
    if (!arena_used || (n && (!reqs || !status || !redirect || !remote))) fail(CG_INVALID_ARGUMENT, "NULL argument");
    *arena_used = 0;
    if (!n) return;
    check_offsets(raw_off, n);
    std::vector<uint32_t> spill;
    for (size_t i = 0; i < n; ++i)
      status[i] = kafka_decode_host_one(*s, raw + raw_off[i], raw_off[i + 1] - raw_off[i], redirect[i], remote[i],
                                        &reqs[i], &spill);
    *arena_used = spill.size();
    if (spill.size() > (arena ? arena_cap : 0)) fail(CG_MAP_FULL, "Kafka topic arena too small");
    if (!spill.empty()) memcpy(arena, spill.data(), spill.size() * 4);
  });
}

}  // extern "C"
