// engine.h — the handle behind the C ABI: device, stream, and the
// per-subsystem snapshots (L4 policy maps, prefilters, HTTP, Kafka).
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "dev_types.h"

namespace cg {

// Device buffer (hipMalloc'ed); empty on a handle without a GPU.
class DevMem {
 public:
  DevMem() = default;
  ~DevMem();
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  DevMem(DevMem&& o) noexcept : p_(o.p_), n_(o.n_) {
    o.p_ = nullptr;
    o.n_ = 0;
  }
  DevMem& operator=(DevMem&& o) noexcept;
  void alloc(size_t bytes);
  void upload(const void* src, size_t bytes);  // alloc + copy (synchronous)
  template <class T>
  void upload_vec(const std::vector<T>& v) {
    upload(v.data(), v.size() * sizeof(T));
  }
  void zero();
  void* get() const { return p_; }
  template <class T>
  T* as() const {
    return static_cast<T*>(p_);
  }
  size_t size() const { return n_; }

 private:
  void* p_ = nullptr;
  size_t n_ = 0;
};

// Retirement fence of a published table set.  Every launch that reads the
// set records an event on its stream after the enqueue (one event per
// stream, re-recorded, so the list stays as short as the set of streams);
// the fence's destructor waits for those events.  Declared as the LAST
// member of a table set, it is destroyed first, so the set's buffers are
// freed only after every queued kernel that reads them has finished — no
// reliance on hipFree synchronizing the device.
class LaunchFence {
 public:
  LaunchFence() = default;
  LaunchFence(const LaunchFence&) = delete;
  LaunchFence& operator=(const LaunchFence&) = delete;
  ~LaunchFence();
  void record(void* stream);  // after a launch on `stream` that reads the set

 private:
  std::mutex mu_;
  std::vector<std::pair<void*, void*>> ev_;  // (stream, hipEvent_t)
};

// One published build of a map's device tables.  A rebuild uploads into a
// fresh set and swaps the shared_ptr under the handle lock; a launch copies
// the shared_ptr (and the table view) under that lock, enqueues, and records
// the set's fence on its stream.  So neither a rebuild nor a destroy
// overwrites or frees tables a queued kernel reads: an old set is freed when
// its last holder lets go, after the kernels recorded on its fence finish.
struct DevTables {
  std::vector<DevMem> bufs;
  std::shared_ptr<DevMem> counters;  // survives rebuilds (per-entry counters)
  LaunchFence fence;                 // last member: destroyed (waited) first
  template <class T>
  T* add(const std::vector<T>& v) {
    bufs.emplace_back();
    bufs.back().upload_vec(v);
    return bufs.back().as<T>();
  }
};

// Page-locked host buffer (hipHostMalloc), grow-only.
class PinnedMem {
 public:
  PinnedMem() = default;
  ~PinnedMem();
  PinnedMem(const PinnedMem&) = delete;
  PinnedMem& operator=(const PinnedMem&) = delete;
  void reserve(size_t bytes);
  void* get() const { return p_; }
  size_t size() const { return n_; }

 private:
  void* p_ = nullptr;
  size_t n_ = 0;
};

// A staging slot for the "_host" entry points: its own stream, grow-only
// device buffers and pinned host buffers, so host calls make no hipMalloc /
// hipFree and copy with async DMA instead of pageable hipMemcpy.
struct StagingSlot {
  static constexpr int kBufs = 29;  // 0..7 host staging, 8..18 the raw HTTP path's workspace, 19..26 its device-layout
                                    // sequence's, 27-28 the Kafka decoder's inflate arena and deferred list
  void* stream = nullptr;  // hipStream_t
  DevMem dev[kBufs];
  PinnedMem host[kBufs];
  void* dev_buf(int i, size_t bytes);  // grow-only device buffer i
  void* host_buf(int i, size_t bytes); // grow-only pinned buffer i
  // The raw HTTP path leaves its work queued on the caller's stream: the
  // event after its last launch (hipEvent_t) and that stream, so the next
  // raw call on this slot from another stream waits for it on the device;
  // raw_seq tags its chunk directory (http_raw.cc).
  void* raw_ev = nullptr;
  void* raw_stream = nullptr;
  uint32_t raw_seq = 0;
  ~StagingSlot();
};

// Slots are leased per call, so concurrent host calls on one handle (Envoy
// workers, proxylib connections) proceed in parallel; a slot returns to the
// pool when the lease ends.
class StagingPool {
 public:
  class Lease {
   public:
    Lease(StagingPool* p, StagingSlot* s) : p_(p), s_(s) {}
    Lease(Lease&& o) noexcept : p_(o.p_), s_(o.s_) { o.s_ = nullptr; }
    ~Lease();
    StagingSlot* operator->() const { return s_; }
    StagingSlot& operator*() const { return *s_; }

   private:
    StagingPool* p_;
    StagingSlot* s_;
  };
  Lease acquire(int device);
  void clear();

 private:
  std::mutex mu_;
  std::vector<std::unique_ptr<StagingSlot>> all_;
  std::vector<StagingSlot*> free_;
};

struct PolicyMapState;
struct PrefilterState;
struct IpcacheState;
struct HttpSnapshot;
struct KafkaSnapshot;
class HttpRing;

struct Engine {
  int device = -1;      // -1: host-only handle (compile/pack only)
  void* stream = nullptr;  // hipStream_t
  bool debug = false;
  int cus = 256;

  std::mutex mu;  // control-plane updates and map state
  uint32_t next_id = 1;
  std::map<uint32_t, std::unique_ptr<PolicyMapState>> maps;
  std::map<uint32_t, std::unique_ptr<PrefilterState>> prefilters;
  std::map<uint32_t, std::unique_ptr<IpcacheState>> ipcaches;
  std::shared_ptr<HttpSnapshot> http;
  std::shared_ptr<KafkaSnapshot> kafka;
  StagingPool staging;  // the "_host" entry points' buffers and streams
  // Kafka decode: compressed payloads decoded on the device / requests the
  // host decoder finished (cg_kafka_decode_stats)
  std::atomic<uint64_t> kafka_inflated{0}, kafka_deferred{0}, kafka_arena_full{0};
  // the persistent verdict ring (cg_http_ring_open, ring.cc), or none
  std::mutex ring_mu;
  std::shared_ptr<HttpRing> ring;

  bool has_gpu() const { return device >= 0; }
  void require_gpu() const {
    if (!has_gpu()) fail(CG_NO_DEVICE, "handle has no GPU (opened with device=-1); no CPU fallback");
  }
  void set_device() const;  // hipSetDevice(device)
};

// HIP helpers (runtime.cc)
void hip_check(int err, const char* what);
void dev_sync(Engine& e, void* stream);

// Element-wise host pipeline for the "_host" entry points: items [0, n) go
// through in chunks; per chunk each input array is copied into a pinned
// buffer, DMA'd to the device (async), `launch` runs on the slot's stream
// over the chunk, and each output array comes back the same way.  Two
// slots alternate, so the CPU copies of one chunk overlap the other's DMA
// and kernel.  elem sizes are bytes per item; `launch` gets the device
// pointers of the chunk's inputs and outputs, the item count and the stream.
struct HostIn {
  const void* src;
  size_t elem;
};
struct HostOut {
  void* dst;
  size_t elem;
};
void host_pipeline(Engine& e, size_t n, const std::vector<HostIn>& ins, const std::vector<HostOut>& outs,
                   const std::function<void(void* const* din, void* const* dout, size_t count, void* stream)>& launch,
                   size_t chunk_items = 0);

}  // namespace cg
