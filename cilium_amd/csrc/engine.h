// engine.h — the handle behind the C ABI: device, stream, and the
// per-subsystem snapshots (L4 policy maps, prefilters, HTTP, Kafka).
#pragma once

#include <atomic>
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

struct PolicyMapState;
struct PrefilterState;
struct IpcacheState;
struct HttpSnapshot;
struct KafkaSnapshot;

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

  bool has_gpu() const { return device >= 0; }
  void require_gpu() const {
    if (!has_gpu()) fail(CG_NO_DEVICE, "handle has no GPU (opened with device=-1); no CPU fallback");
  }
  void set_device() const;  // hipSetDevice(device)
};

// HIP helpers (runtime.cc)
void hip_check(int err, const char* what);
void dev_sync(Engine& e, void* stream);

}  // namespace cg
