// runtime.cc — device memory, HIP error handling, thread-local errors.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>

#include "engine.h"

namespace cg {

namespace {
thread_local std::string g_err;
}

void set_error(const std::string& msg) { g_err = msg; }
const std::string& get_error() { return g_err; }

void hip_check(int err, const char* what) {
  if (err != hipSuccess)
    fail(CG_DEVICE_ERROR, std::string(what) + ": " + hipGetErrorString((hipError_t)err));
}

DevMem::~DevMem() {
  if (p_) (void)hipFree(p_);
}

DevMem& DevMem::operator=(DevMem&& o) noexcept {
  if (this != &o) {
    if (p_) (void)hipFree(p_);
    p_ = o.p_;
    n_ = o.n_;
    o.p_ = nullptr;
    o.n_ = 0;
  }
  return *this;
}

void DevMem::alloc(size_t bytes) {
  if (p_ && n_ >= bytes && n_ <= 2 * bytes + 4096) {
    n_ = bytes;
    return;
  }
  if (p_) {
    (void)hipFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  if (bytes == 0) bytes = 16;
  hip_check(hipMalloc(&p_, bytes), "hipMalloc");
  n_ = bytes;
}

void DevMem::upload(const void* src, size_t bytes) {
  alloc(bytes);
  if (bytes) hip_check(hipMemcpy(p_, src, bytes, hipMemcpyHostToDevice), "hipMemcpy H2D");
}

void DevMem::zero() {
  if (p_ && n_) hip_check(hipMemset(p_, 0, n_), "hipMemset");
}

LaunchFence::~LaunchFence() {
  for (auto& [st, ev] : ev_) {
    (void)hipEventSynchronize((hipEvent_t)ev);
    (void)hipEventDestroy((hipEvent_t)ev);
  }
}

void LaunchFence::record(void* stream) {
  std::lock_guard<std::mutex> lk(mu_);
  void* ev = nullptr;
  for (auto& [st, e] : ev_)
    if (st == stream) ev = e;
  if (!ev) {
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    ev_.emplace_back(stream, (void*)e);
    ev = e;
  }
  hip_check(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream), "hipEventRecord");
}

void Engine::set_device() const {
  if (device >= 0) hip_check(hipSetDevice(device), "hipSetDevice");
}

void dev_sync(Engine& e, void* stream) {
  e.set_device();
  hip_check(hipStreamSynchronize((hipStream_t)(stream ? stream : e.stream)), "hipStreamSynchronize");
}

// ------------------------------------------------------------- staging ----
PinnedMem::~PinnedMem() {
  if (p_) (void)hipHostFree(p_);
}

void PinnedMem::reserve(size_t bytes) {
  if (p_ && n_ >= bytes) return;
  if (p_) {
    (void)hipHostFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  const size_t want = std::max<size_t>(bytes + bytes / 2, 4096);  // grow by 1.5x
  hip_check(hipHostMalloc(&p_, want, hipHostMallocDefault), "hipHostMalloc");
  n_ = want;
}

void* StagingSlot::dev_buf(int i, size_t bytes) {
  DevMem& d = dev[i];
  if (!d.get() || d.size() < bytes) {
    DevMem fresh;
    fresh.alloc(std::max<size_t>(bytes + bytes / 2, 4096));
    d = std::move(fresh);
  }
  return d.get();
}

void* StagingSlot::host_buf(int i, size_t bytes) {
  host[i].reserve(bytes);
  return host[i].get();
}

StagingSlot::~StagingSlot() {
  if (raw_ev) {
    (void)hipEventSynchronize((hipEvent_t)raw_ev);
    (void)hipEventDestroy((hipEvent_t)raw_ev);
  }
  if (stream) {
    (void)hipStreamSynchronize((hipStream_t)stream);
    (void)hipStreamDestroy((hipStream_t)stream);
  }
}

StagingPool::Lease::~Lease() {
  if (!s_) return;
  // an aborted call may leave copies queued: drain before the slot is reused
  (void)hipStreamSynchronize((hipStream_t)s_->stream);
  std::lock_guard<std::mutex> lk(p_->mu_);
  p_->free_.push_back(s_);
}

StagingPool::Lease StagingPool::acquire(int device) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!free_.empty()) {
      StagingSlot* s = free_.back();
      free_.pop_back();
      return Lease(this, s);
    }
  }
  auto slot = std::make_unique<StagingSlot>();
  hip_check(hipSetDevice(device), "hipSetDevice");
  hipStream_t st;
  hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
  slot->stream = st;
  StagingSlot* raw = slot.get();
  std::lock_guard<std::mutex> lk(mu_);
  all_.push_back(std::move(slot));
  return Lease(this, raw);
}

void StagingPool::clear() {
  std::lock_guard<std::mutex> lk(mu_);
  free_.clear();
  all_.clear();
}

void host_pipeline(Engine& e, size_t n, const std::vector<HostIn>& ins, const std::vector<HostOut>& outs,
                   const std::function<void(void* const*, void* const*, size_t, void*)>& launch,
                   size_t chunk_items) {
  e.require_gpu();
  e.set_device();
  if (ins.size() + outs.size() > (size_t)StagingSlot::kBufs) fail(CG_INVALID_ARGUMENT, "too many staged arrays");
  if (n == 0) return;
  size_t per_item = 0;
  for (const auto& a : ins) per_item += a.elem;
  for (const auto& a : outs) per_item += a.elem;
  if (chunk_items == 0) chunk_items = std::max<size_t>(1, ((size_t)64 << 20) / std::max<size_t>(per_item, 1));
  const size_t nch = (n + chunk_items - 1) / chunk_items;
  StagingPool::Lease lease[2] = {e.staging.acquire(e.device), e.staging.acquire(e.device)};
  const size_t ni = ins.size(), no = outs.size();
  auto retire = [&](size_t k) {  // wait for chunk k, copy its outputs to the caller
    StagingSlot& s = *lease[k & 1];
    hip_check(hipStreamSynchronize((hipStream_t)s.stream), "hipStreamSynchronize");
    const size_t off = k * chunk_items, cnt = std::min(chunk_items, n - off);
    for (size_t j = 0; j < no; ++j)
      memcpy((uint8_t*)outs[j].dst + off * outs[j].elem, s.host[ni + j].get(), cnt * outs[j].elem);
  };
  for (size_t k = 0; k < nch + 2; ++k) {
    if (k >= 2) retire(k - 2);
    if (k >= nch) continue;
    StagingSlot& s = *lease[k & 1];
    hipStream_t st = (hipStream_t)s.stream;
    const size_t off = k * chunk_items, cnt = std::min(chunk_items, n - off);
    void* din[StagingSlot::kBufs] = {};
    void* dout[StagingSlot::kBufs] = {};
    for (size_t i = 0; i < ni; ++i) {
      const size_t b = cnt * ins[i].elem;
      void* hb = s.host_buf((int)i, b);
      memcpy(hb, (const uint8_t*)ins[i].src + off * ins[i].elem, b);
      din[i] = s.dev_buf((int)i, b);
      hip_check(hipMemcpyAsync(din[i], hb, b, hipMemcpyHostToDevice, st), "H2D");
    }
    for (size_t j = 0; j < no; ++j) {
      s.host_buf((int)(ni + j), cnt * outs[j].elem);
      dout[j] = s.dev_buf((int)(ni + j), cnt * outs[j].elem + 16);
    }
    launch(din, dout, cnt, st);
    for (size_t j = 0; j < no; ++j)
      hip_check(hipMemcpyAsync(s.host[ni + j].get(), dout[j], cnt * outs[j].elem, hipMemcpyDeviceToHost, st), "D2H");
  }
}

}  // namespace cg
