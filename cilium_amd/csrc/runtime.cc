// runtime.cc — device memory, HIP error handling, thread-local errors.
#include <hip/hip_runtime_api.h>

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

void Engine::set_device() const {
  if (device >= 0) hip_check(hipSetDevice(device), "hipSetDevice");
}

void dev_sync(Engine& e, void* stream) {
  e.set_device();
  hip_check(hipStreamSynchronize((hipStream_t)(stream ? stream : e.stream)), "hipStreamSynchronize");
}

}  // namespace cg
