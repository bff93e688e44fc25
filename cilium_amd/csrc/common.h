// common.h — shared helpers of libciliumgpu (host side).
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cilium_gpu.h"

namespace cg {

// Thread-local last error, surfaced through cg_last_error().
void set_error(const std::string& msg);
const std::string& get_error();

// Error carrying a cg_result code; thrown only inside the library and turned
// into a return code at the C ABI (nothing crosses the boundary as an exception).
struct Error {
  int code;
  std::string msg;
};

[[noreturn]] inline void fail(int code, const std::string& msg) { throw Error{code, msg}; }

inline uint64_t mix64(uint64_t x) {
  // splitmix64 finalizer; also used on the device (kernels.hip) — keep in sync.
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

inline uint32_t next_pow2(uint64_t v) {
  uint32_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

}  // namespace cg
