// atomic_probe.hip — how fast device-scope atomics are on this GPU, for the
// raw path's slot allocation design (scan reserving tile slots per bucket key
// with global atomics instead of a count pass + host layout).
//
//   lane      every lane: atomicAdd (returning) on one of K counters 256 B apart
//   wave      wave-aggregated: one returning atomicAdd per distinct key per wave
//   max       every lane: non-returning atomicMax on one of T words (tile tails)
//   store     every lane: a plain 4-byte store (reference)
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/atomic_probe.hip -o tools/atomic_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ void k_lane(uint32_t* cnt, uint32_t K, uint32_t* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = mix((uint32_t)i) % K;
  out[i] = atomicAdd(&cnt[k * 64], 1u);
}

__global__ void k_wave(uint32_t* cnt, uint32_t K, uint32_t* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = i < n;
  uint32_t k = live ? mix((uint32_t)i) % K : 0xFFFFFFFFu;
  uint32_t slot = 0;
  bool todo = live;
  while (__any(todo)) {
    const uint64_t act = __ballot(todo);
    const int first = __builtin_ctzll(act);
    const uint32_t k0 = (uint32_t)__shfl((int)k, first, 64);
    const uint64_t m = __ballot(todo && k == k0);
    uint32_t base = 0;
    if ((int)(threadIdx.x & 63) == first) base = atomicAdd(&cnt[k0 * 64], (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, first, 64);
    if (todo && k == k0) {
      slot = base + (uint32_t)__popcll(m & ((1ull << (threadIdx.x & 63)) - 1));
      todo = false;
    }
  }
  if (live) out[i] = slot;
}

__global__ void k_max(uint32_t* tab, uint32_t T, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t h = mix((uint32_t)i);
  atomicMax(&tab[(uint32_t)(i / 64) % T], h & 0xFFFFu);
}

__global__ void k_store(uint32_t* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = mix((uint32_t)i);
}

int main() {
  const size_t n = 125829120;
  const uint32_t Ks[] = {64, 660, 5280};
  uint32_t *cnt, *out, *tab;
  hipMalloc(&cnt, 5280 * 256);
  hipMalloc(&out, n * 4);
  hipMalloc(&tab, 4u << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const unsigned grid = (unsigned)((n + 255) / 256);
  auto timeit = [&](const char* name, uint32_t K, auto launch) {
    hipMemset(cnt, 0, 5280 * 256);
    launch();  // warm
    hipMemset(cnt, 0, 5280 * 256);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"probe\": \"%s\", \"keys\": %u, \"ops\": %zu, \"ms\": %.3f, \"Gops\": %.2f}\n", name, K, n, ms / 3,
           n / (ms / 3) / 1e6);
    fflush(stdout);
  };
  timeit("store", 0, [&] { hipLaunchKernelGGL(k_store, dim3(grid), dim3(256), 0, 0, out, n); });
  for (uint32_t K : Ks) {
    timeit("lane", K, [&] { hipLaunchKernelGGL(k_lane, dim3(grid), dim3(256), 0, 0, cnt, K, out, n); });
    timeit("wave", K, [&] { hipLaunchKernelGGL(k_wave, dim3(grid), dim3(256), 0, 0, cnt, K, out, n); });
  }
  timeit("max", 1u << 20, [&] { hipLaunchKernelGGL(k_max, dim3(grid), dim3(256), 0, 0, tab, 1u << 20, n); });
  return 0;
}
