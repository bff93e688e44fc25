// stream_ab.hip — the LDS-DMA A/B of VERDICT r05 item 5: does staging the
// headline kernel's string units through LDS-DMA (global_load_lds_dwordx4,
// nontemporal) raise the streaming floor the kernel sits on, against the
// register loads it uses (global_load_dwordx4 nt)?
//
// The stream has http_kernel's shape (kernels_http.hip): a wave reads a
// tile's meta block (64 x 8 B) and U string units (64 x 16 B = 1 KiB each,
// one contiguous 1 KiB read per unit) and writes one byte per lane; tiles are
// dealt to waves in runs; 1024-thread workgroups at 8 waves per SIMD (64
// VGPRs), with the LDS a workgroup also holds for its program block (so the
// occupancy is the kernel's: 2 workgroups per CU at config 5's 75 KiB block).
// Nothing is walked: each lane folds its bytes into one word so no load is
// dead.  Variants:
//   reg   units into registers, a rolling window of kWin units ahead
//   dma   units by LDS-DMA into a per-wave ring of kWin 1 KiB slots, each
//         read back with ds_read_b128 after a counted vmcnt
// Build (CPU): hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/stream_ab.hip -o tools/stream_ab
// Run (GPU box): tools/stream_ab [GiB] [units per tile]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      exit(2);                                                               \
    }                                                                        \
  } while (0)

constexpr int kThreads = 1024, kWaves = kThreads / 64, kWin = 4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t fold(u32x4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <int U>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void stream_reg(
    const uint8_t* __restrict__ tiles, uint32_t ntiles, uint8_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t tile_bytes = 512 + (size_t)U * 1024;
  for (uint32_t t = blockIdx.x * kWaves + wave; t < ntiles; t += gridDim.x * kWaves) {
    const uint8_t* tb = tiles + (size_t)t * tile_bytes;
    const u32x2 m = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(tb) + lane);
    uint32_t acc = m.x ^ m.y;
    u32x4 w[kWin];
#pragma unroll
    for (int k = 0; k < kWin && k < U; ++k)
      w[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(tb + 512 + (size_t)k * 1024) + lane);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const u32x4 v = w[k % kWin];
      if (k + kWin < U)
        w[k % kWin] =
            __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(tb + 512 + (size_t)(k + kWin) * 1024) + lane);
      acc += fold(v);
    }
    out[(size_t)t * 64 + lane] = (uint8_t)acc;
  }
}

template <int U>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void stream_dma(
    const uint8_t* __restrict__ tiles, uint32_t ntiles, uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // this wave's ring: kWin slots of 1 KiB, after the block the kernel holds
  uint32_t* ring = lds + (size_t)wave * kWin * 256;
  const size_t tile_bytes = 512 + (size_t)U * 1024;
  for (uint32_t t = blockIdx.x * kWaves + wave; t < ntiles; t += gridDim.x * kWaves) {
    const uint8_t* tb = tiles + (size_t)t * tile_bytes;
    const u32x2 m = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(tb) + lane);
    uint32_t acc = m.x ^ m.y;
#pragma unroll
    for (int k = 0; k < kWin && k < U; ++k)
      __builtin_amdgcn_global_load_lds((const void*)(tb + 512 + (size_t)k * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(ring + k * 256), 16, 0, 2);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      // slot k % kWin has landed once at most (issued after it) DMAs remain
      const int later = (U - 1 - k) < (kWin - 1) ? (U - 1 - k) : (kWin - 1);
      if (later >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (later == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if (later == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const u32x4 v = *reinterpret_cast<const u32x4*>(ring + (k % kWin) * 256 + lane * 4);
      acc += fold(v);
      if (k + kWin < U) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's read is done before it is refilled
        __builtin_amdgcn_global_load_lds((const void*)(tb + 512 + (size_t)(k + kWin) * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)(ring + (k % kWin) * 256), 16, 0, 2);
      }
    }
    out[(size_t)t * 64 + lane] = (uint8_t)acc;
  }
}

template <class K>
float run(K kern, const char* name, int U, const uint8_t* d, uint32_t ntiles, uint8_t* out, size_t lds, int cus,
          double bytes) {
  CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  int occ = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)kern, kThreads, lds));
  const int grid = cus * (occ > 0 ? occ : 1);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, 0, d, ntiles, out);
  CHECK(hipDeviceSynchronize());
  const int iters = 10;
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, 0, d, ntiles, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= iters;
  printf("{\"variant\": \"%s\", \"units\": %d, \"lds_bytes\": %zu, \"workgroups_per_cu\": %d, \"ms\": %.4f, "
         "\"GBps\": %.1f, \"frac_of_8TBps\": %.4f}\n",
         name, U, lds, occ, ms, bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 8e12);
  fflush(stdout);
  return ms;
}

template <int U>
void ab(double gib, int cus) {
  const size_t tile_bytes = 512 + (size_t)U * 1024;
  const uint32_t ntiles = (uint32_t)(gib * (1u << 30) / tile_bytes);
  uint8_t *d = nullptr, *out = nullptr;
  CHECK(hipMalloc(&d, (size_t)ntiles * tile_bytes));
  CHECK(hipMalloc(&out, (size_t)ntiles * 64));
  CHECK(hipMemset(d, 0x5A, (size_t)ntiles * tile_bytes));
  const double bytes = (double)ntiles * (tile_bytes + 64);
  // the program block http_kernel holds in LDS (config 5's largest: 75 KiB)
  const size_t block = 75 * 1024;
  for (int rep = 0; rep < 2; ++rep) {
    run(stream_reg<U>, "reg", U, d, ntiles, out, block, cus, bytes);
    run(stream_dma<U>, "dma", U, d, ntiles, out, block + (size_t)kWaves * kWin * 1024, cus, bytes);
    // the ring without the program block: LDS-DMA at the register variant's occupancy
    run(stream_dma<U>, "dma_noblock", U, d, ntiles, out, (size_t)kWaves * kWin * 1024, cus, bytes);
  }
  CHECK(hipFree(d));
  CHECK(hipFree(out));
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 8.0;
  const int units = argc > 2 ? atoi(argv[2]) : 3;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  switch (units) {
    case 2: ab<2>(gib, cus); break;
    case 4: ab<4>(gib, cus); break;
    default: ab<3>(gib, cus); break;
  }
  return 0;
}
