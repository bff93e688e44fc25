// kernels_ipcache.hip — lookup_ip{4,6}_remote_endpoint over a batch
// (bpf/lib/eps.h:48-115) with the callers' resolution (bpf_lxc.c:509-518):
// address → {security identity, tunnel endpoint}.
//
// Integer work bound by the input/output stream plus dependent table loads.
// IPv4: the /16 summary; then, in one round, the /24-level chunk's entry
// (dense, or an encoded run line / sparse map: dev_types.h ipc_chunk_get)
// and — when the /16 holds /32 entries — the exact table's slot (a /32 is
// the longest prefix: a hit is the answer); then the /32-level chunk for a
// pointer entry.  IPv6: the bucket bit, then for a bucket not spanned by one
// WORLD run its entry, then its last 32-B run record with — when the bucket
// holds /128 entries — the exact table's slot, and a short search when the
// run starts after the address.  Entries carry the resolved value inline,
// so the last table load is the answer.  Each lane resolves several
// addresses with every level's loads issued for all of them before the next
// level, so a wave keeps 2-4 (v4) / 2 (v6) independent chains in flight.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <map>
#include <mutex>

#include "dev_types.h"
#include "kernels.h"

namespace cg {

namespace {

constexpr uint32_t kIpcV6 = 2;  // IPv6 addresses per lane per iteration (IPv4: the kernel's K)
constexpr int kIpcThreads = 256;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t u64_of(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

__device__ __forceinline__ void store_val(uint64_t v, IpcVal* out) {
  __builtin_nontemporal_store((unsigned long long)v, reinterpret_cast<unsigned long long*>(out));
}

template <uint32_t kIpcV4>
__global__ __launch_bounds__(kIpcThreads) void ipcache_kernel(IpcacheDev t, const uint32_t* __restrict__ v4,
                                                              size_t n4, IpcVal* __restrict__ out4,
                                                              const uint4* __restrict__ v6, size_t n6,
                                                              IpcVal* __restrict__ out6) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  // ---- IPv4 (daddr as in iphdr, network order)
  for (size_t base = (size_t)blockIdx.x * blockDim.x * kIpcV4; base < n4; base += stride * kIpcV4) {
    uint32_t a[kIpcV4];
    uint64_t e[kIpcV4];
#pragma unroll
    for (uint32_t u = 0; u < kIpcV4; ++u) {
      size_t i = base + u * blockDim.x + threadIdx.x;
      i = i < n4 ? i : n4 - 1;  // unconditional loads: no vmcnt(0) under a branch
      a[u] = __builtin_bswap32(__builtin_nontemporal_load(v4 + i));
    }
    ipc_v4_resolve<kIpcV4>(t, a, e);
#pragma unroll
    for (uint32_t u = 0; u < kIpcV4; ++u) {
      const size_t i = base + u * blockDim.x + threadIdx.x;
      if (i < n4) store_val(e[u], out4 + i);
    }
  }
  // ---- IPv6 (16 address bytes, network order)
  for (size_t base = (size_t)blockIdx.x * blockDim.x * kIpcV6; base < n6; base += stride * kIpcV6) {
    uint64_t hi[kIpcV6], lo[kIpcV6];
    uint32_t L[kIpcV6], R[kIpcV6];
#pragma unroll
    for (uint32_t u = 0; u < kIpcV6; ++u) {
      size_t j = base + u * blockDim.x + threadIdx.x;
      j = j < n6 ? j : n6 - 1;
      const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(v6 + j));
      hi[u] = __builtin_bswap64(u64_of(x.x, x.y));
      lo[u] = __builtin_bswap64(u64_of(x.z, x.w));
    }
    // bucket bit (L2 resident), then a set bucket's entry and its last run;
    // WORLD-spanned buckets read entry / run 0, hot lines, instead of
    // branching around the loads
    uint64_t cw[kIpcV6];
#pragma unroll
    for (uint32_t u = 0; u < kIpcV6; ++u) cw[u] = t.code6[hi[u] >> (69 - t.v6_bits)];
    bool set[kIpcV6];
    uint4 ent[kIpcV6];
#pragma unroll
    for (uint32_t u = 0; u < kIpcV6; ++u) {
      uint32_t k;
      set[u] = ipc_v6_bucket(cw[u], (uint32_t)(hi[u] >> (64 - t.v6_bits)), &k);
      ent[u] = reinterpret_cast<const uint4*>(t.ent6)[set[u] ? k : 0];
    }
    // a plain set bucket: its last run (most buckets hold one run); a crowded
    // one: its crowd line's prefix and shift instead (the last run rarely
    // holds a pod address, so it is not read)
    // (a crowded bucket — many runs, now rare: the /128 pods are in the
    // exact table — reads its crowd line in the last step)
    uint4 kr[kIpcV6], vr[kIpcV6], x0[kIpcV6], x1[kIpcV6];
    bool crowd[kIpcV6], ex[kIpcV6];
    uint32_t hx[kIpcV6];
#pragma unroll
    for (uint32_t u = 0; u < kIpcV6; ++u) {
      L[u] = ent[u].x;
      R[u] = ent[u].y;
      crowd[u] = set[u] && ent[u].z != kIpcNoCrowd;
      const uint4* rec = reinterpret_cast<const uint4*>(t.runs6 + 4 * (size_t)(set[u] && !crowd[u] ? R[u] : 0));
      kr[u] = rec[0];
      vr[u] = rec[1];
      // a bucket holding /128 entries: the exact table's first slot
      ex[u] = set[u] && ent[u].w != 0;
      hx[u] = ipc_ex6_hash(hi[u], lo[u]) & t.ex6_mask;
      x0[u] = x1[u] = make_uint4(0, 0, 0, 0);
      if (ex[u]) {
        const uint4* xs = reinterpret_cast<const uint4*>(t.ex6 + 4 * (size_t)hx[u]);
        x0[u] = xs[0];
        x1[u] = xs[1];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < kIpcV6; ++u) {
      const size_t j = base + u * blockDim.x + threadIdx.x;
      if (j >= n6) continue;
      uint64_t v = u64_of(vr[u].x, vr[u].y), xv = 0;
      const bool used = ex[u] && (x1[u].z | x1[u].w) != 0;
      if (!set[u]) {
        v = kIpcMiss;
      } else if (used && u64_of(x0[u].x, x0[u].y) == hi[u] && u64_of(x0[u].z, x0[u].w) == lo[u]) {
        v = u64_of(x1[u].x, x1[u].y);  // the /128 entry: the longest prefix
      } else if (used && ipc_ex6_find(t, hi[u], lo[u], hx[u] + 1, &xv)) {
        v = xv;
      } else if (crowd[u]) {
        uint32_t i = 0, l = L[u], r = R[u];
        const uint4* cl = reinterpret_cast<const uint4*>(t.crowd6 + 128 * (size_t)ent[u].z);
        const uint4 cp = cl[0], cs = cl[1];
        const uint32_t w = ipc_v6_window(u64_of(cp.x, cp.y), u64_of(cp.z, cp.w), cs.x, hi[u], lo[u], &i);
        if (w == 0) {
          r = l;
        } else if (w == 1) {
          l = r;
        } else {
          const uint8_t* sub = t.crowd6 + 128 * (size_t)ent[u].z + 24;
          l = L[u] + sub[i];
          r = L[u] + sub[i + 1];
        }
        v = t.runs6[4 * (size_t)ipc_v6_run(t, hi[u], lo[u], l, r) + 2];
      } else if (!ipc_le128(u64_of(kr[u].x, kr[u].y), u64_of(kr[u].z, kr[u].w), hi[u], lo[u])) {
        v = ipc_v6_search_value(t, hi[u], lo[u], L[u], R[u], kIpcNoCrowd);
      }
      store_val(v, out6 + j);
    }
  }
}

int resident_blocks(const void* fn, int threads) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, threads, 0) != hipSuccess || nb < 1) nb = 1;
  return nb;
}

}  // namespace

int launch_ipcache(const IpcacheDev& t, const uint32_t* v4, size_t n4, IpcVal* out4, const uint8_t* v6, size_t n6,
                   IpcVal* out6, void* stream, int cus) {
  if (n4 + n6 == 0) return 0;
  // IPv4 addresses per lane per iteration: 2 (the kernel's 62 VGPRs keep 8
  // waves per SIMD for the IPv6 loop too; 2, 3 and 4 run the IPv4 half
  // alike — CILIUM_GPU_IPC_K = 2..4 for the A/B of tools/ipcache_split.py)
  const char* ke = getenv("CILIUM_GPU_IPC_K");
  const uint32_t K = ke && atoi(ke) >= 2 && atoi(ke) <= 4 ? (uint32_t)atoi(ke) : 2u;
  const void* fn = K == 2 ? (const void*)ipcache_kernel<2> : K == 3 ? (const void*)ipcache_kernel<3>
                                                                    : (const void*)ipcache_kernel<4>;
  int dev = 0;
  (void)hipGetDevice(&dev);
  static std::mutex mu;
  static std::map<std::pair<int, uint32_t>, int> occ_by_dev;  // per device ordinal and K
  int occ;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = occ_by_dev.find({dev, K});
    if (it == occ_by_dev.end()) it = occ_by_dev.emplace(std::make_pair(dev, K), resident_blocks(fn, kIpcThreads)).first;
    occ = it->second;
  }
  size_t need = (n4 / K + n6 / kIpcV6 + kIpcThreads) / kIpcThreads;
  const size_t cap = (size_t)cus * occ;
  need = need < cap ? need : cap;
  need = need < 1 ? 1 : need;
  const dim3 g((unsigned)need), b(kIpcThreads);
  if (K == 2)
    hipLaunchKernelGGL(ipcache_kernel<2>, g, b, 0, (hipStream_t)stream, t, v4, n4, out4, (const uint4*)v6, n6, out6);
  else if (K == 3)
    hipLaunchKernelGGL(ipcache_kernel<3>, g, b, 0, (hipStream_t)stream, t, v4, n4, out4, (const uint4*)v6, n6, out6);
  else
    hipLaunchKernelGGL(ipcache_kernel<4>, g, b, 0, (hipStream_t)stream, t, v4, n4, out4, (const uint4*)v6, n6, out6);
  return (int)hipGetLastError();
}

}  // namespace cg
