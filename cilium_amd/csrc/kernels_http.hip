// kernels_http.hip — HTTP L7 verdict kernel (gfx950).
//
// NetworkPolicyMap::Allowed (envoy/cilium_network_policy.h:223-237) for every
// slot of a program-grouped batch (http_pack.cc).  One workgroup takes one
// chunk of ≤ kChunkTiles tiles of a single program: it stages the program's
// comb-packed DFA (comb.h) into LDS once, then each wavefront walks 64
// requests at a time, one lane per request.  Records are tile-transposed, so
// each of a wave's nine 16-byte unit loads is one contiguous 1 KiB read; the
// DFA walk itself touches only LDS (one ds_read_b32 per byte).
#include <hip/hip_runtime.h>

#include "../../include/cilium_gpu.h"
#include "dev_types.h"
#include "kernels.h"

namespace cg {

namespace {

constexpr int kWave = 64;
constexpr int kHttpThreads = 1024;

__device__ __forceinline__ bool masks_meet(const unsigned long long* __restrict__ m, uint32_t a, uint32_t b,
                                           uint32_t w) {
  for (uint32_t i = 0; i < w; ++i)
    if (m[a + i] & m[b + i]) return true;
  return false;
}

__device__ __forceinline__ uint32_t get_byte(const uint4& w, int k) {
  const uint32_t word = (k < 4) ? w.x : (k < 8) ? w.y : (k < 12) ? w.z : w.w;
  return (word >> ((k & 3) * 8)) & 0xFFu;
}

// One comb transition (comb.h), branch-free: every lane reads the table and
// selects.  A dead lane (S = 0) reads cells[b], whose check half is never 0.
__device__ __forceinline__ uint32_t comb_step(const uint32_t* __restrict__ cells, uint32_t self_lo, uint32_t st,
                                             uint32_t b) {
  const uint32_t e = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(cells) + ((st << 2) + (b << 2)));
  const uint32_t dflt = st >= self_lo ? st : 0u;
  return (e & 0xFFFFu) == st ? (e >> 16) : dflt;
}

// Walk the in-record string of a tile's lanes (units 1..8 of the tile).
// Accepting states absorb (comb.h) and the record is zero-padded, so lanes
// step through all 16 bytes of a unit with no per-byte length test; units are
// loaded one ahead and the walk ends once no lane is alive inside its string.
__device__ __forceinline__ uint32_t walk_tile(const uint32_t* __restrict__ cells, uint32_t self_lo, uint32_t st,
                                             const uint4* __restrict__ tb, uint32_t lane, uint32_t len) {
  if (!__any(len != 0 && st != 0)) return st;
  uint4 cur = tb[1 * kWave + lane];
  for (uint32_t u = 0; u < 8; ++u) {
    const bool more = __any((u + 1) * 16 < len);
    uint4 nxt = cur;
    if (more && u < 7) nxt = tb[(u + 2) * kWave + lane];
#pragma unroll
    for (int k = 0; k < 16; ++k) st = comb_step(cells, self_lo, st, get_byte(cur, k));
    if (!more || !__any(st != 0 && (u + 1) * 16 < len)) break;
    cur = nxt;
  }
  return st;
}

// Records longer than a slot live in the overflow arena: byte loop.
__device__ __forceinline__ uint32_t walk_arena(const uint32_t* __restrict__ cells, uint32_t self_lo, uint32_t st,
                                              const uint8_t* __restrict__ arena, uint32_t aoff, uint32_t len) {
  for (uint32_t p = 0; p < len && st != 0; ++p) st = comb_step(cells, self_lo, st, arena[aoff + p]);
  return st;
}

__device__ __forceinline__ uint32_t remote_row_from(const HttpDev& T, unsigned long long key, uint32_t h,
                                                    unsigned long long k0, uint32_t v0, uint32_t dflt) {
  if (k0 == key) return v0;
  if (k0 == ~0ULL) return dflt;
  for (uint32_t probe = 1; probe <= T.rhash_mask; ++probe) {
    h = (h + 1) & T.rhash_mask;
    const unsigned long long k = T.rhash_keys[h];
    if (k == key) return T.rhash_vals[h];
    if (k == ~0ULL) break;
  }
  return dflt;
}

// One tile of 64 requests of program `prog` (a real, non-trivial program).
// `pcells`: the program's cell block when it is rebased (LDS copy or global),
// else the global table (parts walk from their own offsets).
__device__ __forceinline__ void http_tile(const HttpDev& T, const HttpProg& pg, uint32_t prog,
                                          const uint32_t* __restrict__ pcells, bool rebased,
                                          const uint4* __restrict__ tb, const uint8_t* __restrict__ arena,
                                          uint8_t* __restrict__ out, size_t slot, uint32_t lane, uint32_t* n_allow,
                                          uint32_t* n_deny) {
  const uint4 meta = tb[lane];
  const uint32_t remote = meta.x;
  const uint32_t flags = meta.w >> 24;
  const uint32_t aoff = (meta.w & 0xFFFFFFu) * 16u;
  const bool counted = !(flags & (CG_HTTP_F_PAD | CG_HTTP_F_MALFORMED));
  const bool overflow = counted && (flags & CG_HTTP_F_OVERFLOW);
  const uint32_t len = counted && !overflow ? meta.z : 0u;
  // first probe of the remote-identity mask, issued before the walk so its
  // latency hides behind it
  const unsigned long long rkey = ((unsigned long long)prog << 32) | remote;
  const uint32_t rh = hash64to32(rkey) & T.rhash_mask;
  const unsigned long long rk0 = T.rhash_keys[rh];
  const uint32_t rv0 = T.rhash_vals[rh];
  uint32_t verdict = 0;
  uint32_t rrow = 0;
  bool have_rrow = false;
  for (uint32_t pi = 0; pi < pg.part_count; ++pi) {
    const HttpPart pt = T.parts[pg.part_begin + pi];
    const uint32_t* __restrict__ cells = rebased ? pcells : pcells + pt.walk_off;
    uint32_t st = walk_tile(cells, pt.self_lo, pt.start, tb, lane, len);
    if (__any(overflow)) {
      const uint32_t sa = walk_arena(cells, pt.self_lo, pt.start, arena, aoff, overflow ? meta.z : 0u);
      if (overflow) st = sa;
    }
    if (!counted) st = 0;
    const uint32_t lab = st ? (cells[st - 1] >> 16) : 0xFFFFu;
    if (lab != 0xFFFFu && !verdict) {
      if (!have_rrow) {
        rrow = remote_row_from(T, rkey, rh, rk0, rv0, pg.default_remote);
        have_rrow = true;
      }
      if (masks_meet(T.masks, T.acc[pt.acc_off + lab], rrow, pg.mask_words)) verdict = 1;
    }
  }
  if (counted && !verdict && (pg.flags & kProgHasAlways)) {
    if (!have_rrow) rrow = remote_row_from(T, rkey, rh, rk0, rv0, pg.default_remote);
    if (masks_meet(T.masks, pg.always_off, rrow, pg.mask_words)) verdict = 1;
  }
  out[slot] = (uint8_t)verdict;
  *n_allow += counted && verdict;
  *n_deny += counted && !verdict;
}

__global__ __launch_bounds__(kHttpThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void http_kernel(HttpDev T, const uint8_t* __restrict__ batch,
                                                            size_t nslots, const uint8_t* __restrict__ arena,
                                                            uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lcells[];
  const HttpBatchHeader* H = reinterpret_cast<const HttpBatchHeader*>(batch);
  const uint32_t magic = H->magic, epoch = H->epoch, nchunks = H->nchunks, ntiles = H->ntiles;
  const uint64_t toff = H->tiles_off;
  if (magic != kBatchMagic || epoch != T.epoch || (size_t)ntiles * kWave > nslots) {
    // packed against another snapshot (or not a batch): deny every slot
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (size_t)gridDim.x * blockDim.x)
      out[i] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&T.counters[2 * T.nprogs], 1ULL);
    return;
  }
  const HttpChunk* chunks = reinterpret_cast<const HttpChunk*>(batch + sizeof(HttpBatchHeader));
  const uint4* tiles = reinterpret_cast<const uint4*>(batch + toff);
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const HttpChunk ch = chunks[c];
    if (ch.first_tile + ch.ntiles > ntiles || ch.ntiles > kChunkTiles) continue;  // malformed chunk
    const uint32_t prog = ch.prog;
    const bool real = prog < T.nprogs;
    HttpProg pg{};
    if (real) pg = T.progs[prog];
    const bool walkp = real && !(pg.flags & kProgAllowAll);
    const bool lds = walkp && (pg.flags & kProgRebased) && pg.cell_count <= T.lds_cells;
    uint32_t n_allow = 0, n_deny = 0;
    __syncthreads();  // the previous chunk is done with lcells
    if (lds)
      for (uint32_t i = threadIdx.x; i < pg.cell_count; i += blockDim.x) lcells[i] = T.cells[pg.cell_begin + i];
    __syncthreads();
    for (uint32_t t = ch.first_tile + wave; t < ch.first_tile + ch.ntiles; t += nw) {
      const uint4* tb = tiles + (size_t)t * (CG_HTTP_UNITS * kWave);
      const size_t slot = (size_t)t * kWave + lane;
      if (!walkp) {
        // no policy for the port → allow; unknown policy → deny; a scope
        // without HTTP rules → allow (cilium_network_policy.h:129-138,187-191)
        const uint32_t flags = tb[lane].w >> 24;
        const bool counted = !(flags & (CG_HTTP_F_PAD | CG_HTTP_F_MALFORMED));
        const uint32_t v = counted && (prog == kProgAllow || real) ? 1u : 0u;
        out[slot] = (uint8_t)v;
        n_allow += real && counted;
      } else if (lds) {
        http_tile(T, pg, prog, lcells, true, tb, arena, out, slot, lane, &n_allow, &n_deny);
      } else if (pg.flags & kProgRebased) {
        http_tile(T, pg, prog, T.cells + pg.cell_begin, true, tb, arena, out, slot, lane, &n_allow, &n_deny);
      } else {
        http_tile(T, pg, prog, T.cells, false, tb, arena, out, slot, lane, &n_allow, &n_deny);
      }
    }
    if (real) {
      // wave totals → two atomics per wave per chunk
      for (int o = 32; o > 0; o >>= 1) {
        n_allow += __shfl_down(n_allow, o, kWave);
        n_deny += __shfl_down(n_deny, o, kWave);
      }
      if (lane == 0) {
        if (n_allow) atomicAdd(&T.counters[2 * prog], (unsigned long long)n_allow);
        if (n_deny) atomicAdd(&T.counters[2 * prog + 1], (unsigned long long)n_deny);
      }
    }
  }
}

}  // namespace

int launch_http(const HttpDev& t, const void* batch, size_t nslots, const uint8_t* arena, uint8_t* out, void* stream,
                int cus) {
  if (nslots == 0) return 0;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)http_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  // one resident wave of workgroups: as many per CU as LDS and registers
  // allow (the program table size sets the LDS share), then grid-stride
  const size_t lds = (size_t)t.lds_cells * 4;
  static size_t occ_lds = ~(size_t)0;
  static int occ = 1;
  if (occ_lds != lds) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)http_kernel, kHttpThreads, lds) != hipSuccess ||
        nb < 1)
      nb = 1;
    occ = nb;
    occ_lds = lds;
  }
  size_t tiles = nslots / kWave;
  size_t grid = std::min<size_t>(std::max<size_t>(tiles, 1), (size_t)cus * occ);
  hipLaunchKernelGGL(http_kernel, dim3((unsigned)grid), dim3(kHttpThreads), lds,
                     (hipStream_t)stream, t, (const uint8_t*)batch, nslots, arena, out);
  return (int)hipGetLastError();
}

}  // namespace cg
