// kernels.hip — gfx950 verdict kernels.
//
// All four kernels are byte/integer work bound by HBM streaming plus table
// probes (no MFMA): one lane per item, 64-lane wavefronts, vector loads of the
// packed input, counters privatized in LDS and flushed once per block.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include "../../include/cilium_gpu.h"
#include "dev_types.h"
#include "kernels.h"

namespace cg {

namespace {

constexpr int kWave = 64;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// =============================================================== L4 ======
// __policy_can_access (bpf/lib/policy.h:46-110) per tuple.

// Verdict for one tuple given which lookup hit (1: L4, 2: L3, 3: wildcard
// identity L4, 0: none) and the slot value {entry id, proxy_port_be << 16}.
__device__ __forceinline__ int32_t l4_verdict(int which, uint32_t val, uint32_t flags) {
  if (which == 1 || which == 3) return (int32_t)(val >> 16);  // return policy->proxy_port
  if (which == 2) return 0;  // TC_ACT_OK: the L3 entry's proxy_port is ignored
  if (flags & CG_L4_F_CB_POLICY) return 0;
  return (flags & CG_L4_F_FRAGMENT) ? CG_DROP_FRAG_NOSUPPORT : CG_DROP_POLICY;
}

// The verdict wrappers (bpf/lib/policy.h:126-163).  mode & 3:
// CG_L4_CAN_ACCESS = __policy_can_access with the tuple's own direction and
// fragment flags; CG_L4_INGRESS = policy_can_access_ingress (dir CT_INGRESS,
// the tuple's is_fragment); CG_L4_EGRESS = policy_can_egress (dir CT_EGRESS,
// is_fragment false).  Both wrappers return DROP_POLICY for any negative
// result, or TC_ACT_OK when built with IGNORE_DROP (mode & CG_L4_IGNORE_DROP).
__device__ __forceinline__ uint32_t l4_mode_word(uint32_t w1, uint32_t mode) {
  const uint32_t m = mode & 3u;
  if (m == CG_L4_INGRESS) return w1 | (CG_L4_F_INGRESS << 24);
  if (m == CG_L4_EGRESS) return w1 & ~((CG_L4_F_INGRESS | CG_L4_F_FRAGMENT) << 24);
  return w1;
}
__device__ __forceinline__ int32_t l4_wrap(int32_t v, uint32_t mode) {
  if ((mode & 3u) != CG_L4_CAN_ACCESS && v < 0) return (mode & CG_L4_IGNORE_DROP) ? 0 : CG_DROP_POLICY;
  return v;
}

// The three policy_key lookups of __policy_can_access (bpf/lib/policy.h:61-109)
// in priority order: j=0 {id, dport, proto, dir} (skipped for fragments),
// j=1 {id, 0, 0, dir}, j=2 {0, dport, proto, dir} (skipped for fragments).
// The keys share their hash products: h_j = fin(lo_j*M1 + hi_j*M2) with
// lo in {id, id, 0} and hi in {pp, eg, pp}.
//
// Candidates come from the fingerprint words: a zero-byte test on word^fp
// (it can flag a byte next to a true match as well, which only costs a slot
// read); bit p = slot*8 + j*2 + c for key j, bucket choice c.  A policy key
// sits in one slot, so the lowest j whose slot key matches is the verdict;
// candidates are walked in bit order and a j=0 match ends the walk.
struct L4Cand {
  uint64_t cand;   // candidate bits (slot*8 + j*2 + c)
  uint32_t bk[6];  // bucket of (key j, choice c) at index j*2+c
  uint32_t w0, pp, eg;
};

template <typename FpWord>
__device__ __forceinline__ L4Cand l4_candidates(const L4Dev& t, FpWord fpw, uint32_t w0, uint32_t w1, bool frag) {
  L4Cand r;
  const uint32_t flags = w1 >> 24;
  // key.egress = !dir with dir = CT_INGRESS(1) / CT_EGRESS(0)
  r.eg = (flags & CG_L4_F_INGRESS) ? 0u : (1u << 24);
  r.pp = (w1 & 0xFFFFFF) | r.eg;  // dport | proto << 16 | egress << 24
  r.w0 = w0;
  const uint32_t P = w0 * kL4MulLo, Q = r.pp * kL4MulHi, E = r.eg * kL4MulHi;
  const uint32_t h[3] = {l4_fin(P + Q), l4_fin(P + E), l4_fin(Q)};
  r.cand = 0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    uint32_t fp;
    l4_place_h(h[j], t.bucket_mask, &r.bk[2 * j], &r.bk[2 * j + 1], &fp);
    if (j != 1 && frag) continue;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint32_t x = fpw(r.bk[2 * j + c]) ^ (fp * 0x01010101u);
      const uint32_t z = (x - 0x01010101u) & ~x & 0x80808080u;  // bit 8s+7: byte s zero
      r.cand |= (uint64_t)(z >> 7) << (j * 2 + c);
    }
  }
  return r;
}

// The slot a candidate bit names (selects, not indexing: a dynamically
// indexed array would live in scratch).
__device__ __forceinline__ const uint4* l4_slot(const L4Dev& t, const L4Cand& r, int bit) {
  const uint32_t jc = bit & 7;
  // masks, not a select chain: the compiler turns that into a scratch array
  const uint32_t b = (r.bk[0] & (0u - (jc == 0))) | (r.bk[1] & (0u - (jc == 1))) | (r.bk[2] & (0u - (jc == 2))) |
                     (r.bk[3] & (0u - (jc == 3))) | (r.bk[4] & (0u - (jc == 4))) | (r.bk[5] & (0u - (jc >= 5)));
  return reinterpret_cast<const uint4*>(t.slots + (size_t)b * 4 + (bit >> 3));
}

__device__ __forceinline__ bool l4_key_is(const L4Cand& r, int j, const uint4& v) {
  const uint32_t klo = j == 2 ? 0u : r.w0;
  const uint32_t khi = j == 1 ? r.eg : r.pp;
  return v.x == klo && v.y == khi;
}

// Candidates walked in bit order; a key sits in one slot, so the lowest j
// whose slot matches is the verdict, and a j=0 match ends the walk.  The
// first candidate's slot arrives loaded (v0, issued together with the other
// tuples' first loads); later ones load here (false fingerprint matches and
// tuples that need more than one key are the minority).
__device__ __forceinline__ int l4_walk(const L4Dev& t, const L4Cand& r, const uint4& v0, uint32_t* val) {
  uint64_t cand = r.cand;
  if (!cand) return 0;
  int best = 0;
  {
    const int bit = __builtin_ctzll(cand);
    cand &= cand - 1;
    const int j = (bit & 7) >> 1;
    if (l4_key_is(r, j, v0)) {
      *val = v0.z;
      best = j + 1;
      if (j == 0) return best;
    }
  }
  while (cand) {
    const int bit = __builtin_ctzll(cand);
    cand &= cand - 1;
    const int j = (bit & 7) >> 1;
    if (best && j + 1 >= best) continue;
    const uint4 v = *l4_slot(t, r, bit);
    if (l4_key_is(r, j, v)) {
      *val = v.z;
      best = j + 1;
      if (j == 0) break;
    }
  }
  return best;
}

// The three policy_key lookups of __policy_can_access (bpf/lib/policy.h:61-109)
// in priority order: j=0 {id, dport, proto, dir} (skipped for fragments),
// j=1 {id, 0, 0, dir}, j=2 {0, dport, proto, dir} (skipped for fragments).
// The keys share their hash products: h_j = fin(lo_j*M1 + hi_j*M2) with
// lo in {id, id, 0} and hi in {pp, eg, pp}.
//
// Candidates come from the fingerprint words: a zero-byte test on word^fp
// (it can flag a byte next to a true match as well, which only costs a slot
// read); bit p = slot*8 + j*2 + c for key j, bucket choice c.
template <typename FpWord>
__device__ __forceinline__ int l4_resolve(const L4Dev& t, FpWord fpw, uint32_t w0, uint32_t w1, bool frag,
                                          uint32_t* val) {
  const L4Cand r = l4_candidates(t, fpw, w0, w1, frag);
  const uint4 v0 = r.cand ? *l4_slot(t, r, __builtin_ctzll(r.cand)) : make_uint4(0, 0, 0, 0);
  return l4_walk(t, r, v0, val);
}

// Counter entry in LDS: one u64 per entry id, packets in bits 40..63, bytes in
// bits 0..39 (lengths below 64 KiB; longer ones go straight to the global
// byte counter).  A block flushes before it has counted 2^24 tuples, so
// neither field wraps (2^24 - 1 packets; (2^24 - 1) x 65535 bytes < 2^40).
constexpr uint32_t kL4Tuples = 4;       // tuples per thread per iteration
constexpr bool kL4Pipe = false;         // true: the next iteration's tuples load before this one resolves (measured equal)
constexpr size_t kL4FlushTuples = (size_t)1 << 24;

__device__ __forceinline__ void l4_count(const L4Dev& t, unsigned long long* lcnt, uint32_t id, uint32_t len) {
  if (len < 65536u) {
    atomicAdd(&lcnt[id], (1ULL << 40) | len);
  } else {
    atomicAdd(&lcnt[id], 1ULL << 40);
    atomicAdd(&t.counters[2 * id + 1], (unsigned long long)len);
  }
}

__device__ void l4_flush(const L4Dev& t, unsigned long long* lcnt) {
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < t.max_entries; e += blockDim.x) {
    const unsigned long long c = lcnt[e];
    if (c) {
      atomicAdd(&t.counters[2 * e], c >> 40);
      if (c & ((1ULL << 40) - 1)) atomicAdd(&t.counters[2 * e + 1], c & ((1ULL << 40) - 1));
      lcnt[e] = 0;
    }
  }
  __syncthreads();
}

// The remote identity of the egress flow (bpf_lxc.c:205-215 v6, :509-518 v4):
// lookup_ip{4,6}_remote_endpoint resolved to sec_label, or WORLD_ID on a miss
// or a zero sec_label (the tables store that resolution, dev_types.h).
__device__ __forceinline__ uint32_t ipc_v6_identity(const IpcacheDev& ipc, uint64_t hi, uint64_t lo, uint4 en,
                                                    uint4 kr, uint32_t v) {
  uint64_t xv;
  if (en.w && ipc_ex6_find(ipc, hi, lo, ipc_ex6_hash(hi, lo) & ipc.ex6_mask, &xv)) return (uint32_t)xv;  // a /128
  if (!ipc_le128(((uint64_t)kr.y << 32) | kr.x, ((uint64_t)kr.w << 32) | kr.z, hi, lo))
    v = (uint32_t)ipc_v6_search_value(ipc, hi, lo, en.x, en.y, en.z);
  return v;
}

// Tables whose fingerprints and counters fit LDS together (max_entries*8 +
// nbuckets*4 <= 160 KiB; the 16,384-entry default): per tuple three key
// hashes, six LDS fingerprint reads, and a slot read only on a fingerprint
// match (hits, and ~1.6% false matches per key).
// kFam 4 / 6: the tuple's identity is replaced by the ipcache resolution of
// its remote address (addrs: u32 IPv4 / 16-byte IPv6, network order) — the
// egress flow of bpf_lxc.c:509-527 (v4) and :205-220 (v6).
template <int kFam>
__global__ __launch_bounds__(1024) void l4_fp_kernel(L4Dev t, IpcacheDev ipc, const void* __restrict__ addrs,
                                                     const uint32_t* __restrict__ tuples, size_t n,
                                                     int32_t* __restrict__ out, uint32_t mode) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long l4_lds[];
  unsigned long long* lcnt = l4_lds;
  uint32_t* lfp = reinterpret_cast<uint32_t*>(l4_lds + t.max_entries);
  const uint32_t nb = t.bucket_mask + 1;
  for (uint32_t e = threadIdx.x; e < t.max_entries; e += blockDim.x) lcnt[e] = 0;
  for (uint32_t e = threadIdx.x; e < nb; e += blockDim.x) lfp[e] = t.fp[e];
  __syncthreads();
  const size_t per_iter = (size_t)blockDim.x * kL4Tuples;
  const size_t stride = (size_t)gridDim.x * per_iter;
  size_t since_flush = 0;
  // the next iteration's tuples load while this one resolves (software
  // pipelining: one HBM latency per iteration is hidden under the hashing,
  // fingerprint and slot phases of the previous one)
  uint32_t w[kL4Tuples][3], wn[kL4Tuples][3];
  uint4 a6[kL4Tuples], a6n[kL4Tuples];
  auto load = [&](size_t b, uint32_t (&ww)[kL4Tuples][3], uint4 (&aa)[kL4Tuples]) {
#pragma unroll
    for (uint32_t u = 0; u < kL4Tuples; ++u) {
      size_t i = b + u * blockDim.x + threadIdx.x;
      i = i < n ? i : n - 1;  // unconditional loads (see kafka_kernel)
      if (kFam == 6) {
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(addrs) + i);
        aa[u] = make_uint4(x.x, x.y, x.z, x.w);
        ww[u][0] = 0;
      } else {
        ww[u][0] = kFam == 4 ? __builtin_bswap32(__builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(addrs) + i))
                             : __builtin_nontemporal_load(tuples + i * 3 + 0);
      }
      ww[u][1] = l4_mode_word(__builtin_nontemporal_load(tuples + i * 3 + 1), mode);
      ww[u][2] = __builtin_nontemporal_load(tuples + i * 3 + 2);
    }
  };
  if ((size_t)blockIdx.x * per_iter < n) load((size_t)blockIdx.x * per_iter, wn, a6n);
  for (size_t base = (size_t)blockIdx.x * per_iter; base < n; base += stride) {
#pragma unroll
    for (uint32_t u = 0; u < kL4Tuples; ++u) {
      w[u][0] = wn[u][0];
      w[u][1] = wn[u][1];
      w[u][2] = wn[u][2];
      a6[u] = a6n[u];
    }
    if (kL4Pipe) {
      if (base + stride < n) load(base + stride, wn, a6n);  // uniform
    } else if (base + stride < n) {
      __builtin_amdgcn_sched_barrier(0);
    }
    if (kFam == 4) {  // the trie levels, each issued for all tuples of the lane
      uint64_t e[kL4Tuples];
      uint32_t a[kL4Tuples];
#pragma unroll
      for (uint32_t u = 0; u < kL4Tuples; ++u) a[u] = w[u][0];
      ipc_v4_resolve<kL4Tuples>(ipc, a, e);
#pragma unroll
      for (uint32_t u = 0; u < kL4Tuples; ++u) w[u][0] = (uint32_t)e[u];
    }
    if (kFam == 6) {  // bucket bits, entries, then each bucket's last run, for all tuples of the lane
      uint64_t hi[kL4Tuples], lo[kL4Tuples], cw[kL4Tuples];
      uint32_t L[kL4Tuples], R[kL4Tuples];
      uint4 ent[kL4Tuples];
      bool set[kL4Tuples];
#pragma unroll
      for (uint32_t u = 0; u < kL4Tuples; ++u) {
        hi[u] = __builtin_bswap64(((uint64_t)a6[u].y << 32) | a6[u].x);
        lo[u] = __builtin_bswap64(((uint64_t)a6[u].w << 32) | a6[u].z);
        cw[u] = ipc.code6[hi[u] >> (69 - ipc.v6_bits)];
      }
#pragma unroll
      for (uint32_t u = 0; u < kL4Tuples; ++u) {
        uint32_t k;
        set[u] = ipc_v6_bucket(cw[u], (uint32_t)(hi[u] >> (64 - ipc.v6_bits)), &k);
        ent[u] = reinterpret_cast<const uint4*>(ipc.ent6)[set[u] ? k : 0];
      }
      uint4 kr[kL4Tuples], vr[kL4Tuples];
#pragma unroll
      for (uint32_t u = 0; u < kL4Tuples; ++u) {
        L[u] = ent[u].x;
        R[u] = ent[u].y;
        const uint4* rec = reinterpret_cast<const uint4*>(ipc.runs6 + 4 * (size_t)(set[u] ? R[u] : 0));
        kr[u] = rec[0];
        vr[u] = rec[1];
      }
#pragma unroll
      for (uint32_t u = 0; u < kL4Tuples; ++u)
        w[u][0] = set[u] ? ipc_v6_identity(ipc, hi[u], lo[u], ent[u], kr[u], vr[u].x) : (uint32_t)kIpcMiss;
    }
    // candidates of every tuple, then every tuple's first slot load in
    // flight together, then the walks
    L4Cand rc[kL4Tuples];
    uint4 v0[kL4Tuples];
#pragma unroll
    for (uint32_t u = 0; u < kL4Tuples; ++u)
      rc[u] = l4_candidates(t, [&](uint32_t b) { return lfp[b]; }, w[u][0], w[u][1],
                            (w[u][1] >> 24) & CG_L4_F_FRAGMENT);
#pragma unroll
    for (uint32_t u = 0; u < kL4Tuples; ++u)  // a lane with no candidate re-reads bucket 0's first slot
      v0[u] = *l4_slot(t, rc[u], rc[u].cand ? __builtin_ctzll(rc[u].cand) : 0);
#pragma unroll
    for (uint32_t u = 0; u < kL4Tuples; ++u) {
      const size_t i = base + u * blockDim.x + threadIdx.x;
      if (i >= n) continue;
      uint32_t val = 0;
      const int which = l4_walk(t, rc[u], v0[u], &val);
      __builtin_nontemporal_store(l4_wrap(l4_verdict(which, val, w[u][1] >> 24), mode), out + i);
      if (which) l4_count(t, lcnt, val & 0xFFFF, w[u][2]);
    }
    since_flush += per_iter;
    // flush while the next iteration could bring the count to 2^24
    if (since_flush + per_iter >= kL4FlushTuples && base + stride < n) {
      l4_flush(t, lcnt);
      since_flush = 0;
    }
    if (!kL4Pipe && base + stride < n) load(base + stride, wn, a6n);
  }
  l4_flush(t, lcnt);
}

// Larger tables: fingerprints read from global memory (L2), counters as
// global atomics.
template <int kFam>
__global__ __launch_bounds__(256) void l4_kernel(L4Dev t, IpcacheDev ipc, const void* __restrict__ addrs,
                                                 const uint32_t* __restrict__ tuples, size_t n,
                                                 int32_t* __restrict__ out, uint32_t mode) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint32_t w0;
    if (kFam == 4) {
      w0 = (uint32_t)ipc_v4_value(ipc, __builtin_bswap32(reinterpret_cast<const uint32_t*>(addrs)[i]));
    } else if (kFam == 6) {
      const uint4 x = reinterpret_cast<const uint4*>(addrs)[i];
      const uint64_t hi = __builtin_bswap64(((uint64_t)x.y << 32) | x.x);
      const uint64_t lo = __builtin_bswap64(((uint64_t)x.w << 32) | x.z);
      const uint32_t tb = (uint32_t)(hi >> (64 - ipc.v6_bits));
      uint32_t k, L, R;
      w0 = (uint32_t)kIpcMiss;
      if (ipc_v6_bucket(ipc.code6[tb >> 5], tb, &k)) {
        const uint4 en = reinterpret_cast<const uint4*>(ipc.ent6)[k];
        L = en.x;
        R = en.y;
        const uint4* rec = reinterpret_cast<const uint4*>(ipc.runs6 + 4 * (size_t)R);
        w0 = ipc_v6_identity(ipc, hi, lo, en, rec[0], rec[1].x);
      }
    } else {
      w0 = tuples[i * 3 + 0];
    }
    const uint32_t w1 = l4_mode_word(tuples[i * 3 + 1], mode), len = tuples[i * 3 + 2];
    const bool frag = (w1 >> 24) & CG_L4_F_FRAGMENT;
    uint32_t val = 0;
    const int which = l4_resolve(t, [&](uint32_t b) { return t.fp[b]; }, w0, w1, frag, &val);
    out[i] = l4_wrap(l4_verdict(which, val, w1 >> 24), mode);
    if (which) {
      const uint32_t id = val & 0xFFFF;
      atomicAdd(&t.counters[2 * id], 1ULL);
      atomicAdd(&t.counters[2 * id + 1], (unsigned long long)len);
    }
  }
}

// ============================================================== LPM ======
// check_v4 / check_v6 (bpf/bpf_xdp.c:97-156): drop when the source is covered
// by the CIDR maps, else pass iff the destination is a local endpoint.

__device__ __forceinline__ uint64_t u64_of(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

// Endpoint probes continue past the first slot (the first one is issued by
// the caller together with the other requests' loads).
__device__ __forceinline__ bool ep4_probe_more(const LpmDev& t, uint32_t a, uint32_t h) {
  for (uint32_t probe = 1; probe <= t.ep4_mask; ++probe) {
    h = (h + 1) & t.ep4_mask;
    const uint32_t k = t.ep4_keys[h];
    if (k == a) return true;
    if (k == 0) return false;
  }
  return false;
}

__device__ __forceinline__ bool ep6_probe_more(const LpmDev& t, uint64_t hi, uint64_t lo, uint32_t h) {
  for (uint32_t probe = 1; probe <= t.ep6_mask; ++probe) {
    h = (h + 1) & t.ep6_mask;
    const uint4 k = *reinterpret_cast<const uint4*>(t.ep6_keys + 2 * (size_t)h);
    if (u64_of(k.x, k.y) == hi && u64_of(k.z, k.w) == lo) return true;
    if ((k.x | k.y | k.z | k.w) == 0) return false;
  }
  return false;
}

// A mixed /16: its /24 code, then for a partial /24 the leaf by rank.
__device__ __forceinline__ bool v4_mixed(const LpmDev& t, uint32_t s, uint32_t tw) {
  const uint32_t q = s >> 16;
  const uint32_t m = t.top_rank[q >> 4] + __popc(lpm_partials(tw) & ((1u << (2 * (q & 15))) - 1));
  const uint32_t k = (s >> 8) & 255;
  const uint4* chunk = reinterpret_cast<const uint4*>(t.mid + (size_t)m * 16);
  const uint4 cw = chunk[k >> 6];
  const uint32_t wi = (k >> 4) & 3;
  const uint32_t w = wi == 0 ? cw.x : wi == 1 ? cw.y : wi == 2 ? cw.z : cw.w;
  const uint32_t c = (w >> (2 * (k & 15))) & 3;
  if (c != kLpmPartial) return c == 1;
  uint32_t rank = t.leaf_base[m];
  for (uint32_t j = 0; j < (k >> 6); ++j) {
    const uint4 x = chunk[j];
    rank += __popc(lpm_partials(x.x)) + __popc(lpm_partials(x.y)) + __popc(lpm_partials(x.z)) +
            __popc(lpm_partials(x.w));
  }
  rank += (wi > 0 ? __popc(lpm_partials(cw.x)) : 0) + (wi > 1 ? __popc(lpm_partials(cw.y)) : 0) +
          (wi > 2 ? __popc(lpm_partials(cw.z)) : 0);
  rank += __popc(lpm_partials(w) & ((1u << (2 * (k & 15))) - 1));
  return (t.leaves[(size_t)rank * 4 + ((s & 0xFF) >> 6)] >> (s & 63)) & 1;
}

__device__ __forceinline__ bool le128(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
  return ah < bh || (ah == bh && al <= bl);
}

// Binary search over intervals [L, R] for the last lo <= addr (more than two
// candidates in a mixed bucket: rare with ~2 buckets per interval).
__device__ __forceinline__ int64_t v6_search(const LpmDev& t, uint64_t hi, uint64_t lo, int64_t L, int64_t R) {
  int64_t ans = -1;
  while (L <= R) {
    const int64_t m = (L + R) >> 1;
    const uint4 x = *reinterpret_cast<const uint4*>(t.v6_iv + 4 * m);
    if (le128(u64_of(x.x, x.y), u64_of(x.z, x.w), hi, lo)) {
      ans = m;
      L = m + 1;
    } else {
      R = m - 1;
    }
  }
  return ans;
}

constexpr uint32_t kLpmV4 = 8, kLpmV6 = 2;  // addresses per lane per iteration

__global__ __launch_bounds__(256) void lpm_kernel(LpmDev t, bool v4f, bool v6f, const uint2* __restrict__ v4,
                                                  size_t n4, uint8_t* __restrict__ out4,
                                                  const uint4* __restrict__ v6, size_t n6,
                                                  uint8_t* __restrict__ out6) {
  uint32_t drops = 0, passes = 0;
  const size_t nthreads = (size_t)gridDim.x * blockDim.x;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  // ---- IPv4: {saddr, daddr} per packet
  for (size_t base = (size_t)blockIdx.x * blockDim.x * kLpmV4; base < n4; base += nthreads * kLpmV4) {
    uint2 r[kLpmV4];
#pragma unroll
    for (uint32_t u = 0; u < kLpmV4; ++u) {
      size_t i = base + u * blockDim.x + threadIdx.x;
      i = i < n4 ? i : n4 - 1;  // unconditional loads (see kafka_kernel)
      const unsigned long long x =
          __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(v4) + i);
      r[u] = make_uint2((uint32_t)x, (uint32_t)(x >> 32));
    }
    uint32_t w[kLpmV4], ek[kLpmV4], eh[kLpmV4];
#pragma unroll
    for (uint32_t u = 0; u < kLpmV4; ++u) {
      const uint32_t s = bswap32(r[u].x);
      w[u] = v4f ? t.top[s >> 20] : 0u;
      eh[u] = ep_hash32(r[u].y) & t.ep4_mask;
      ek[u] = t.ep4_keys[eh[u]];
    }
#pragma unroll
    for (uint32_t u = 0; u < kLpmV4; ++u) {
      const size_t i = base + u * blockDim.x + threadIdx.x;
      if (i >= n4) continue;
      const uint32_t s = bswap32(r[u].x);
      const uint32_t c = (w[u] >> (2 * ((s >> 16) & 15))) & 3;
      bool drop = c == 1;
      if (c == kLpmPartial) drop = v4_mixed(t, s, w[u]);
      if (!drop) {
        const uint32_t a = r[u].y;
        bool has;
        if (a == 0) has = t.ep4_zero;
        else if (ek[u] == a) has = true;
        else if (ek[u] == 0) has = false;
        else has = ep4_probe_more(t, a, eh[u]);
        drop = !has;
      }
      const uint8_t v = drop ? CG_XDP_DROP : CG_XDP_PASS;
      __builtin_nontemporal_store(v, out4 + i);
      drops += drop;
      passes += !drop;
    }
  }
  // ---- IPv6: {saddr[16], daddr[16]} per packet
  for (size_t base = (size_t)blockIdx.x * blockDim.x * kLpmV6; base < n6; base += nthreads * kLpmV6) {
    uint64_t sh[kLpmV6], sl[kLpmV6], dh[kLpmV6], dl[kLpmV6];
#pragma unroll
    for (uint32_t u = 0; u < kLpmV6; ++u) {
      size_t j = base + u * blockDim.x + threadIdx.x;
      j = j < n6 ? j : n6 - 1;
      const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(v6 + 2 * j));
      const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(v6 + 2 * j + 1));
      sh[u] = bswap64(u64_of(a.x, a.y));
      sl[u] = bswap64(u64_of(a.z, a.w));
      dh[u] = bswap64(u64_of(b.x, b.y));
      dl[u] = bswap64(u64_of(b.z, b.w));
    }
    uint64_t cw[kLpmV6];
    uint4 e[kLpmV6];
    uint32_t eh[kLpmV6];
#pragma unroll
    for (uint32_t u = 0; u < kLpmV6; ++u) {
      cw[u] = v6f ? t.v6_code[sh[u] >> (68 - t.v6_bits)] : 0;
      eh[u] = ep_hash128(dh[u], dl[u]) & t.ep6_mask;
      e[u] = *reinterpret_cast<const uint4*>(t.ep6_keys + 2 * (size_t)eh[u]);
    }
    // level 2 (mixed buckets only; the others read entry 0, a hot line,
    // instead of branching around the load)
    uint32_t code[kLpmV6], mx[kLpmV6];
#pragma unroll
    for (uint32_t u = 0; u < kLpmV6; ++u) {
      uint32_t m;
      code[u] = v6_code_of(cw[u], (uint32_t)(sh[u] >> (64 - t.v6_bits)), &m);
      mx[u] = t.v6_mix[code[u] == kLpmPartial ? m : 0];
    }
    // the top two candidates of a mixed bucket, loaded together
    int64_t L[kLpmV6], R[kLpmV6];
    uint4 c1lo[kLpmV6], c1hi[kLpmV6], c0lo[kLpmV6], c0hi[kLpmV6];
#pragma unroll
    for (uint32_t u = 0; u < kLpmV6; ++u) {
      const bool mixed = code[u] == kLpmPartial;
      const uint32_t span = mx[u] & 15;
      R[u] = mixed ? (int64_t)(mx[u] >> 4) : -1;
      L[u] = span == 15 ? 0 : R[u] - span;
      const int64_t r1 = mixed ? R[u] : 0, r0 = mixed && R[u] - 1 >= L[u] ? R[u] - 1 : r1;
      const uint4* p1 = reinterpret_cast<const uint4*>(t.v6_iv + 4 * r1);
      const uint4* p0 = reinterpret_cast<const uint4*>(t.v6_iv + 4 * r0);
      c1lo[u] = p1[0];
      c1hi[u] = p1[1];
      c0lo[u] = p0[0];
      c0hi[u] = p0[1];
    }
#pragma unroll
    for (uint32_t u = 0; u < kLpmV6; ++u) {
      const size_t j = base + u * blockDim.x + threadIdx.x;
      if (j >= n6) continue;
      bool drop = code[u] == 1;
      if (code[u] == kLpmPartial) {
        uint64_t eh_ = 0, el_ = 0;
        bool found = false;
        if (le128(u64_of(c1lo[u].x, c1lo[u].y), u64_of(c1lo[u].z, c1lo[u].w), sh[u], sl[u])) {
          eh_ = u64_of(c1hi[u].x, c1hi[u].y);
          el_ = u64_of(c1hi[u].z, c1hi[u].w);
          found = true;
        } else if (R[u] - 1 >= L[u]) {
          if (le128(u64_of(c0lo[u].x, c0lo[u].y), u64_of(c0lo[u].z, c0lo[u].w), sh[u], sl[u])) {
            eh_ = u64_of(c0hi[u].x, c0hi[u].y);
            el_ = u64_of(c0hi[u].z, c0hi[u].w);
            found = true;
          } else if (R[u] - 2 >= L[u]) {
            const int64_t ans = v6_search(t, sh[u], sl[u], L[u], R[u] - 2);
            if (ans >= 0) {
              const uint4 x = reinterpret_cast<const uint4*>(t.v6_iv + 4 * ans)[1];
              eh_ = u64_of(x.x, x.y);
              el_ = u64_of(x.z, x.w);
              found = true;
            }
          }
        }
        drop = found && le128(sh[u], sl[u], eh_, el_);
      }
      if (!drop) {
        bool has;
        if ((dh[u] | dl[u]) == 0) has = t.ep6_zero;
        else if (u64_of(e[u].x, e[u].y) == dh[u] && u64_of(e[u].z, e[u].w) == dl[u]) has = true;
        else if ((e[u].x | e[u].y | e[u].z | e[u].w) == 0) has = false;
        else has = ep6_probe_more(t, dh[u], dl[u], eh[u]);
        drop = !has;
      }
      const uint8_t v = drop ? CG_XDP_DROP : CG_XDP_PASS;
      __builtin_nontemporal_store(v, out6 + j);
      drops += drop;
      passes += !drop;
    }
  }
  (void)tid;
  // wave reduce then one atomic per wave
  for (int o = 32; o > 0; o >>= 1) {
    drops += __shfl_down(drops, o, kWave);
    passes += __shfl_down(passes, o, kWave);
  }
  if ((threadIdx.x & 63) == 0) {
    if (drops) atomicAdd(&t.counters[0], (unsigned long long)drops);
    if (passes) atomicAdd(&t.counters[1], (unsigned long long)passes);
  }
}

// ============================================================ Kafka ======
// kafkaRedirect.canAccess → RequestMessage.MatchesRule
// (pkg/proxy/kafka.go:117-153, pkg/kafka/policy.go:144-225).

__device__ __forceinline__ bool kf_is_topic_key(int k) {
  // isTopicAPIKey (pkg/kafka/policy.go:27-52) as a bitmask over 0..37
  const unsigned long long m = (1ULL << 0) | (1ULL << 1) | (1ULL << 2) | (1ULL << 3) | (1ULL << 4) |
                               (1ULL << 5) | (1ULL << 6) | (1ULL << 8) | (1ULL << 9) | (1ULL << 19) |
                               (1ULL << 20) | (1ULL << 21) | (1ULL << 23) | (1ULL << 24) | (1ULL << 27) |
                               (1ULL << 28) | (1ULL << 34) | (1ULL << 35) | (1ULL << 37);
  return k >= 0 && k < 64 && ((m >> k) & 1);
}

__device__ __forceinline__ bool kf_rule_matches(const KafkaRuleDev& r, int key, int ver, uint32_t kind,
                                                uint32_t client) {
  if (!(r.flags & kKfKeyWild)) {
    if (key < 0 || key >= 64 || !((r.keys >> key) & 1)) return false;
  }
  if (!(r.flags & kKfVerWild) && r.version != ver) return false;
  const bool has_client = r.flags & kKfHasClient;
  const bool has_topic = r.flags & kKfHasTopic;
  if (!has_topic && !has_client) return true;
  if (kind == CG_KAFKA_K_TYPED) return !has_client || r.client_id == client;
  if (kind == CG_KAFKA_K_CONSUMER_METADATA) return true;
  return !(has_topic && kf_is_topic_key(key));
}

__device__ __forceinline__ void kf_flush(unsigned long long* counters, uint32_t red, uint32_t allow,
                                         uint32_t deny) {
  if (allow) atomicAdd(&counters[red * 2], (unsigned long long)allow);
  if (deny) atomicAdd(&counters[red * 2 + 1], (unsigned long long)deny);
}

// Slow part of one request: clientID table (typed requests against clientID
// rules), exception rules, then per topic the (group, topic) rule list.
__device__ __forceinline__ uint32_t kf_slow(const KafkaDev& T, const uint32_t* tids, const uint32_t* __restrict__ arena,
                                         uint32_t g, uint32_t si, uint4 tail, int key, int ver, uint32_t kind,
                                         uint32_t c, uint32_t nt, uint32_t client) {
  const bool vin = ver >= 0 && ver < 64;
  if (c == 0 && (tail.x & kKfSumHasClients)) {
    const unsigned long long k = ((unsigned long long)si << 32) | client;
    uint32_t hh = kf_hash(k) & T.chash_mask;
    for (uint32_t probe = 0; probe <= T.chash_mask; ++probe) {
      const KafkaClientDev* e = T.chash + hh;
      const uint4 a = *reinterpret_cast<const uint4*>(e);
      const unsigned long long kk = (unsigned long long)a.x | ((unsigned long long)a.y << 32);
      if (kk == k) {
        const unsigned long long cvm = (unsigned long long)a.z | ((unsigned long long)a.w << 32);
        if (e->any != 0 || (vin && ((cvm >> ver) & 1))) return 1;
        break;
      }
      if (kk == ~0ULL) break;
      hh = (hh + 1) & T.chash_mask;
    }
  }
  for (uint32_t j = 0; j < tail.z; ++j)
    if (kf_rule_matches(T.rules[tail.y + j], key, ver, kind, client)) return 1;
  if (nt == 0) return 0;
  // topic ids re-read from the record, or its topic tail (cached)
  const uint32_t* tsrc = nt > CG_KAFKA_MAX_TOPICS ? arena + tids[0] : tids;
  if (nt == CG_KAFKA_TOPICS_IN_ARENA) nt = tids[1];
  for (uint32_t t = 0; t < nt; ++t) {
    const unsigned long long k = ((unsigned long long)g << 32) | tsrc[t];
    uint32_t hh = kf_hash(k) & T.thash_mask;
    bool cov = false;
    for (uint32_t probe = 0; probe <= T.thash_mask; ++probe) {
      const KafkaTopicDev e = T.thash[hh];
      if (e.key == k) {
        for (uint32_t j = 0; j < e.cnt && !cov; ++j)
          cov = kf_rule_matches(T.rules[e.off + j], key, ver, kind, client);
        break;
      }
      if (e.key == ~0ULL) break;
      hh = (hh + 1) & T.thash_mask;
    }
    if (!cov) return 0;
  }
  return 1;
}

// kKafkaReqs requests per lane per iteration, in phases so that each phase's
// loads for all of them are in flight together: the 16-B record heads, the
// (redirect, identity) group slots, the decision summaries.  The summary for
// (group, topics?, apiKey) settles most requests with two bit tests.  The
// rest (clientID comparisons, exception rules, topic lists) are queued in LDS
// and evaluated 256 at a time by the whole block, so a few such requests do
// not make every wave walk the slow path.  Counters accumulate per lane while
// the redirect stays the same and are wave-reduced at the end.
constexpr uint32_t kKafkaReqs = 4;
constexpr uint32_t kKafkaThreads = 256;
constexpr uint32_t kKafkaQueue = kKafkaThreads * (kKafkaReqs + 1);

struct KfCount {
  uint32_t red = ~0u, allow = 0, deny = 0;
  __device__ __forceinline__ void add(const KafkaDev& T, uint32_t r, uint32_t v) {
    if (r != red) {
      if (red != ~0u) kf_flush(T.counters, red, allow, deny);
      red = r;
      allow = deny = 0;
    }
    allow += v;
    deny += v ^ 1;
  }
};

// Where a request's 16-byte head and 48-byte topic ids are: the 64-byte
// record (cg_kafka_request: head stride 4 uint4, topics right after it) or
// the split layout (cg_kafka_verdicts_split_*: heads and topic tails in two
// arrays, so the common path reads 16 bytes per request, not a 64-byte line).
struct KfLayout {
  const uint4* __restrict__ heads;
  const uint4* __restrict__ tails;
  uint32_t hstride, tstride;  // in uint4
  __device__ __forceinline__ const uint4* head(size_t i) const { return heads + i * hstride; }
  __device__ __forceinline__ const uint32_t* tids(size_t i) const {
    return reinterpret_cast<const uint32_t*>(tails + i * tstride);
  }
};

// One queued request: its head words x (apiKey | version << 16), y (kind,
// topic count, redirect) and w (clientID) come from the queue, not from HBM
// again (the head was read nontemporal: a re-read is a second fetch).
__device__ __forceinline__ void kf_slow_one(const KafkaDev& T, const KfLayout& L,
                                            const uint32_t* __restrict__ arena, uint8_t* __restrict__ out,
                                            uint32_t i, uint32_t g, uint4 h, KfCount& cnt) {
  const int key = (int16_t)(h.x & 0xFFFF), ver = (int16_t)(h.x >> 16);
  const uint32_t kind = h.y & 0xFF, nt = (h.y >> 8) & 0xFF, red = h.y >> 16;
  const uint32_t b = (key >= 0 && key < 64) ? (uint32_t)key : 64u;
  const uint32_t c = kind == CG_KAFKA_K_TYPED ? 0 : kind == CG_KAFKA_K_CONSUMER_METADATA ? 1 : 2;
  const uint32_t si = g * kKfSumsPerGroup + (nt == 0 ? kKfBuckets : 0) + b;
  const uint4 tail = *reinterpret_cast<const uint4*>(&T.sums[si].any);
  const uint32_t v = kf_slow(T, L.tids(i), arena, g, si, tail, key, ver, kind, c, nt, h.w);
  out[i] = (uint8_t)v;
  cnt.add(T, red, v);
}

__global__ __launch_bounds__(kKafkaThreads) void kafka_kernel(KafkaDev T, KfLayout L, size_t n,
                                                              const uint32_t* __restrict__ arena,
                                                              uint8_t* __restrict__ out) {
  __shared__ uint32_t q_i[kKafkaQueue], q_g[kKafkaQueue], q_x[kKafkaQueue], q_y[kKafkaQueue], q_w[kKafkaQueue];
  __shared__ uint32_t q_n;
  if (threadIdx.x == 0) q_n = 0;
  __syncthreads();
  const size_t per_iter = (size_t)kKafkaThreads * kKafkaReqs;
  const size_t stride = (size_t)gridDim.x * per_iter;
  const uint32_t lane = threadIdx.x & 63;
  KfCount cnt;
  for (size_t base = (size_t)blockIdx.x * per_iter; base < n; base += stride) {
    uint4 h[kKafkaReqs];
#pragma unroll
    for (uint32_t u = 0; u < kKafkaReqs; ++u) {
      const size_t i = base + u * kKafkaThreads + threadIdx.x;
      // unconditional (clamped) loads: a load under a branch gets its own
      // vmcnt(0) at the join, which would serialize the four
      const size_t ic = i < n ? i : n - 1;
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(L.head(ic)));
      h[u] = make_uint4(v.x, v.y, v.z, v.w);
    }
    // group slot probes (first probe for every request; further ones rare)
    uint32_t g[kKafkaReqs];
    uint4 e[kKafkaReqs];
    uint32_t hh[kKafkaReqs];
#pragma unroll
    for (uint32_t u = 0; u < kKafkaReqs; ++u) {
      const uint32_t red = h[u].y >> 16;
      hh[u] = kf_hash(((unsigned long long)red << 32) | h[u].z) & T.ghash_mask;
      e[u] = *reinterpret_cast<const uint4*>(T.ghash + hh[u]);
      g[u] = T.dflt_group[red < T.nredirects ? red : 0];
    }
#pragma unroll
    for (uint32_t u = 0; u < kKafkaReqs; ++u) {
      if (h[u].z == 0) continue;
      const uint32_t red = h[u].y >> 16;
      if (e[u].x == h[u].z && e[u].y == red) {
        g[u] = e[u].z;
        continue;
      }
      if (e[u].x == ~0u && e[u].y == ~0u) continue;
      // collision: linear probing from the next slot (a separate loop, so the
      // first probe's registers are not turned into a pointer phi)
      uint32_t slot = hh[u];
      for (uint32_t probe = 1; probe <= T.ghash_mask; ++probe) {
        slot = (slot + 1) & T.ghash_mask;
        const uint4 x = *reinterpret_cast<const uint4*>(T.ghash + slot);
        if (x.x == h[u].z && x.y == red) {
          g[u] = x.z;
          break;
        }
        if (x.x == ~0u && x.y == ~0u) break;
      }
    }
    // summaries
    uint4 tail[kKafkaReqs];
    unsigned long long vm[kKafkaReqs];
#pragma unroll
    for (uint32_t u = 0; u < kKafkaReqs; ++u) {
      const int key = (int16_t)(h[u].x & 0xFFFF);
      const uint32_t kind = h[u].y & 0xFF, nt = (h[u].y >> 8) & 0xFF;
      const uint32_t b = (key >= 0 && key < 64) ? (uint32_t)key : 64u;
      const uint32_t c = kind == CG_KAFKA_K_TYPED ? 0 : kind == CG_KAFKA_K_CONSUMER_METADATA ? 1 : 2;
      const KafkaSumDev* su = T.sums + g[u] * kKfSumsPerGroup + (nt == 0 ? kKfBuckets : 0) + b;
      tail[u] = *reinterpret_cast<const uint4*>(&su->any);
      vm[u] = su->vm[c];
    }
#pragma unroll
    for (uint32_t u = 0; u < kKafkaReqs; ++u) {
      const size_t i = base + u * kKafkaThreads + threadIdx.x;
      const int ver = (int16_t)(h[u].x >> 16);
      const uint32_t kind = h[u].y & 0xFF, nt = (h[u].y >> 8) & 0xFF, red = h[u].y >> 16;
      const uint32_t c = kind == CG_KAFKA_K_TYPED ? 0 : kind == CG_KAFKA_K_CONSUMER_METADATA ? 1 : 2;
      const bool live = i < n;
      const bool known = red < T.nredirects;
      uint32_t v = known ? (((tail[u].x >> c) & 1) | ((ver >= 0 && ver < 64) ? (uint32_t)((vm[u] >> ver) & 1) : 0u))
                         : 0u;
      const bool slow =
          live && known && !v && ((c == 0 && (tail[u].x & kKfSumHasClients)) || tail[u].z != 0 || nt != 0);
      // wave-aggregated append to the block's queue
      const unsigned long long m = __ballot(slow);
      if (m) {
        uint32_t qb = 0;
        if (lane == 0) qb = atomicAdd(&q_n, (uint32_t)__popcll(m));
        qb = __shfl(qb, 0, kWave);
        if (slow) {
          const uint32_t p = qb + (uint32_t)__popcll(m & ((1ULL << lane) - 1));
          q_i[p] = (uint32_t)i;
          q_g[p] = g[u];
          q_x[p] = h[u].x;
          q_y[p] = h[u].y;
          q_w[p] = h[u].w;
        }
      }
      if (live && !slow) {
        __builtin_nontemporal_store((uint8_t)v, out + i);
        if (known) cnt.add(T, red, v);
      }
    }
    __syncthreads();
    uint32_t nq = q_n;
    while (nq >= kKafkaThreads) {
      const uint32_t p = nq - kKafkaThreads + threadIdx.x;
      kf_slow_one(T, L, arena, out, q_i[p], q_g[p], make_uint4(q_x[p], q_y[p], 0u, q_w[p]), cnt);
      nq -= kKafkaThreads;
      __syncthreads();
      if (threadIdx.x == 0) q_n = nq;
      __syncthreads();
    }
  }
  __syncthreads();
  if (threadIdx.x < q_n) {
    const uint32_t p = threadIdx.x;
    kf_slow_one(T, L, arena, out, q_i[p], q_g[p], make_uint4(q_x[p], q_y[p], 0u, q_w[p]), cnt);
  }
  // the common case: every lane of the wave counted for the same redirect
  const uint32_t first = __builtin_amdgcn_readfirstlane(cnt.red);
  if (__all(cnt.red == first)) {
    uint32_t callow = cnt.allow, cdeny = cnt.deny;
    for (int o = 32; o > 0; o >>= 1) {
      callow += __shfl_down(callow, o, kWave);
      cdeny += __shfl_down(cdeny, o, kWave);
    }
    if (lane == 0 && first != ~0u) kf_flush(T.counters, first, callow, cdeny);
  } else if (cnt.red != ~0u) {
    kf_flush(T.counters, cnt.red, cnt.allow, cnt.deny);
  }
}

// Resident blocks per CU for a kernel (occupancy query, cached per kernel):
// grid-stride kernels launch exactly what fits, so no block runs as a tail.
int resident(const void* fn, int threads, size_t lds) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, threads, lds) != hipSuccess || nb < 1) nb = 1;
  return nb;
}

// resident() per (kernel, device), cached under a lock.
int resident_cached(const void* fn, int threads) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({fn, dev});
  if (it == cache.end()) it = cache.emplace(std::make_pair(fn, dev), resident(fn, threads, 0)).first;
  return it->second;
}

int grid_for(size_t items, int per_block, int cus, int blocks_per_cu) {
  size_t need = (items + per_block - 1) / per_block;
  size_t cap = (size_t)cus * blocks_per_cu;
  if (need > cap) need = cap;
  if (need < 1) need = 1;
  return (int)need;
}

}  // namespace

// hipFuncSetAttribute per (kernel, device): the attribute is per device, and
// handles on several GPUs may launch from several threads.
template <class F>
void set_max_lds_once(F fn, int dev_count_hint) {
  static std::once_flag flags[64];
  int d = 0;
  (void)hipGetDevice(&d);
  (void)dev_count_hint;
  std::call_once(flags[d & 63], [&] {
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  });
}

template <int kFam>
int launch_l4_t(const L4Dev& t, const IpcacheDev& ipc, const void* addrs, const void* tuples, size_t n,
                int32_t* out, uint32_t mode, void* stream, int cus) {
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = (size_t)t.max_entries * 8 + (size_t)(t.bucket_mask + 1) * 4;
  if (lds <= 160 * 1024) {
    set_max_lds_once(l4_fp_kernel<kFam>, 0);
    hipLaunchKernelGGL(l4_fp_kernel<kFam>, dim3(grid_for(n, 1024 * kL4Tuples, cus, 1)), dim3(1024), lds, s, t, ipc,
                       addrs, (const uint32_t*)tuples, n, out, mode);
  } else {
    hipLaunchKernelGGL(l4_kernel<kFam>, dim3(grid_for(n, 256, cus, 8)), dim3(256), 0, s, t, ipc, addrs,
                       (const uint32_t*)tuples, n, out, mode);
  }
  return (int)hipGetLastError();
}

int launch_l4(const L4Dev& t, const void* tuples, size_t n, int32_t* out, uint32_t mode, void* stream, int cus) {
  return launch_l4_t<0>(t, IpcacheDev{}, nullptr, tuples, n, out, mode, stream, cus);
}

int launch_l4_ipcache(const L4Dev& t, const IpcacheDev& ipc, int family, const void* addrs, const void* tuples,
                      size_t n, int32_t* out, uint32_t mode, void* stream, int cus) {
  if (family == 6) return launch_l4_t<6>(t, ipc, addrs, tuples, n, out, mode, stream, cus);
  return launch_l4_t<4>(t, ipc, addrs, tuples, n, out, mode, stream, cus);
}

int launch_lpm(const LpmDev& t, bool v4f, bool v6f, const uint32_t* v4, size_t n4, uint8_t* out4,
               const uint8_t* v6, size_t n6, uint8_t* out6, void* stream, int cus) {
  if (n4 + n6 == 0) return 0;
  const int occ = resident_cached((const void*)lpm_kernel, 256);
  hipLaunchKernelGGL(lpm_kernel, dim3(grid_for(n4 / kLpmV4 + n6 / kLpmV6 + 1, 256, cus, occ)), dim3(256), 0,
                     (hipStream_t)stream, t, v4f,
                     v6f, (const uint2*)v4, n4, out4, (const uint4*)v6, n6, out6);
  return (int)hipGetLastError();
}

int launch_kafka(const KafkaDev& t, const void* reqs, size_t n, const uint32_t* arena, uint8_t* out,
                 void* stream, int cus, const void* tails) {
  if (n == 0) return 0;
  const int occ = resident_cached((const void*)kafka_kernel, kKafkaThreads);
  // tails == nullptr: 64-byte records; else 16-byte heads + 48-byte tails
  const KfLayout L = tails ? KfLayout{(const uint4*)reqs, (const uint4*)tails, 1, 3}
                           : KfLayout{(const uint4*)reqs, (const uint4*)reqs + 1, 4, 4};
  hipLaunchKernelGGL(kafka_kernel, dim3(grid_for(n, kKafkaThreads * kKafkaReqs, cus, occ)), dim3(kKafkaThreads), 0,
                     (hipStream_t)stream, t, L, n, arena, out);
  return (int)hipGetLastError();
}

}  // namespace cg
