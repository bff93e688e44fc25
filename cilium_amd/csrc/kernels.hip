// kernels.hip — gfx950 verdict kernels.
//
// All four kernels are byte/integer work bound by HBM streaming plus table
// probes (no MFMA): one lane per item, 64-lane wavefronts, vector loads of the
// packed input, counters privatized in LDS and flushed once per block.
#include <hip/hip_runtime.h>

#include "../../include/cilium_gpu.h"
#include "dev_types.h"
#include "kernels.h"

namespace cg {

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// =============================================================== L4 ======
// __policy_can_access (bpf/lib/policy.h:46-110) per tuple.

__device__ __forceinline__ bool l4_probe_bucket(const L4Slot* slots, uint32_t b, uint64_t key,
                                                uint32_t* val, uint32_t* slot_out) {
  const uint4* p = reinterpret_cast<const uint4*>(slots + (size_t)b * 4);
  bool hit = false;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    uint4 v = p[s];
    uint64_t k = (uint64_t)v.x | ((uint64_t)v.y << 32);
    if (k == key) {
      hit = true;
      *val = v.z;
    }
  }
  return hit;
}

__device__ __forceinline__ bool l4_lookup(const L4Dev& t, uint64_t key, uint32_t* val) {
  uint32_t dummy;
  if (l4_probe_bucket(t.slots, (uint32_t)l4_hash1(key) & t.bucket_mask, key, val, &dummy)) return true;
  return l4_probe_bucket(t.slots, (uint32_t)l4_hash2(key) & t.bucket_mask, key, val, &dummy);
}

template <bool kLdsCounters>
__global__ __launch_bounds__(1024) void l4_kernel(L4Dev t, const uint32_t* __restrict__ tuples, size_t n,
                                                  int32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* lpk = lds;
  uint32_t* lby = lds + t.max_entries;
  if (kLdsCounters) {
    for (uint32_t i = threadIdx.x; i < 2 * t.max_entries; i += blockDim.x) lds[i] = 0;
    __syncthreads();
  }
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t per_chunk = (size_t)65536;  // tuples per thread-block between flushes ≤ 64K
  size_t done_in_chunk = 0;
  for (size_t base = (size_t)blockIdx.x * blockDim.x; base < n; base += stride) {
    size_t i = base + threadIdx.x;
    if (i < n) {
      const uint32_t w0 = tuples[i * 3 + 0];
      const uint32_t w1 = tuples[i * 3 + 1];
      const uint32_t len = tuples[i * 3 + 2];
      const uint32_t identity = w0;
      const uint32_t dport = w1 & 0xFFFF;
      const uint32_t proto = (w1 >> 16) & 0xFF;
      const uint32_t flags = w1 >> 24;
      const bool frag = flags & CG_L4_F_FRAGMENT;
      // key.egress = !dir with dir = CT_INGRESS(1) / CT_EGRESS(0)
      const uint64_t eg = (flags & CG_L4_F_INGRESS) ? 0ULL : 1ULL;
      uint32_t val = 0;
      int32_t verdict;
      int which = 0;  // 1: L4 hit, 2: L3 hit, 3: wildcard-identity L4 hit
      if (!frag && l4_lookup(t, (uint64_t)identity | ((uint64_t)dport << 32) | ((uint64_t)proto << 48) | (eg << 56), &val))
        which = 1;
      else if (l4_lookup(t, (uint64_t)identity | (eg << 56), &val))
        which = 2;
      else if (!frag && l4_lookup(t, ((uint64_t)dport << 32) | ((uint64_t)proto << 48) | (eg << 56), &val))
        which = 3;
      if (which == 1 || which == 3) {
        verdict = (int32_t)(val >> 16);  // return policy->proxy_port (be16 as stored)
      } else if (which == 2) {
        verdict = 0;  // TC_ACT_OK: the L3 entry's proxy_port is ignored
      } else if (flags & CG_L4_F_CB_POLICY) {
        verdict = 0;
      } else {
        verdict = frag ? CG_DROP_FRAG_NOSUPPORT : CG_DROP_POLICY;
      }
      out[i] = verdict;
      if (which) {
        const uint32_t id = val & 0xFFFF;
        if (kLdsCounters) {
          atomicAdd(&lpk[id], 1u);
          if (len < 65536u)
            atomicAdd(&lby[id], len);
          else
            atomicAdd(&t.counters[2 * id + 1], (unsigned long long)len);
        } else {
          atomicAdd(&t.counters[2 * id], 1ULL);
          atomicAdd(&t.counters[2 * id + 1], (unsigned long long)len);
        }
      }
    }
    if (kLdsCounters) {
      if (++done_in_chunk == per_chunk / 1024 || base + stride >= n) {
        done_in_chunk = 0;
        __syncthreads();
        for (uint32_t e = threadIdx.x; e < t.max_entries; e += blockDim.x) {
          uint32_t p = lpk[e], b = lby[e];
          if (p) {
            atomicAdd(&t.counters[2 * e], (unsigned long long)p);
            lpk[e] = 0;
          }
          if (b) {
            atomicAdd(&t.counters[2 * e + 1], (unsigned long long)b);
            lby[e] = 0;
          }
        }
        __syncthreads();
      }
    }
  }
}

// ============================================================== LPM ======
// check_v4 / check_v6 (bpf/bpf_xdp.c:97-156).

__device__ __forceinline__ bool ep4_has(const LpmDev& t, uint32_t a) {
  uint32_t h = ep_hash32(a) & t.ep4_mask;
  for (uint32_t probe = 0; probe <= t.ep4_mask; ++probe) {
    if (!t.ep4_occ[h]) return false;
    if (t.ep4_keys[h] == a) return true;
    h = (h + 1) & t.ep4_mask;
  }
  return false;
}

__device__ __forceinline__ bool ep6_has(const LpmDev& t, uint64_t hi, uint64_t lo) {
  uint32_t h = ep_hash128(hi, lo) & t.ep6_mask;
  for (uint32_t probe = 0; probe <= t.ep6_mask; ++probe) {
    if (!t.ep6_occ[h]) return false;
    if (t.ep6_keys[2 * h] == hi && t.ep6_keys[2 * h + 1] == lo) return true;
    h = (h + 1) & t.ep6_mask;
  }
  return false;
}

__device__ __forceinline__ bool v4_covered(const LpmDev& t, uint32_t a /* host order */) {
  uint32_t e = t.dir24[a >> 8];
  if (e < 2) return e == 1;
  const uint64_t* l = t.leaves + (size_t)(e - 2) * 4;
  uint32_t x = a & 0xFF;
  return (l[x >> 6] >> (x & 63)) & 1;
}

__device__ __forceinline__ bool lt128(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
  return ah < bh || (ah == bh && al < bl);
}

__device__ __forceinline__ bool v6_covered(const LpmDev& t, uint64_t hi, uint64_t lo) {
  const uint32_t top = (uint32_t)(hi >> 48);
  int64_t L = t.v6_idx[top];
  int64_t cnt = t.v6_idx[65536];
  int64_t R = t.v6_idx[top + 1];
  if (R > cnt - 1) R = cnt - 1;
  // last interval in [L, R] with lo_i <= addr
  int64_t ans = -1;
  while (L <= R) {
    int64_t m = (L + R) >> 1;
    uint64_t mh = t.v6_lo[2 * m], ml = t.v6_lo[2 * m + 1];
    if (!lt128(hi, lo, mh, ml)) {
      ans = m;
      L = m + 1;
    } else {
      R = m - 1;
    }
  }
  if (ans < 0) return false;
  uint64_t eh = t.v6_hi[2 * ans], el = t.v6_hi[2 * ans + 1];
  return !lt128(eh, el, hi, lo);
}

__global__ __launch_bounds__(256) void lpm_kernel(LpmDev t, bool v4f, bool v6f, const uint2* __restrict__ v4,
                                                  size_t n4, uint8_t* __restrict__ out4,
                                                  const uint4* __restrict__ v6, size_t n6,
                                                  uint8_t* __restrict__ out6) {
  uint32_t drops = 0, passes = 0;
  const size_t total = n4 + n6;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    uint8_t v;
    if (i < n4) {
      uint2 r = v4[i];
      bool drop = v4f && v4_covered(t, bswap32(r.x));
      if (!drop) drop = !ep4_has(t, r.y);
      v = drop ? CG_XDP_DROP : CG_XDP_PASS;
      out4[i] = v;
    } else {
      size_t j = i - n4;
      uint4 s = v6[2 * j], d = v6[2 * j + 1];
      uint64_t shi = bswap64((uint64_t)s.x | ((uint64_t)s.y << 32));
      uint64_t slo = bswap64((uint64_t)s.z | ((uint64_t)s.w << 32));
      bool drop = v6f && v6_covered(t, shi, slo);
      if (!drop) {
        uint64_t dhi = bswap64((uint64_t)d.x | ((uint64_t)d.y << 32));
        uint64_t dlo = bswap64((uint64_t)d.z | ((uint64_t)d.w << 32));
        drop = !ep6_has(t, dhi, dlo);
      }
      v = drop ? CG_XDP_DROP : CG_XDP_PASS;
      out6[j] = v;
    }
    drops += v == CG_XDP_DROP;
    passes += v == CG_XDP_PASS;
  }
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

// One lane per request (64-B records, four 16-B loads).  The group lookup is
// one hash probe; the summary for (group, topics?, apiKey) settles most
// requests with two bit tests; the rest walk exception rules and, per topic,
// the (group, topic) rule list.  Counters accumulate per lane while the
// redirect stays the same and are wave-reduced at the end.
__global__ __launch_bounds__(256) void kafka_kernel(KafkaDev T, const uint4* __restrict__ reqs, size_t n,
                                                    const uint32_t* __restrict__ arena, uint8_t* __restrict__ out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t cred = ~0u, callow = 0, cdeny = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint4* r = reqs + i * 4;
    const uint4 h = r[0];
    const uint4 t0 = r[1], t1 = r[2], t2 = r[3];
    const int key = (int16_t)(h.x & 0xFFFF);
    const int ver = (int16_t)(h.x >> 16);
    const uint32_t kind = h.y & 0xFF;
    const uint32_t nt = (h.y >> 8) & 0xFF;
    const uint32_t red = h.y >> 16;
    const uint32_t remote = h.z;
    const uint32_t client = h.w;
    uint32_t v = 0;
    if (red < T.nredirects) {
      uint32_t g = T.dflt_group[red];
      if (remote != 0) {
        const unsigned long long k = ((unsigned long long)red << 32) | remote;
        uint32_t hh = hash64to32(k) & T.ghash_mask;
        for (uint32_t probe = 0; probe <= T.ghash_mask; ++probe) {
          const unsigned long long kk = T.ghash_keys[hh];
          if (kk == k) {
            g = T.ghash_vals[hh];
            break;
          }
          if (kk == ~0ULL) break;
          hh = (hh + 1) & T.ghash_mask;
        }
      }
      const uint32_t b = (key >= 0 && key < 64) ? (uint32_t)key : 64u;
      const KafkaSumDev* su = T.sums + (size_t)g * kKfSumsPerGroup + (nt == 0 ? kKfBuckets : 0) + b;
      const uint32_t c = kind == CG_KAFKA_K_TYPED ? 0 : kind == CG_KAFKA_K_CONSUMER_METADATA ? 1 : 2;
      const uint4 tail = *reinterpret_cast<const uint4*>(&su->any);
      const unsigned long long vm = su->vm[c];
      v = ((tail.x >> c) & 1) | ((ver >= 0 && ver < 64) ? (uint32_t)((vm >> ver) & 1) : 0u);
      for (uint32_t j = 0; j < tail.z && !v; ++j)
        if (kf_rule_matches(T.rules[tail.y + j], key, ver, kind, client)) v = 1;
      if (!v && nt != 0) {
        const uint32_t tids[CG_KAFKA_MAX_TOPICS] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y,
                                                    t1.z, t1.w, t2.x, t2.y, t2.z, t2.w};
        const bool ovf = nt > CG_KAFKA_MAX_TOPICS;
        bool all = true;
        for (uint32_t t = 0; t < nt && all; ++t) {
          const uint32_t tid = ovf ? arena[tids[0] + t] : tids[t];
          const unsigned long long k = ((unsigned long long)g << 32) | tid;
          uint32_t hh = hash64to32(k) & T.thash_mask;
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
          all = cov;
        }
        v = all ? 1 : 0;
      }
      if (red != cred) {
        if (cred != ~0u) kf_flush(T.counters, cred, callow, cdeny);
        cred = red;
        callow = cdeny = 0;
      }
      callow += v;
      cdeny += v ^ 1;
    }
    out[i] = (uint8_t)v;
  }
  // the common case: every lane of the wave counted for the same redirect
  const uint32_t first = __builtin_amdgcn_readfirstlane(cred);
  if (__all(cred == first)) {
    for (int o = 32; o > 0; o >>= 1) {
      callow += __shfl_down(callow, o, kWave);
      cdeny += __shfl_down(cdeny, o, kWave);
    }
    if ((threadIdx.x & 63) == 0 && first != ~0u) kf_flush(T.counters, first, callow, cdeny);
  } else if (cred != ~0u) {
    kf_flush(T.counters, cred, callow, cdeny);
  }
}

int grid_for(size_t items, int per_block, int cus, int blocks_per_cu) {
  size_t need = (items + per_block - 1) / per_block;
  size_t cap = (size_t)cus * blocks_per_cu;
  if (need > cap) need = cap;
  if (need < 1) need = 1;
  return (int)need;
}

}  // namespace

int launch_l4(const L4Dev& t, const void* tuples, size_t n, int32_t* out, void* stream, int cus) {
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (t.max_entries <= 16384) {
    size_t lds = (size_t)t.max_entries * 2 * sizeof(uint32_t);
    static bool attr_set = false;
    if (!attr_set) {
      hipFuncSetAttribute((const void*)l4_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr_set = true;
    }
    hipLaunchKernelGGL(l4_kernel<true>, dim3(grid_for(n, 1024, cus, 1)), dim3(1024), lds, s, t,
                       (const uint32_t*)tuples, n, out);
  } else {
    hipLaunchKernelGGL(l4_kernel<false>, dim3(grid_for(n, 1024, cus, 2)), dim3(1024), 0, s, t,
                       (const uint32_t*)tuples, n, out);
  }
  return (int)hipGetLastError();
}

int launch_lpm(const LpmDev& t, bool v4f, bool v6f, const uint32_t* v4, size_t n4, uint8_t* out4,
               const uint8_t* v6, size_t n6, uint8_t* out6, void* stream, int cus) {
  if (n4 + n6 == 0) return 0;
  hipLaunchKernelGGL(lpm_kernel, dim3(grid_for(n4 + n6, 256, cus, 8)), dim3(256), 0, (hipStream_t)stream, t, v4f,
                     v6f, (const uint2*)v4, n4, out4, (const uint4*)v6, n6, out6);
  return (int)hipGetLastError();
}

int launch_kafka(const KafkaDev& t, const void* reqs, size_t n, const uint32_t* arena, uint8_t* out,
                 void* stream, int cus) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(kafka_kernel, dim3(grid_for(n, 256, cus, 8)), dim3(256), 0, (hipStream_t)stream, t,
                     (const uint4*)reqs, n, arena, out);
  return (int)hipGetLastError();
}

}  // namespace cg
