// kernels_kafka.hip — Kafka request decoding on the GPU.
//
// One lane per request runs kw_decode (kafka_wire.h, the restatement of
// ReadRequest and the optiopay/kafka decoders it calls) on the request's own
// bytes in HBM and writes its cg_kafka_request record (64 B) for the
// verdict kernel.  Topic and clientID strings are interned against the
// snapshot's rule-string dictionaries (FNV-1a open addressing, the bytes
// compared against the dictionary blob).  Produce message sets are parsed in
// full: each message's CRC-32 is computed slicing-by-8 from tables in LDS
// (8 KiB per block), the request's bytes read as aligned dwords.  A gzip /
// snappy message's payload is decoded on the device too (DevInflate,
// kw_inflate.h); the few the device cannot finish end as kKwDefer and the
// host decodes those requests (cg_kafka_decode_dev, capi.cc).
//
// Topic lists longer than CG_KAFKA_MAX_TOPICS go to the arena: the first pass
// learns the count, then a second pass of that request (only) writes the ids
// at an offset reserved with one 64-bit atomic.  Requests declaring more
// topics than they carry fail in pass 1 and reserve nothing, so the arena a
// batch needs is bounded by its bytes / 2.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>

#include "kafka_wire.h"
#include "kernels.h"
#include "kw_inflate.h"

namespace cg {
namespace {

constexpr uint32_t kKwThreads = 256;
constexpr uint32_t kKwWaves = kKwThreads / 64;
// per-wave LDS stage of the wave's 64 requests (bytes; 0 = none): requests
// reaching past it read HBM directly
// (a template parameter of the kernel: 4, 8 or 16 KiB, CILIUM_GPU_KAFKA_STAGE_KB
// for the A/B; 4 KiB by default — measured 2.65 / 2.43 / 2.09 G requests/s:
// the occupancy a larger stage costs outweighs the HBM reads it saves,
// profiles/r06ze_kafka_stage_ab.txt)
// CRC-32 tables (slicing-by-kKwSlices, kKwSlices KiB of LDS per block)
constexpr uint32_t kKwSlices = 8;

// CRC-32 (IEEE, reflected), slicing-by-kKwSlices over tables t[k][256] in
// LDS: byte j of a kKwSlices-byte block goes through table kKwSlices-1-j.
// The unaligned head and the tail (< kKwSlices bytes) go through the same
// tables up to 4 bytes per step, so no per-byte dependency chain remains.
struct LdsCrc {
  const uint32_t* t;
  // r (0..4) bytes of p in one step
  __device__ __forceinline__ uint32_t small(uint32_t c, const uint8_t* p, uint32_t r) const {
    if (!r) return c;
    uint32_t d = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t v = p[k < r ? k : r - 1];
      d |= (k < r ? v : 0u) << (8 * k);
    }
    const uint32_t x = c ^ d;
    uint32_t o = r == 4 ? 0u : c >> (8 * r);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
      if (j < r) o ^= t[(r - 1 - j) * 256 + ((x >> (8 * j)) & 0xFF)];
    return o;
  }
  __device__ uint32_t operator()(const uint8_t* p, uint32_t n) const {
    uint32_t c = 0xFFFFFFFFu;
    uint32_t h = (4u - ((uint32_t)(uintptr_t)p & 3u)) & 3u;
    h = h < n ? h : n;
    c = small(c, p, h);
    p += h;
    n -= h;
    for (; n >= kKwSlices; n -= kKwSlices, p += kKwSlices) {
      uint32_t w[kKwSlices / 4];
#pragma unroll
      for (uint32_t q = 0; q < kKwSlices / 4; ++q) w[q] = reinterpret_cast<const uint32_t*>(p)[q];
      w[0] ^= c;
      c = 0;
#pragma unroll
      for (uint32_t j = 0; j < kKwSlices; ++j) c ^= t[(kKwSlices - 1 - j) * 256 + ((w[j / 4] >> (8 * (j % 4))) & 0xFF)];
    }
    while (n) {
      const uint32_t r = n < 4 ? n : 4;
      c = small(c, p, r);
      p += r;
      n -= r;
    }
    return ~c;
  }
};

// Intern p[0, n): FNV-1a over the bytes, one 32-byte slot per probe.  The
// first 16 bytes are loaded with clamped indices (independent loads, no
// per-byte branch) and compared in registers against the slot's copy.
__device__ __forceinline__ uint32_t kw_intern(const KafkaDictDev& d, const uint8_t* p, uint32_t n) {
  uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  uint32_t h = 2166136261u;
  if (n) {
    const uint32_t m = n < 16 ? n : 16;
    uint32_t c[16];
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) c[k] = p[k < m ? k : m - 1];
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      const uint32_t v = k < m ? c[k] : 0u;
      if (k < m) h = (h ^ v) * 16777619u;
      const uint32_t sh = v << (8 * (k & 3));
      if (k < 4) w0 |= sh;
      else if (k < 8) w1 |= sh;
      else if (k < 12) w2 |= sh;
      else w3 |= sh;
    }
    for (uint32_t k = 16; k < n; ++k) h = (h ^ p[k]) * 16777619u;
  }
  uint32_t s = h & d.mask;
  for (uint32_t probe = 0; probe <= d.mask; ++probe, s = (s + 1) & d.mask) {
    const uint4* e = reinterpret_cast<const uint4*>(d.slots + (size_t)s * kKfDictSlotWords);
    const uint4 hd = e[0], pre = e[1];
    if (hd.y == kKfDictEmpty) break;
    if (hd.x == h && hd.y == n && pre.x == w0 && pre.y == w1 && pre.z == w2 && pre.w == w3) {
      uint32_t j = 16;
      while (j < n && d.blob[hd.w + j - 16] == p[j]) ++j;
      if (j >= n) return hd.z;
    }
  }
  return CG_KAFKA_UNKNOWN_STR;
}

// GetTopics into dst[0, lim): pass 1 writes the record's inline ids when the
// list fits (lim = 0 otherwise), pass 2 the arena entries.
struct DevSink {
  const KafkaDictDev* d;
  const uint8_t* raw;
  uint32_t* dst;
  uint32_t lim, inline_lim;
  uint32_t k = 0, nt = 0;
  __device__ void begin(int32_t n) {
    nt = (uint32_t)n;
    if (nt > inline_lim) lim = 0;
  }
  __device__ void topic(uint32_t o, uint32_t n) {
    if (k < lim) dst[k] = kw_intern(*d, raw + o, n);
    ++k;
  }
};

struct DevDefer {
  __device__ uint8_t operator()(uint32_t, const uint8_t*, uint32_t, int16_t) const { return kKwDefer; }
};
// A second pass over a request whose first pass returned kKwOk (its inner
// sets were decoded and validated then): the outer topic list is all it
// needs, so compressed payloads are passed over — the set's next message
// follows from the outer framing alone — and no arena space is reserved
// again.
// One atomic per wave for the active lanes that want a slot of a shared
// counter (a returning atomic per lane on one address serializes at the L2:
// hundreds of thousands of them per call), each lane's index by its rank
// among them.  Called by every active lane together (divergence is fine: the
// ballot is over the lanes active here).
__device__ __forceinline__ unsigned long long wave_append(unsigned long long* ctr, bool want) {
  const unsigned long long m = __ballot(want);
  if (!m) return 0;
  const uint32_t lane = __lane_id(), leader = (uint32_t)__builtin_ctzll(m);
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(m));
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)base, (int)leader, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(base >> 32), (int)leader, 64);
  return ((unsigned long long)hi << 32 | lo) + (unsigned long long)__popcll(m & ((1ull << lane) - 1));
}

struct DevValidated {
  __device__ uint8_t operator()(uint32_t, const uint8_t*, uint32_t, int16_t) const { return kKwOk; }
};

// A compressed message's payload decoded on the device (kw_inflate.h) into a
// reservation of the call's inflate arena, then its inner set parsed
// (messages.go:460-480).  The reservation is sized before decoding: gzip from
// the member's trailing ISIZE, snappy from its length varint(s).  What the
// device does not finish goes to the host decoder (kKwDefer): a payload it
// cannot size, a full arena, a second gzip member, output past the sized
// buffer, and compressed sets nested inside compressed sets.
// A payload that decodes to at most kInfLds bytes (most of a Kafka produce
// request's sets: a few small messages) is decoded into the lane's LDS
// buffer instead: the inflater's back-references read what it just wrote,
// and a byte written to HBM and read back costs an L2 round trip, in LDS a
// few dozen cycles.  The inner set is only validated, never kept, so
// nothing is copied out.
constexpr uint32_t kInfLds = 256, kInfLdsStride = 260;  // (65 words: lanes at one offset hit distinct banks)
struct DevInflate {
  uint8_t* arena;
  unsigned long long cap;
  unsigned long long* used;  // bytes reserved (ctr[2])
  unsigned long long* done;  // payloads decoded on the device (ctr[3])
  unsigned long long* full;  // payloads deferred unreserved: arena full or an impossible size (ctr[5])
  const LdsCrc* crc;
  uint8_t* lds_out;  // this lane's kInfLds bytes of LDS, or nullptr
  __device__ uint8_t operator()(uint32_t codec, const uint8_t* p, uint32_t n, int16_t version) const {
    if (!arena) return kKwDefer;
    uint64_t need = 0;
    if (codec == 1) {
      if (n >= 4) need = (uint64_t)p[n - 4] | (uint64_t)p[n - 3] << 8 | (uint64_t)p[n - 2] << 16 | (uint64_t)p[n - 1] << 24;
    } else if (!kwz::snappy_size(p, n, &need)) {
      return kKwDefer;
    }
    if (need > kKafkaMaxParseBuf) return kKwDefer;
    // a size no payload of n bytes decodes to (DEFLATE expands at most
    // 1032:1, a snappy copy op 64 bytes from 3): the host decoder decides,
    // and the sender's claim reserves nothing
    if (need > (uint64_t)n * (codec == 1 ? 1032u : 32u) + 64u) {
      atomicAdd(full, 1ull);
      return kKwDefer;
    }
    uint8_t* dst = lds_out;
    if (!lds_out || need > kInfLds) {
      const unsigned long long at = atomicAdd(used, (unsigned long long)need);
      if (at + need > cap) {
        atomicAdd(full, 1ull);
        return kKwDefer;
      }
      dst = arena + at;
    }
    uint32_t got = 0;
    const int r = codec == 1 ? kwz::gunzip_one(p, n, dst, (uint32_t)need, &got, *crc)
                             : kwz::snappy_go(p, n, dst, (uint32_t)need, &got);
    if (r == kwz::kKwzMore) return kKwDefer;
    if (r != kwz::kKwzOk) return kKwError;
    (void)wave_append(done, true);
    KwStream inner{dst, got, 0};
    return kw_message_set(&inner, (int32_t)got, version, *crc, DevDefer{});
  }
};

// One request: decode from p (its bytes, in LDS or HBM), write the record
// and status.
template <class Inflate>
__device__ __forceinline__ void decode_one(const KafkaDictDev& dt, const KafkaDictDev& dc, const LdsCrc& crc,
                                           const uint8_t* p, uint32_t len, size_t i, uint32_t red, uint32_t rem,
                                           uint4* __restrict__ recs, uint32_t* __restrict__ arena,
                                           unsigned long long arena_cap, unsigned long long* __restrict__ ctr,
                                           uint8_t* __restrict__ status, const Inflate& inflate,
                                           unsigned long long* defer_ctr, uint32_t* defer_list) {
  uint4* rec = recs + i * 4;
  const uint4 zero = make_uint4(0, 0, 0, 0);
  rec[1] = zero;
  rec[2] = zero;
  rec[3] = zero;
  KwRequest r;
  DevSink sink{&dt, p, reinterpret_cast<uint32_t*>(rec + 1), CG_KAFKA_MAX_TOPICS, CG_KAFKA_MAX_TOPICS};
  uint8_t st = kw_decode(p, len, crc, &r, sink, inflate);
  uint32_t nt = sink.nt, t0 = 0, t1 = 0;
  if (st == kKwOk && nt > CG_KAFKA_MAX_TOPICS) {
    const unsigned long long at = atomicAdd(ctr, (unsigned long long)nt);
    const bool fits = at + nt <= arena_cap;
    KwRequest r2;
    DevSink s2{&dt, p, arena + (fits ? at : 0), fits ? nt : 0u, 0xFFFFFFFFu};
    // the same outcome as pass 1 by construction; anything else would leave
    // topic ids unwritten, so it goes to the host decoder
    if (kw_decode(p, len, crc, &r2, s2, DevValidated{}) != kKwOk || s2.nt != nt) st = kKwDefer;
    t0 = (uint32_t)at;
    t1 = nt >= CG_KAFKA_TOPICS_IN_ARENA ? nt : 0;
  }
  {
    const unsigned long long j = wave_append(defer_ctr, st == kKwDefer);
    if (st == kKwDefer && defer_list) defer_list[j] = (uint32_t)i;
  }
  uint4 h;
  if (st == kKwOk) {
    const uint32_t ntb = nt < CG_KAFKA_TOPICS_IN_ARENA ? nt : CG_KAFKA_TOPICS_IN_ARENA;
    h = make_uint4((uint32_t)(uint16_t)r.api_key | (uint32_t)(uint16_t)r.version << 16,
                   (uint32_t)r.cls | ntb << 8 | red << 16, rem, kw_intern(dc, p + r.client_off, r.client_len));
    if (nt > CG_KAFKA_MAX_TOPICS) rec[1] = make_uint4(t0, t1, 0, 0);
  } else {
    // ReadRequest failed: a record that is denied.  A deferred one keeps
    // its redirect for the host decoder, which rewrites the record.
    h = make_uint4(0, CG_KAFKA_K_NIL | (st == kKwDefer ? red : 0xFFFFu) << 16, rem, 0);
    if (sink.k) {  // topics pass 1 stored before the error
      rec[1] = zero;
      rec[2] = zero;
      rec[3] = zero;
    }
  }
  rec[0] = h;
  status[i] = st;
}

template <uint32_t kKwStage>
__global__ __launch_bounds__(kKwThreads) void kafka_decode_kernel(
    KafkaDictDev dt, KafkaDictDev dc, const uint8_t* __restrict__ raw, const uint64_t* __restrict__ off, size_t n,
    const uint16_t* __restrict__ redirect, const uint32_t* __restrict__ remote, uint4* __restrict__ recs,
    uint32_t* __restrict__ arena, unsigned long long arena_cap, unsigned long long* __restrict__ ctr,
    uint8_t* __restrict__ status, uint32_t* __restrict__ defer_list) {
  __shared__ uint32_t s_crc[kKwSlices * 256];
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[kKwWaves][kKwStage ? kKwStage : 16];
  for (uint32_t i = threadIdx.x; i < 256; i += kKwThreads) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    s_crc[i] = c;
  }
  __syncthreads();
  for (uint32_t k = 1; k < kKwSlices; ++k) {
    for (uint32_t i = threadIdx.x; i < 256; i += kKwThreads) {
      const uint32_t prev = s_crc[(k - 1) * 256 + i];
      s_crc[k * 256 + i] = (prev >> 8) ^ s_crc[prev & 0xFF];
    }
    __syncthreads();
  }
  const LdsCrc crc{s_crc};
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint8_t* stage = s_stage[wid];
  const size_t groups = (n + 63) / 64;
  for (size_t g = (size_t)blockIdx.x * kKwWaves + wid; g < groups; g += (size_t)gridDim.x * kKwWaves) {
    const size_t i0 = g * 64, i = i0 + lane;
    const bool live = i < n;
    const size_t last = i0 + 63 < n ? i0 + 63 : n - 1;
    const uint64_t a = off[live ? i : last], b = off[(live ? i : last) + 1];
    // the wave's bytes [off[i0], off[last+1]) (every byte of it belongs to
    // some request when the end is above the start), up to kKwStage of them
    // from a 16-byte boundary of the POINTER, loaded coalesced into this
    // wave's LDS stage.  Only bytes inside [start, end) are read: blocks that
    // straddle either end go byte by byte, so a d_raw buffer that ends
    // exactly at raw_off[n] (or starts unaligned) is never overrun.
    const int64_t start = (int64_t)off[i0], end = (int64_t)off[last + 1];
    const int64_t lo = start - (int64_t)(((uintptr_t)raw + (uint64_t)start) & 15);
    int64_t hi = end > start ? end : start;
    hi = lo + ((hi - lo + 15) & ~(int64_t)15);
    if (hi > lo + kKwStage) hi = lo + kKwStage;
    if (kKwStage) {
      for (int64_t x = lo + lane * 16; x < hi; x += 64 * 16) {
        if (x >= start && x + 16 <= end) {
          *reinterpret_cast<uint4*>(stage + (x - lo)) = *reinterpret_cast<const uint4*>(raw + x);
        } else {
          for (int k = 0; k < 16; ++k)
            if (x + k >= start && x + k < end) stage[x - lo + k] = raw[x + k];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const uint64_t len64 = b > a ? b - a : 0;
    const uint32_t len = len64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len64;
    const bool staged = kKwStage && (int64_t)a >= lo && (int64_t)(a + len) <= hi;
    // one copy of the decoder over flat addresses (a wave-uniform split into
    // an LDS copy and an HBM copy measured slower: twice the code)
    if (live)
      decode_one(dt, dc, crc, staged ? stage + ((int64_t)a - lo) : raw + a, len, i, redirect[i], remote[i], recs, arena,
                 arena_cap, ctr, status, DevDefer{}, ctr + 1, defer_list);
    // every lane has read its bytes before the stage is refilled
    __builtin_amdgcn_wave_barrier();
  }
}

// The requests the decode kernel deferred (defer_list[0, ctr[1])): decoded
// again, one lane each from HBM, with their compressed payloads decoded on
// the device (DevInflate).  A separate kernel, so the inflate code's
// registers and scratch do not set the common decoder's occupancy.  What it
// still defers (ctr[4]) the host decodes.
__global__ __launch_bounds__(kKwThreads) void kafka_inflate_kernel(
    KafkaDictDev dt, KafkaDictDev dc, const uint8_t* __restrict__ raw, const uint64_t* __restrict__ off,
    const uint16_t* __restrict__ redirect, const uint32_t* __restrict__ remote, uint4* __restrict__ recs,
    uint32_t* __restrict__ arena, unsigned long long arena_cap, unsigned long long* __restrict__ ctr,
    uint8_t* __restrict__ status, const uint32_t* __restrict__ defer_list, uint8_t* __restrict__ zarena,
    unsigned long long zcap) {
  __shared__ uint32_t s_crc[kKwSlices * 256];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kKwThreads * kInfLdsStride];
  const unsigned long long nd = ctr[1];
  if (nd == 0) return;  // uniform: the common case
  for (uint32_t i = threadIdx.x; i < 256; i += kKwThreads) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    s_crc[i] = c;
  }
  __syncthreads();
  for (uint32_t k = 1; k < kKwSlices; ++k) {
    for (uint32_t i = threadIdx.x; i < 256; i += kKwThreads) {
      const uint32_t prev = s_crc[(k - 1) * 256 + i];
      s_crc[k * 256 + i] = (prev >> 8) ^ s_crc[prev & 0xFF];
    }
    __syncthreads();
  }
  const LdsCrc crc{s_crc};
  const DevInflate inflate{zarena, zcap, ctr + 2, ctr + 3, ctr + 5, &crc, s_out + threadIdx.x * kInfLdsStride};
  for (unsigned long long j = (unsigned long long)blockIdx.x * kKwThreads + threadIdx.x; j < nd;
       j += (unsigned long long)gridDim.x * kKwThreads) {
    const uint32_t i = defer_list[j];
    const uint64_t a = off[i], b = off[i + 1];
    const uint64_t len64 = b > a ? b - a : 0;
    const uint32_t len = len64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len64;
    decode_one(dt, dc, crc, raw + a, len, i, redirect[i], remote[i], recs, arena, arena_cap, ctr, status, inflate,
               ctr + 4, (uint32_t*)nullptr);
  }
}

}  // namespace

int launch_kafka_decode(const KafkaDictDev& topics, const KafkaDictDev& clients, const uint8_t* raw,
                        const uint64_t* off, size_t n, const uint16_t* redirect, const uint32_t* remote, void* recs,
                        uint32_t* arena, size_t arena_cap, unsigned long long* ctr, uint8_t* status, void* stream,
                        int cus, uint32_t* defer_list, uint8_t* zarena, size_t zcap) {
  if (n == 0) return hipSuccess;
  const size_t need = (n + kKwThreads - 1) / kKwThreads;  // one 64-request group per wave
  const int grid = (int)std::min<size_t>(need, (size_t)std::max(cus, 1) * (4096 / kKwThreads));
  const char* sk = getenv("CILIUM_GPU_KAFKA_STAGE_KB");
  const int kb = sk ? atoi(sk) : 4;
  auto k = kb == 8 ? kafka_decode_kernel<8192> : kb == 16 ? kafka_decode_kernel<16384> : kafka_decode_kernel<4096>;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kKwThreads), 0, (hipStream_t)stream, topics, clients, raw, off, n, redirect,
                     remote, (uint4*)recs, arena, (unsigned long long)arena_cap, ctr, status, defer_list);
  // the deferred requests (their count stays on the device: a small grid
  // that exits at once when there are none) — two workgroups per CU, the
  // inflater's occupancy (230 VGPRs: 2 waves per SIMD)
  hipLaunchKernelGGL(kafka_inflate_kernel, dim3(2 * (unsigned)std::max(cus, 1)), dim3(kKwThreads), 0, (hipStream_t)stream,
                     topics, clients, raw, off, redirect, remote, (uint4*)recs, arena, (unsigned long long)arena_cap,
                     ctr, status, defer_list, zarena, (unsigned long long)zcap);
  return hipGetLastError();
}

}  // namespace cg
