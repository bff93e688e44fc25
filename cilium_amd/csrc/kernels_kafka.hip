// kernels_kafka.hip — Kafka request decoding on the GPU.
//
// One lane per request runs kw_decode (kafka_wire.h, the restatement of
// ReadRequest and the optiopay/kafka decoders it calls) on the request's own
// bytes in HBM and writes its cg_kafka_request record (64 B) for the
// verdict kernel.  Topic and clientID strings are interned against the
// snapshot's rule-string dictionaries (FNV-1a open addressing, the bytes
// compared against the dictionary blob).  Produce message sets are parsed in
// full: each message's CRC-32 is computed slicing-by-8 from tables in LDS
// (8 KiB per block), the request's bytes read as aligned dwords.  A request
// whose message set holds a gzip / snappy message ends as kKwDefer; the host
// decodes those (cg_kafka_decode_dev, capi.cc).
//
// Topic lists longer than CG_KAFKA_MAX_TOPICS go to the arena: the first pass
// learns the count, then a second pass of that request (only) writes the ids
// at an offset reserved with one 64-bit atomic.  Requests declaring more
// topics than they carry fail in pass 1 and reserve nothing, so the arena a
// batch needs is bounded by its bytes / 2.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kafka_wire.h"
#include "kernels.h"

namespace cg {
namespace {

constexpr uint32_t kKwThreads = 256;

// CRC-32 (IEEE, reflected), slicing-by-8 over tables t[k][256] in LDS.
struct LdsCrc {
  const uint32_t* t;
  __device__ uint32_t operator()(const uint8_t* p, uint32_t n) const {
    uint32_t c = 0xFFFFFFFFu;
    while (n && ((uintptr_t)p & 3)) {
      c = t[(c ^ *p++) & 0xFF] ^ (c >> 8);
      --n;
    }
    for (; n >= 8; n -= 8, p += 8) {
      const uint32_t a = *reinterpret_cast<const uint32_t*>(p) ^ c;
      const uint32_t b = *reinterpret_cast<const uint32_t*>(p + 4);
      c = t[7 * 256 + (a & 0xFF)] ^ t[6 * 256 + ((a >> 8) & 0xFF)] ^ t[5 * 256 + ((a >> 16) & 0xFF)] ^
          t[4 * 256 + (a >> 24)] ^ t[3 * 256 + (b & 0xFF)] ^ t[2 * 256 + ((b >> 8) & 0xFF)] ^
          t[256 + ((b >> 16) & 0xFF)] ^ t[b >> 24];
    }
    while (n--) c = t[(c ^ *p++) & 0xFF] ^ (c >> 8);
    return ~c;
  }
};

__device__ uint32_t kw_intern(const KafkaDictDev& d, const uint8_t* p, uint32_t n) {
  const uint32_t h = kf_fnv1a(p, n);
  uint32_t s = h & d.mask;
  for (uint32_t k = 0; k <= d.mask; ++k, s = (s + 1) & d.mask) {
    const uint4 e = *reinterpret_cast<const uint4*>(d.slots + (size_t)s * 4);
    if (e.y == kKfDictEmpty) break;
    if (e.x == h && e.y == n) {
      uint32_t j = 0;
      while (j < n && d.blob[e.z + j] == p[j]) ++j;
      if (j == n) return e.w;
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

__global__ __launch_bounds__(kKwThreads) void kafka_decode_kernel(
    KafkaDictDev dt, KafkaDictDev dc, const uint8_t* __restrict__ raw, const uint64_t* __restrict__ off, size_t n,
    const uint16_t* __restrict__ redirect, const uint32_t* __restrict__ remote, uint4* __restrict__ recs,
    uint32_t* __restrict__ arena, unsigned long long arena_cap, unsigned long long* __restrict__ ctr,
    uint8_t* __restrict__ status) {
  __shared__ uint32_t s_crc[8 * 256];
  for (uint32_t i = threadIdx.x; i < 256; i += kKwThreads) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    s_crc[i] = c;
  }
  __syncthreads();
  for (uint32_t k = 1; k < 8; ++k) {
    for (uint32_t i = threadIdx.x; i < 256; i += kKwThreads) {
      const uint32_t prev = s_crc[(k - 1) * 256 + i];
      s_crc[k * 256 + i] = (prev >> 8) ^ s_crc[prev & 0xFF];
    }
    __syncthreads();
  }
  const LdsCrc crc{s_crc};
  const size_t stride = (size_t)gridDim.x * kKwThreads;
  for (size_t i = (size_t)blockIdx.x * kKwThreads + threadIdx.x; i < n; i += stride) {
    const uint64_t a = off[i], b = off[i + 1];
    const uint64_t len64 = b > a ? b - a : 0;
    const uint32_t len = len64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len64;
    const uint8_t* p = raw + a;
    const uint32_t red = redirect[i], rem = remote[i];
    uint4* rec = recs + i * 4;
    const uint4 zero = make_uint4(0, 0, 0, 0);
    rec[1] = zero;
    rec[2] = zero;
    rec[3] = zero;
    KwRequest r;
    DevSink sink{&dt, p, reinterpret_cast<uint32_t*>(rec + 1), CG_KAFKA_MAX_TOPICS, CG_KAFKA_MAX_TOPICS};
    uint8_t st = kw_decode(p, len, crc, &r, sink, DevDefer{});
    uint32_t nt = sink.nt, t0 = 0, t1 = 0;
    if (st == kKwOk && nt > CG_KAFKA_MAX_TOPICS) {
      const unsigned long long at = atomicAdd(ctr, (unsigned long long)nt);
      const bool fits = at + nt <= arena_cap;
      KwRequest r2;
      DevSink s2{&dt, p, arena + (fits ? at : 0), fits ? nt : 0u, 0xFFFFFFFFu};
      kw_decode(p, len, crc, &r2, s2, DevDefer{});
      t0 = (uint32_t)at;
      t1 = nt >= CG_KAFKA_TOPICS_IN_ARENA ? nt : 0;
    }
    if (st == kKwDefer) atomicAdd(ctr + 1, 1ull);
    uint4 h;
    if (st == kKwOk) {
      const uint32_t ntb = nt < CG_KAFKA_TOPICS_IN_ARENA ? nt : CG_KAFKA_TOPICS_IN_ARENA;
      h = make_uint4((uint32_t)(uint16_t)r.api_key | (uint32_t)(uint16_t)r.version << 16,
                     (uint32_t)r.cls | ntb << 8 | red << 16, rem,
                     kw_intern(dc, p + r.client_off, r.client_len));
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
}

}  // namespace

int launch_kafka_decode(const KafkaDictDev& topics, const KafkaDictDev& clients, const uint8_t* raw,
                        const uint64_t* off, size_t n, const uint16_t* redirect, const uint32_t* remote, void* recs,
                        uint32_t* arena, size_t arena_cap, unsigned long long* ctr, uint8_t* status, void* stream,
                        int cus) {
  if (n == 0) return hipSuccess;
  const size_t need = (n + kKwThreads - 1) / kKwThreads;
  const int grid = (int)std::min<size_t>(need, (size_t)std::max(cus, 1) * 8);
  hipLaunchKernelGGL(kafka_decode_kernel, dim3(grid), dim3(kKwThreads), 0, (hipStream_t)stream, topics, clients,
                     raw, off, n, redirect, remote, (uint4*)recs, arena, (unsigned long long)arena_cap, ctr, status);
  return hipGetLastError();
}

}  // namespace cg
