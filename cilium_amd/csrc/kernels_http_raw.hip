// kernels_http_raw.hip — HTTP/1 request heads straight from HBM into the
// http_kernel batch format (gfx950), so raw request streams go from device
// memory to verdicts without the host parser and packer.
//
// The steps of http_parse.cc (the codec: request line, header fields, Host →
// :authority, rejected heads) and http_pack.cc (program lookup, the walked
// string v_1 SEP .. v_F SEP / REST, class codes, grouping by program and
// string units) run one lane per request:
//   raw_scan_kernel   parse (value spans kept); program, string length, bucket key (program
//                     group × string units) and the bucket histogram
//   (host)            bucket counts → groups, chunks, bucket cursors
//   raw_tiles_kernel  tile table (fixed 17-granule stride per tile, units =
//                     the largest walked string the tile holds), padding slots
//   raw_emit_kernel   the scan's value spans; a slot from the bucket cursor; meta, the
//                     class-coded string units (zero padded) or an overflow
//                     arena entry; the tile's tail bytes
//   http_kernel       the verdicts (kernels_http.hip)
//   raw_scatter       slot verdicts back to request order
// Slots within a bucket come in atomic order: the verdicts are per request,
// so they do not depend on it.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/cilium_gpu.h"
#include "dev_types.h"
#include "kernels.h"

namespace cg {

namespace {

constexpr int kRawThreads = 256;
constexpr uint32_t kAbsentSpan = 0xFFFFFFFFu;

// RFC 7230 tchar as two 64-bit masks (bytes 0..63, 64..127)
constexpr uint64_t tchar_lo() {
  uint64_t m = 0;
  for (char c : {'!', '#', '$', '%', '&', '\'', '*', '+', '-', '.'}) m |= 1ull << c;
  for (int c = '0'; c <= '9'; ++c) m |= 1ull << c;
  return m;
}
constexpr uint64_t tchar_hi() {
  uint64_t m = 0;
  for (int c = 'A'; c <= 'Z'; ++c) m |= 1ull << (c - 64);
  for (int c = 'a'; c <= 'z'; ++c) m |= 1ull << (c - 64);
  for (char c : {'^', '_', '`', '|', '~'}) m |= 1ull << (c - 64);
  return m;
}
__device__ __forceinline__ bool tchar(uint32_t c) {
  return c < 64 ? (tchar_lo() >> c) & 1 : c < 128 ? (tchar_hi() >> (c - 64)) & 1 : false;
}
__device__ __forceinline__ uint32_t lower(uint32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

// Four bytes that are all "plain": > 0x20 and not 0x7F (no control byte, no
// SP / HTAB / CR): target and field-value bytes that need no decision.
// hasless(q, 0x21) and haszero(q ^ 0x7F..) are exact presence tests.
__device__ __forceinline__ bool all_plain(uint32_t q) {
  const uint32_t lt = (q - 0x21212121u) & ~q & 0x80808080u;
  const uint32_t y = q ^ 0x7F7F7F7Fu;
  const uint32_t del = (y - 0x01010101u) & ~y & 0x80808080u;
  return (lt | del) == 0;
}

// A lane's head: from its wave's LDS stage when the head lies inside it
// (the common case), else through 16-byte aligned global loads with one
// block kept in registers (blocks reaching outside the head are assembled
// from byte loads of the head's own bytes).
struct HeadReader {
  const uint8_t* p;
  uint32_t n;
  const uint8_t* lp;  // the head in LDS, or nullptr
  uint64_t cur;
  uint4 w;
  __device__ __forceinline__ HeadReader(const uint8_t* p_, uint32_t n_, const uint8_t* lp_)
      : p(p_), n(n_), lp(lp_), cur(~0ull), w{0, 0, 0, 0} {}
  // bytes k..k+3 (little-endian; bytes past the head are unspecified): from
  // LDS two aligned dword reads and a byte align, so a walk pays one LDS
  // round trip per 4 bytes instead of one per byte
  __device__ __forceinline__ uint32_t quad(uint32_t k) {
    if (lp) {
      const uintptr_t a = (uintptr_t)(lp + k);
      const uint32_t* w4 = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
      return __builtin_amdgcn_alignbyte(w4[1], w4[0], (uint32_t)(a & 3));
    }
    uint32_t q = 0;  // global: never past the head (it may end the buffer)
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
      if (k + j < n) q |= at(k + j) << (8 * j);
    return q;
  }
  __device__ __forceinline__ uint32_t at(uint32_t k) {
    if (lp) return lp[k];
    const uint64_t a = (uint64_t)(uintptr_t)(p + k);
    const uint64_t blk = a & ~15ull;
    if (blk != cur) {
      cur = blk;
      const uint64_t lo = (uint64_t)(uintptr_t)p, hi = lo + n;
      if (blk >= lo && blk + 16 <= hi) {
        w = *reinterpret_cast<const uint4*>((uintptr_t)blk);
      } else {
        uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          const uint64_t x = blk + b;
          const uint32_t byte = (x >= lo && x < hi) ? *reinterpret_cast<const uint8_t*>((uintptr_t)x) : 0u;
          const uint32_t sh = (b & 3) * 8;
          if (b < 4) v0 |= byte << sh;
          else if (b < 8) v1 |= byte << sh;
          else if (b < 12) v2 |= byte << sh;
          else v3 |= byte << sh;
        }
        w = make_uint4(v0, v1, v2, v3);
      }
    }
    const uint32_t o = (uint32_t)(a & 15);
    const uint32_t d = o >> 2;
    // masks, not a select chain: the compiler turns that into a scratch array
    const uint32_t x = (w.x & (0u - (d == 0))) | (w.y & (0u - (d == 1))) | (w.z & (0u - (d == 2))) |
                       (w.w & (0u - (d == 3)));
    return (x >> ((o & 3) * 8)) & 0xFFu;
  }
};

// The wave's 64 consecutive heads [off[i0], off[i1]) copied into its LDS
// stage (kStage bytes) with coalesced 16-byte loads: returns the global
// address the stage starts at (16-byte aligned) and, in *len, the bytes it
// holds.  Bytes outside the heads' range are loaded byte-wise, only those
// inside it.
// 6 KiB: 64 heads of ~70 B fit with room to spare (heads past the stage are
// read from HBM), and four waves' stages leave room for 3+ workgroups per CU
// (8 KiB: 1.69, 6 KiB: 2.01, 4 KiB: 1.12 G requests/s on config 5)
constexpr uint32_t kStage = 6144;
__device__ __forceinline__ uint64_t stage_heads(const uint8_t* __restrict__ raw, uint64_t lo, uint64_t hi,
                                                uint8_t* stage, uint32_t lane, uint32_t* len) {
  const uint64_t glo = (uint64_t)(uintptr_t)(raw + lo), ghi = (uint64_t)(uintptr_t)(raw + hi);
  const uint64_t a0 = glo & ~15ull;
  const uint32_t nb = (uint32_t)min<uint64_t>((ghi - a0 + 15) & ~15ull, kStage);
  for (uint32_t j = lane * 16; j < nb; j += 64 * 16) {
    const uint64_t a = a0 + j;
    uint4 v;
    if (a >= glo && a + 16 <= ghi) {
      v = *reinterpret_cast<const uint4*>((uintptr_t)a);
    } else {
      uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const uint64_t x = a + b;
        const uint32_t byte = (x >= glo && x < ghi) ? *reinterpret_cast<const uint8_t*>((uintptr_t)x) : 0u;
        const uint32_t sh = (b & 3) * 8;
        if (b < 4) v0 |= byte << sh;
        else if (b < 8) v1 |= byte << sh;
        else if (b < 12) v2 |= byte << sh;
        else v3 |= byte << sh;
      }
      v = make_uint4(v0, v1, v2, v3);
    }
    *reinterpret_cast<uint4*>(stage + j) = v;
  }
  *len = nb;
  return a0;
}

// A wave's LDS writes visible to its own later reads (and its reads done
// before it overwrites the stage)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// The field a header name (lowercase FNV-1a h, length nl, at head offset k)
// is, or -1.
__device__ __forceinline__ int field_of(const HttpRawDev& R, HeadReader& hr, uint32_t h, uint32_t nl, uint32_t k) {
  uint32_t sl = h & R.fmask;
  for (uint32_t probe = 0; probe <= R.fmask; ++probe) {
    const uint4 e = reinterpret_cast<const uint4*>(R.fslots)[sl];
    if (e.y == 0) return -1;
    if (e.x == h && e.y == nl) {
      bool eq = true;
      for (uint32_t j = 0; j < nl && eq; ++j) eq = lower(hr.at(k + j)) == R.fnames[e.w + j];
      if (eq) return (int)e.z;
    }
    sl = (sl + 1) & R.fmask;
  }
  return -1;
}

// parse_head (http_parse.cc) for one head: the value span {start << 16 |
// length} of every field it sets in sp[f * stride] (kAbsentSpan otherwise);
// false = the codec rejects the head.
__device__ __forceinline__ bool parse_head(const HttpRawDev& R, HeadReader& hr, uint32_t* sp, uint32_t stride) {
  for (uint32_t f = 0; f < R.nfields; ++f) sp[f * stride] = kAbsentSpan;
  const uint32_t n = hr.n;
  if (n > kRawMaxHead) return false;
  uint32_t k = 0;
  while (k < n && tchar(hr.at(k))) ++k;  // method
  if (k == 0 || k >= n || hr.at(k) != ' ') return false;
  const uint32_t mlen = k++, t0 = k;
  while (k < n) {  // request-target
    if (k + 4 <= n && all_plain(hr.quad(k))) {
      k += 4;
      continue;
    }
    const uint32_t c = hr.at(k);
    if (c <= 0x20 || c == 0x7F) break;
    ++k;
  }
  if (k == t0 || k >= n || hr.at(k) != ' ') return false;
  const uint32_t tlen = k - t0;
  ++k;
  if (k + 10 > n) return false;  // "HTTP/" DIGIT "." DIGIT CRLF
  {
    const uint32_t d1 = hr.at(k + 5), d2 = hr.at(k + 7);
    if (hr.at(k) != 'H' || hr.at(k + 1) != 'T' || hr.at(k + 2) != 'T' || hr.at(k + 3) != 'P' || hr.at(k + 4) != '/' ||
        d1 < '0' || d1 > '9' || hr.at(k + 6) != '.' || d2 < '0' || d2 > '9' || hr.at(k + 8) != '\r' ||
        hr.at(k + 9) != '\n')
      return false;
  }
  k += 10;
  bool have_host = false;
  uint32_t auth = kAbsentSpan;
  while (true) {
    if (k + 1 >= n) return false;  // no CRLF left: incomplete head
    if (hr.at(k) == '\r' && hr.at(k + 1) == '\n') break;  // empty line: end of head
    uint32_t c = k, h = kRawFnvInit;
    for (bool more = true; more && c < n;) {  // a quad at a time
      const uint32_t q = hr.quad(c);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t x = (q >> (8 * j)) & 0xFFu;
        if (more && (c >= n || !tchar(x))) more = false;
        if (more) {
          h = raw_fnv(h, (uint8_t)lower(x));
          ++c;
        }
      }
    }
    if (c == k || c >= n || hr.at(c) != ':') return false;
    const uint32_t nl = c - k;
    uint32_t v = c + 1, first = kAbsentSpan, lend = v;
    while (true) {  // field-value up to CRLF: IS_HEADER_CHAR, OWS trimmed
      if (v + 4 <= n && all_plain(hr.quad(v))) {
        if (first == kAbsentSpan) first = v;
        v += 4;
        lend = v;
        continue;
      }
      if (v >= n) return false;
      const uint32_t x = hr.at(v);
      if (x == '\r') {
        if (v + 1 < n && hr.at(v + 1) == '\n') break;
        return false;
      }
      if (!(x == '\t' || (x >= 0x20 && x != 0x7F))) return false;
      if (x != ' ' && x != '\t') {
        if (first == kAbsentSpan) first = v;
        lend = v + 1;
      }
      ++v;
    }
    const uint32_t span = first == kAbsentSpan ? (v << 16) : (first << 16 | (lend - first));
    const bool is_host = nl == 4 && lower(hr.at(k)) == 'h' && lower(hr.at(k + 1)) == 'o' &&
                         lower(hr.at(k + 2)) == 's' && lower(hr.at(k + 3)) == 't';
    if (is_host) {
      if (!have_host) auth = span;  // the first value is the one the filter sees
      have_host = true;
    } else {
      const int f = field_of(R, hr, h, nl, k);
      if (f >= 0 && sp[f * stride] == kAbsentSpan) sp[f * stride] = span;  // first value wins
    }
    k = v + 2;
  }
  if (R.f_method >= 0) sp[R.f_method * stride] = mlen;
  if (R.f_path >= 0) sp[R.f_path * stride] = t0 << 16 | tlen;
  if (R.f_authority >= 0 && have_host) sp[R.f_authority * stride] = auth;
  return true;
}

// Length of the walked string (http_pack.cc): values of the fields up to the
// last present one, each SEP-terminated (absent: 0x01), then REST (0x02) if
// any field after it is absent.
__device__ __forceinline__ uint32_t string_len(const HttpRawDev& R, const uint32_t* sp, uint32_t stride,
                                               uint32_t* last_out) {
  uint32_t last = 0, len = 0;
  for (uint32_t f = 0; f < R.nfields; ++f) {
    const uint32_t s = sp[f * stride];
    if (s != kAbsentSpan) last = f + 1;
  }
  for (uint32_t f = 0; f < last; ++f) {
    const uint32_t s = sp[f * stride];
    len += (s == kAbsentSpan ? 1u : (s & 0xFFFFu)) + 1u;
  }
  if (last < R.nfields) len += 1;
  *last_out = last;
  return len;
}

__device__ __forceinline__ uint32_t lookup_prog(const HttpRawDev& R, uint32_t policy, bool ingress, uint32_t port) {
  if (policy >= R.npolicies) return kProgDeny;
  const uint32_t key = (policy << 17) | ((uint32_t)ingress << 16) | (port & 0xFFFF);
  uint32_t h = hash32(key) & R.phash_mask;
  for (uint32_t probe = 0; probe <= R.phash_mask; ++probe) {
    const uint32_t kk = R.phash_keys[h];
    if (kk == key) return R.phash_vals[h];
    if (kk == 0xFFFFFFFFu) break;
    h = (h + 1) & R.phash_mask;
  }
  return R.dflt[policy * 2 + (ingress ? 1 : 0)];
}

__device__ __forceinline__ bool walked(const HttpRawDev& R, uint32_t prog) {
  return prog < R.nprogs && !(R.progs[prog].flags & kProgAllowAll);
}

__device__ __forceinline__ uint32_t group_of(const HttpRawDev& R, uint32_t prog) {
  return prog < R.nprogs ? prog : R.nprogs + (prog == kProgAllow ? 0u : 1u);
}

// Dynamic LDS of the scan and emit kernels: [spans: nfields × 256 u32]
// [4 wave stages × kStage bytes][bucket counters/cursors: nkeys u32, when
// they fit (lds_keys)].
__device__ __forceinline__ uint8_t* wave_stage(uint32_t* lds, uint32_t F, uint32_t wave) {
  return reinterpret_cast<uint8_t*>(lds + F * kRawThreads) + wave * kStage;
}
__device__ __forceinline__ uint32_t* key_counters(uint32_t* lds, uint32_t F) {
  return reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(lds + F * kRawThreads) + 4 * kStage);
}
// The head of request i as a reader: in the stage if it lies inside it.
__device__ __forceinline__ HeadReader head_of(const uint8_t* __restrict__ raw, const uint64_t* __restrict__ off,
                                              size_t i, const uint8_t* stage, uint64_t sbase, uint32_t slen) {
  const uint64_t a = off[i], b = off[i + 1];
  const uint32_t n = b > a ? (uint32_t)min<uint64_t>(b - a, 0xFFFFFFFFull) : 0u;
  const uint64_t ga = (uint64_t)(uintptr_t)(raw + a);
  const bool in = ga >= sbase && ga + n <= sbase + slen;
  return HeadReader(raw + a, n, in ? stage + (ga - sbase) : nullptr);
}

// ---- pass 1: program, string length, bucket key; per-block bucket counts
// (bcount[key * gridDim.x + block], lds_keys) or a global histogram
__global__ __launch_bounds__(kRawThreads) void raw_scan_kernel(HttpRawDev R, const uint8_t* __restrict__ raw,
                                                               const uint64_t* __restrict__ off, size_t n,
                                                               const uint32_t* __restrict__ policy,
                                                               const uint8_t* __restrict__ ingress,
                                                               const uint16_t* __restrict__ port,
                                                               uint32_t* __restrict__ counts, uint2* __restrict__ rinfo,
                                                               uint32_t* __restrict__ gspans,
                                                               unsigned long long* __restrict__ ovf_bytes,
                                                               uint32_t lds_keys) {
  extern __shared__ uint32_t lds[];
  const uint32_t F = max(R.nfields, 1u), wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* sp = lds + threadIdx.x;  // this lane's spans: sp[f * kRawThreads]
  uint8_t* stage = wave_stage(lds, F, wave);
  uint32_t* lk = key_counters(lds, F);
  const uint32_t nk = (R.nprogs + 2) * kRawKeys;
  if (lds_keys)
    for (uint32_t k = threadIdx.x; k < nk; k += blockDim.x) lk[k] = 0;
  __syncthreads();
  for (size_t base = (size_t)blockIdx.x * kRawThreads; base < n; base += (size_t)gridDim.x * kRawThreads) {
    const size_t i0 = base + (size_t)wave * 64;
    if (i0 >= n) continue;  // wave-uniform
    const size_t i = i0 + lane;
    const bool live = i < n;
    const uint32_t prog = live ? lookup_prog(R, policy[i], ingress[i] != 0, port[i]) : kProgDeny;
    // every request but an unknown policy's is parsed: a head the codec
    // rejects is denied in any program (flagged malformed)
    const bool parse = live && prog != kProgDeny;
    uint32_t slen = 0;
    uint64_t sbase = 0;
    if (__any(parse)) sbase = stage_heads(raw, off[i0], off[min(i0 + 64, n)], stage, lane, &slen);
    wave_sync();
    if (live) {
      uint32_t key = 0, len = 0, bad = 0;
      if (parse) {
        HeadReader hr = head_of(raw, off, i, stage, sbase, slen);
        if (!parse_head(R, hr, sp, kRawThreads)) {
          bad = 1;
        } else if (walked(R, prog)) {
          uint32_t last;
          len = string_len(R, sp, kRawThreads, &last);
          key = len > CG_HTTP_SLOT_BYTES ? kRawKeys - 1 : (len + 15) / 16;
          // the value spans for the emit pass (field-major: coalesced)
          for (uint32_t f = 0; f < R.nfields; ++f) gspans[(size_t)f * n + i] = sp[f * kRawThreads];
          if (len > CG_HTTP_SLOT_BYTES) atomicAdd(ovf_bytes, (unsigned long long)((4 + len + 15) & ~15u));
        }
      }
      rinfo[i] = make_uint2(prog, len | bad << 31);
      const uint32_t k = group_of(R, prog) * kRawKeys + key;
      if (lds_keys) atomicAdd(&lk[k], 1u);
      else atomicAdd(&counts[k], 1u);
    }
    wave_sync();  // the stage is read before the next iteration overwrites it
  }
  if (lds_keys) {
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nk; k += blockDim.x) counts[(size_t)k * gridDim.x + blockIdx.x] = lk[k];
  }
}

// Per bucket key: exclusive prefix of the per-block counts (each block's
// first slot offset within the key's bucket) and the key's total.
__global__ __launch_bounds__(256) void raw_prefix_kernel(const uint32_t* __restrict__ bcount, uint32_t nblk,
                                                         uint32_t* __restrict__ bbase, uint32_t* __restrict__ hist) {
  __shared__ uint32_t part[256];
  const uint32_t k = blockIdx.x, t = threadIdx.x;
  const uint32_t* row = bcount + (size_t)k * nblk;
  const uint32_t per = (nblk + 255) / 256, lo = min(t * per, nblk), hi = min(lo + per, nblk);
  uint32_t sum = 0;
  for (uint32_t j = lo; j < hi; ++j) sum += row[j];
  part[t] = sum;
  __syncthreads();
  if (t == 0) {
    uint32_t run = 0;
    for (uint32_t j = 0; j < 256; ++j) {
      const uint32_t v = part[j];
      part[j] = run;
      run += v;
    }
    hist[k] = run;
  }
  __syncthreads();
  uint32_t run = part[t];
  for (uint32_t j = lo; j < hi; ++j) {
    bbase[(size_t)k * nblk + j] = run;
    run += row[j];
  }
}

// ---- tile table and padding slots
__global__ __launch_bounds__(kRawThreads) void raw_tiles_kernel(const HttpRawGroup* __restrict__ groups,
                                                                uint32_t ngroups, uint32_t ntiles,
                                                                HttpTile* __restrict__ ttab,
                                                                uint8_t* __restrict__ tiles,
                                                                uint32_t* __restrict__ order) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  // the group holding tile t (groups ascending by tile0, all non-empty)
  uint32_t lo = 0, hi = ngroups;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (groups[mid].tile0 <= t) lo = mid;
    else hi = mid;
  }
  const HttpRawGroup& g = groups[lo];
  const uint32_t j = t - g.tile0;
  // units: the largest walked string among the tile's slots (keys are
  // ascending within the group; key kRawKeys-1 is the arena, walked 0)
  const uint32_t e = g.bstart[kRawKeys - 1];
  uint32_t units = 0;
  if (64 * j < e) {
    const uint32_t s_last = min(64 * j + 63, e - 1);
    for (uint32_t k = 0; k + 1 < kRawKeys; ++k)
      if (g.bstart[k] <= s_last && s_last < g.bstart[k + 1]) units = k;
  }
  ttab[t].at = t * kRawTileGranules;
  ttab[t].units = units;
  // padding slots after the group's requests
  uint2* meta = reinterpret_cast<uint2*>(tiles + (size_t)t * kRawTileGranules * 512);
  for (uint32_t l = 0; l < 64; ++l)
    if (64 * j + l >= g.count) {
      meta[l] = make_uint2(0, CG_HTTP_F_PAD << 24);
      order[(size_t)t * 64 + l] = 0xFFFFFFFFu;
    }
}

// 16-byte chunks of a lane's output string: stored to dst, then dst +=
// stride (uint4 units: a tile's next string unit, or the next arena line).
struct Out16 {
  uint32_t w0, w1, w2, w3;
  uint32_t pos, stored;
  uint4* dst;
  uint32_t stride;
  __device__ __forceinline__ Out16(uint4* d, uint32_t s) : w0(0), w1(0), w2(0), w3(0), pos(0), stored(0), dst(d), stride(s) {}
  // nb (1..4) bytes, little-endian in v (its bytes past nb zero), at byte
  // pos: one 64-bit shift spreads them over dword pos / 4 and the next; the
  // part past the 16 bytes starts the next chunk
  __device__ __forceinline__ void put4(uint32_t v, uint32_t nb) {
    const uint64_t t = (uint64_t)v << ((pos & 3) * 8);
    const uint32_t lo = (uint32_t)t, hi = (uint32_t)(t >> 32), q = pos >> 2;
    w0 |= lo & (0u - (q == 0));
    w1 |= (lo & (0u - (q == 1))) | (hi & (0u - (q == 0)));
    w2 |= (lo & (0u - (q == 2))) | (hi & (0u - (q == 1)));
    w3 |= (lo & (0u - (q == 3))) | (hi & (0u - (q == 2)));
    pos += nb;
    if (pos >= 16) {
      const uint32_t rest = pos - 16;
      flush();
      w0 = hi & (0u - (q == 3));
      pos = rest;
    }
  }
  __device__ __forceinline__ void put(uint32_t b) { put4(b, 1); }
  __device__ __forceinline__ void flush() {
    *dst = make_uint4(w0, w1, w2, w3);
    dst += stride;
    w0 = w1 = w2 = w3 = 0;
    pos = 0;
    ++stored;
  }
};

// The walked string through the program's code map into o.
__device__ __forceinline__ void emit_string(const HttpRawDev& R, HeadReader& hr, const uint32_t* sp, uint32_t stride,
                                            uint32_t last, const uint8_t* __restrict__ code, Out16& o) {
  for (uint32_t f = 0; f < last; ++f) {
    const uint32_t s = sp[f * stride];
    if (s == kAbsentSpan) {
      o.put(code[1]);
    } else {
      const uint32_t a = s >> 16, L = s & 0xFFFFu;
      for (uint32_t k = 0; k < L; k += 4) {  // a quad at a time: four code bytes, one insert
        const uint32_t q = hr.quad(a + k), nb = min(L - k, 4u);
        const uint32_t c = (uint32_t)code[q & 0xFFu] | (uint32_t)code[(q >> 8) & 0xFFu] << 8 |
                           (uint32_t)code[(q >> 16) & 0xFFu] << 16 | (uint32_t)code[q >> 24] << 24;
        o.put4(nb == 4 ? c : c & ((1u << (8 * nb)) - 1), nb);
      }
    }
    o.put(code[0]);
  }
  if (last < R.nfields) o.put(code[2]);
}

// ---- pass 2: slots, meta, strings.  Slots: the block's LDS cursor per key
// (the key's first slot + this block's prefix, lds_keys), else a global
// cursor per key.
__global__ __launch_bounds__(kRawThreads) void raw_emit_kernel(
    HttpRawDev R, const uint8_t* __restrict__ raw, const uint64_t* __restrict__ off, size_t n,
    const uint8_t* __restrict__ ingress, const uint32_t* __restrict__ remote, const uint2* __restrict__ rinfo,
    uint32_t* __restrict__ cursor, const uint32_t* __restrict__ bbase, uint32_t lds_keys, HttpTile* __restrict__ ttab,
    uint8_t* __restrict__ tiles, uint32_t* __restrict__ order, uint8_t* __restrict__ arena,
    unsigned long long* __restrict__ arena_cursor, const uint32_t* __restrict__ gspans, uint32_t lds_codes) {
  extern __shared__ uint32_t lds[];
  const uint32_t F = max(R.nfields, 1u), wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* sp = lds + threadIdx.x;
  uint8_t* stage = wave_stage(lds, F, wave);
  uint32_t* lk = key_counters(lds, F);
  const uint32_t nk = (R.nprogs + 2) * kRawKeys;
  if (lds_keys)
    for (uint32_t k = threadIdx.x; k < nk; k += blockDim.x)
      lk[k] = cursor[k] + bbase[(size_t)k * gridDim.x + blockIdx.x];
  // the programs' code maps in LDS (after the key cursors) when they fit
  uint8_t* lcode = reinterpret_cast<uint8_t*>(lk + (lds_keys ? nk : 0));
  if (lds_codes)
    for (uint32_t k = threadIdx.x; k < R.nprogs * 64; k += blockDim.x)
      reinterpret_cast<uint32_t*>(lcode)[k] = reinterpret_cast<const uint32_t*>(R.codes)[k];
  __syncthreads();
  for (size_t base = (size_t)blockIdx.x * kRawThreads; base < n; base += (size_t)gridDim.x * kRawThreads) {
    const size_t i0 = base + (size_t)wave * 64;
    if (i0 >= n) continue;  // wave-uniform
    const size_t i = i0 + lane;
    const bool live = i < n;
    const uint2 ri = live ? rinfo[i] : make_uint2(kProgDeny, 0);
    const uint32_t prog = ri.x, len = ri.y & 0x7FFFFFFFu;
    const bool bad = ri.y >> 31, walk = live && walked(R, prog) && !bad;
    uint32_t slen = 0;
    uint64_t sbase = 0;
    if (__any(walk)) sbase = stage_heads(raw, off[i0], off[min(i0 + 64, n)], stage, lane, &slen);
    wave_sync();
    if (live) {
      const uint32_t key = !walk ? 0u : len > CG_HTTP_SLOT_BYTES ? kRawKeys - 1 : (len + 15) / 16;
      const uint32_t k = group_of(R, prog) * kRawKeys + key;
      const uint32_t slot = lds_keys ? atomicAdd(&lk[k], 1u) : atomicAdd(&cursor[k], 1u);
      order[slot] = (uint32_t)i;
      const uint32_t t = slot >> 6, sl = slot & 63;
      const HttpTile tt = ttab[t];
      uint8_t* tb = tiles + (size_t)tt.at * 512;
      uint32_t flags = (ingress[i] ? CG_HTTP_F_INGRESS : 0u) | (bad ? CG_HTTP_F_MALFORMED : 0u);
      uint32_t aoff16 = 0;
      if (walked(R, prog) && !walk) {  // a rejected head in a walked tile: zero units
        Out16 o(reinterpret_cast<uint4*>(tb + 512 + (size_t)sl * 16), 1024 / 16);
        while (o.stored < tile_units(tt)) o.flush();
      }
      if (walk) {
        HeadReader hr = head_of(raw, off, i, stage, sbase, slen);
        for (uint32_t f = 0; f < R.nfields; ++f) sp[f * kRawThreads] = gspans[(size_t)f * n + i];  // pass 1's
        uint32_t last;
        string_len(R, sp, kRawThreads, &last);
        const uint8_t* code = (lds_codes ? lcode : R.codes) + (size_t)prog * 256;
        if (key == kRawKeys - 1) {  // overflow arena entry: u32 length, the string, 16-byte aligned
          flags |= CG_HTTP_F_OVERFLOW;
          const unsigned long long ao = atomicAdd(arena_cursor, (unsigned long long)((4 + len + 15) & ~15u));
          aoff16 = (uint32_t)(ao / 16);
          Out16 o(reinterpret_cast<uint4*>(arena + ao), 1);
          o.w0 = len;
          o.pos = 4;
          emit_string(R, hr, sp, kRawThreads, last, code, o);
          if (o.pos) o.flush();
          Out16 z(reinterpret_cast<uint4*>(tb + 512 + (size_t)sl * 16), 1024 / 16);
          while (z.stored < tile_units(tt)) z.flush();  // the tile's units are not this lane's string
        } else {
          const uint32_t units = tile_units(tt);
          Out16 o(reinterpret_cast<uint4*>(tb + 512 + (size_t)sl * 16), 1024 / 16);
          emit_string(R, hr, sp, kRawThreads, last, code, o);
          if (o.pos) o.flush();
          while (o.stored < units) o.flush();  // zero padding up to the tile's units
          if (key == units && units) atomicMax(&ttab[t].units, units | (len - 16 * (units - 1)) << 16);
        }
      }
      reinterpret_cast<uint2*>(tb)[sl] = make_uint2(remote[i], (aoff16 & 0xFFFFFFu) | flags << 24);
    }
    wave_sync();
  }
}

__global__ void raw_scatter_kernel(const uint32_t* __restrict__ order, const uint8_t* __restrict__ vslot,
                                   size_t nslots, uint8_t* __restrict__ out) {
  for (size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < nslots; s += (size_t)gridDim.x * blockDim.x) {
    const uint32_t r = order[s];
    if (r != 0xFFFFFFFFu) out[r] = vslot[s];
  }
}

unsigned grid_for(size_t n, int cus, unsigned per_cu) {
  const size_t want = (n + kRawThreads - 1) / kRawThreads;
  return (unsigned)std::max<size_t>(1, std::min<size_t>(want, (size_t)cus * per_cu));
}

// LDS of the scan / emit kernels (see wave_stage, key_counters)
size_t raw_lds(const HttpRawDev& R, bool lds_keys, bool lds_codes) {
  const size_t nk = ((size_t)R.nprogs + 2) * kRawKeys;
  return (size_t)std::max(R.nfields, 1u) * kRawThreads * 4 + 4 * (size_t)kStage + (lds_keys ? nk * 4 : 0) +
         (lds_codes ? (size_t)R.nprogs * 256 : 0) + 16;  // + slack: a quad read may pass the last stage by 7 bytes
}
// code maps in LDS only while small: a larger table costs workgroups per CU
// (occupancy) more than its global (L1-cached) lookups cost
bool lds_codes_fit(const HttpRawDev& R) { return (size_t)R.nprogs * 256 <= 4 * 1024; }

}  // namespace

size_t http_raw_grid(size_t n, int cus) { return grid_for(n, cus, 4); }

bool http_raw_lds_keys(const HttpRawDev& R) { return ((size_t)R.nprogs + 2) * kRawKeys * 4 <= 32 * 1024; }

int launch_http_raw_scan(const HttpRawDev& R, const uint8_t* raw, const uint64_t* off, size_t n,
                         const uint32_t* policy, const uint8_t* ingress, const uint16_t* port, uint32_t* counts,
                         void* rinfo, uint32_t* spans, unsigned long long* ovf_bytes, void* stream, int cus) {
  if (!n) return 0;
  const bool lk = http_raw_lds_keys(R);
  const size_t lds = raw_lds(R, lk, false);
  (void)hipFuncSetAttribute((const void*)raw_scan_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(raw_scan_kernel, dim3((unsigned)http_raw_grid(n, cus)), dim3(kRawThreads), lds,
                     (hipStream_t)stream, R, raw, off, n, policy, ingress, port, counts, (uint2*)rinfo, spans,
                     ovf_bytes, (uint32_t)lk);
  return (int)hipGetLastError();
}

int launch_http_raw_prefix(const uint32_t* bcount, uint32_t nkeys, uint32_t nblk, uint32_t* bbase, uint32_t* hist,
                           void* stream) {
  if (!nkeys) return 0;
  hipLaunchKernelGGL(raw_prefix_kernel, dim3(nkeys), dim3(256), 0, (hipStream_t)stream, bcount, nblk, bbase, hist);
  return (int)hipGetLastError();
}

int launch_http_raw_tiles(const HttpRawGroup* groups, uint32_t ngroups, uint32_t ntiles, HttpTile* ttab,
                          uint8_t* tiles, uint32_t* order, void* stream) {
  if (!ntiles) return 0;
  hipLaunchKernelGGL(raw_tiles_kernel, dim3((ntiles + kRawThreads - 1) / kRawThreads), dim3(kRawThreads), 0,
                     (hipStream_t)stream, groups, ngroups, ntiles, ttab, tiles, order);
  return (int)hipGetLastError();
}

int launch_http_raw_emit(const HttpRawDev& R, const uint8_t* raw, const uint64_t* off, size_t n,
                         const uint8_t* ingress, const uint32_t* remote, const void* rinfo, uint32_t* cursor,
                         const uint32_t* bbase, HttpTile* ttab, uint8_t* tiles, uint32_t* order, uint8_t* arena,
                         unsigned long long* arena_cursor, const uint32_t* spans, void* stream, int cus) {
  if (!n) return 0;
  const bool lk = http_raw_lds_keys(R), lc = lds_codes_fit(R);
  const size_t lds = raw_lds(R, lk, lc);
  (void)hipFuncSetAttribute((const void*)raw_emit_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(raw_emit_kernel, dim3((unsigned)http_raw_grid(n, cus)), dim3(kRawThreads), lds,
                     (hipStream_t)stream, R, raw, off, n, ingress, remote, (const uint2*)rinfo, cursor, bbase,
                     (uint32_t)lk, ttab, tiles, order, arena, arena_cursor, spans, (uint32_t)lc);
  return (int)hipGetLastError();
}

int launch_http_raw_scatter(const uint32_t* order, const uint8_t* vslot, size_t nslots, uint8_t* out, void* stream,
                            int cus) {
  if (!nslots) return 0;
  hipLaunchKernelGGL(raw_scatter_kernel, dim3(grid_for(nslots, cus, 8)), dim3(kRawThreads), 0, (hipStream_t)stream,
                     order, vslot, nslots, out);
  return (int)hipGetLastError();
}

}  // namespace cg
