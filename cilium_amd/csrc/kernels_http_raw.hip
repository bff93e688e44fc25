// kernels_http_raw.hip — HTTP/1 request heads straight from HBM into the
// http_kernel batch format (gfx950), so raw request streams go from device
// memory to verdicts without the host parser and packer.
//
// The steps of http_parse.cc (the codec: request line, header fields, Host →
// :authority, rejected heads) and http_pack.cc (program lookup, the walked
// string v_1 SEP .. v_F SEP / REST, class codes, grouping by program and
// string units):
//   raw_scan_kernel   one lane per head (the wave's heads staged in LDS):
//                     parse, program, the walked string class-coded into a
//                     request-ordered string buffer (16-byte aligned per
//                     request), bucket key (program group × string units)
//                     and the per-block bucket counts
//   (host)            bucket counts → chunks, runs of equal-units tiles,
//                     bucket cursors
//   raw_rank_kernel   a slot per request from its bucket cursor: order[slot]
//   raw_build_kernel  one wave per tile: each lane's string gathered from the
//                     string buffer and stored unit-major (whole 1 KiB lines
//                     per unit), meta words, the tile table entry (units and
//                     tail from the wave's longest string), overflow strings
//                     into the arena
//   http_kernel       the verdicts, written straight to request order
//                     through order[] (kernels_http.hip VOut)
// Slots within a bucket come in atomic order: the verdicts are per request,
// so they do not depend on it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "../../include/cilium_gpu.h"
#include "dev_types.h"
#include "kernels.h"

namespace cg {

namespace {

constexpr int kRawThreads = 256;
constexpr uint32_t kAbsentSpan = 0xFFFFFFFFu;

// Explicit address spaces for the scan's LDS stage, bitmaps, spans and tables
// and for the heads in HBM: through generic pointers every stage access
// compiled to a flat load (waiting on vmcnt like an HBM load).
#define CG_LDS __attribute__((address_space(3)))
#define CG_GLB __attribute__((address_space(1)))
typedef CG_LDS uint8_t lds_u8;
typedef CG_LDS uint32_t lds_u32;
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));  // (HIP's uint4 class takes no address space)
typedef CG_LDS v4u32 lds_v4;
typedef const CG_GLB v4u32 glb_v4;
__device__ __forceinline__ uint4 to_uint4(v4u32 v) { return make_uint4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ v4u32 to_v4(uint4 v) { return v4u32{v.x, v.y, v.z, v.w}; }
typedef const CG_GLB uint8_t glb_u8;
typedef const CG_GLB uint32_t glb_u32;
// The lookup tables of the scan (name keys, field slots, names, program
// hash): staged in LDS when they fit, else read from HBM.
template <class P32, class P8>
struct RawTabs {
  P32 nkeys, fslots, phk, phv, walk;
  P8 fnames;
};
using LdsTabs = RawTabs<const lds_u32*, const lds_u8*>;
using GlbTabs = RawTabs<glb_u32*, glb_u8*>;

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
  glb_u8* p;
  uint32_t n;
  const lds_u8* lp;  // the head in LDS (in)
  bool in;
  uint64_t cur;
  uint4 w;
  __device__ __forceinline__ HeadReader(glb_u8* p_, uint32_t n_, const lds_u8* lp_, bool in_)
      : p(p_), n(n_), lp(lp_), in(in_), cur(~0ull), w{0, 0, 0, 0} {}
  // bytes k..k+3 (little-endian; bytes past the head are unspecified): from
  // LDS two aligned dword reads and a byte align, so a walk pays one LDS
  // round trip per 4 bytes instead of one per byte
  __device__ __forceinline__ uint32_t quad(uint32_t k) {
    if (in) {
      const uint32_t a = (uint32_t)(uintptr_t)(lp + k);
      const lds_u32* w4 = (const lds_u32*)(uintptr_t)(a & ~3u);
      return __builtin_amdgcn_alignbyte(w4[1], w4[0], a & 3u);
    }
    uint32_t q = 0;  // global: never past the head (it may end the buffer)
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
      if (k + j < n) q |= at(k + j) << (8 * j);
    return q;
  }
  __device__ __forceinline__ uint32_t at(uint32_t k) {
    if (in) return lp[k];
    const uint64_t a = (uint64_t)(uintptr_t)(p + k);
    const uint64_t blk = a & ~15ull;
    if (blk != cur) {
      cur = blk;
      const uint64_t lo = (uint64_t)(uintptr_t)p, hi = lo + n;
      if (blk >= lo && blk + 16 <= hi) {
        w = to_uint4(*(glb_v4*)(uintptr_t)blk);
      } else {
        uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          const uint64_t x = blk + b;
          const uint32_t byte = (x >= lo && x < hi) ? *(glb_u8*)(uintptr_t)x : 0u;
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
constexpr uint32_t kMaskWords = kStage / 32;  // u32 words per structural mask of a stage
__device__ __forceinline__ uint64_t stage_heads(glb_u8* raw, uint64_t lo, uint64_t hi, lds_u8* stage, uint32_t lane,
                                                uint32_t* len) {
  const uint64_t glo = (uint64_t)(uintptr_t)(raw + lo), ghi = (uint64_t)(uintptr_t)(raw + hi);
  const uint64_t a0 = glo & ~15ull;
  const uint32_t nb = (uint32_t)min<uint64_t>((ghi - a0 + 15) & ~15ull, kStage);
  for (uint32_t j = lane * 16; j < nb; j += 64 * 16) {
    const uint64_t a = a0 + j;
    uint4 v;
    if (a >= glo && a + 16 <= ghi) {
      v = to_uint4(*(glb_v4*)(uintptr_t)a);
    } else {
      uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const uint64_t x = a + b;
        const uint32_t byte = (x >= glo && x < ghi) ? *(glb_u8*)(uintptr_t)x : 0u;
        const uint32_t sh = (b & 3) * 8;
        if (b < 4) v0 |= byte << sh;
        else if (b < 8) v1 |= byte << sh;
        else if (b < 12) v2 |= byte << sh;
        else v3 |= byte << sh;
      }
      v = make_uint4(v0, v1, v2, v3);
    }
    *(lds_v4*)(stage + j) = to_v4(v);
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
template <class Tabs>
__device__ __forceinline__ int field_of(const HttpRawDev& R, const Tabs& T, HeadReader& hr, uint32_t h, uint32_t nl,
                                        uint32_t k) {
  uint32_t sl = h & R.fmask;
  for (uint32_t probe = 0; probe <= R.fmask; ++probe) {
    const uint4 e = make_uint4(T.fslots[4 * sl], T.fslots[4 * sl + 1], T.fslots[4 * sl + 2], T.fslots[4 * sl + 3]);
    if (e.y == 0) return -1;
    if (e.x == h && e.y == nl) {
      bool eq = true;
      for (uint32_t j = 0; j < nl && eq; ++j) eq = lower(hr.at(k + j)) == T.fnames[e.w + j];
      if (eq) return (int)e.z;
    }
    sl = (sl + 1) & R.fmask;
  }
  return -1;
}

// parse_head (http_parse.cc) for one head: the value span {start << 16 |
// length} of every field it sets in sp[f * stride] (kAbsentSpan otherwise);
// false = the codec rejects the head.
template <class Tabs>
__device__ __forceinline__ bool parse_head(const HttpRawDev& R, const Tabs& T, HeadReader& hr, lds_u32* sp,
                                           uint32_t stride) {
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
      const int f = field_of(R, T, hr, h, nl, k);
      if (f >= 0 && sp[f * stride] == kAbsentSpan) sp[f * stride] = span;  // first value wins
    }
    k = v + 2;
  }
  if (R.f_method >= 0) sp[R.f_method * stride] = mlen;
  if (R.f_path >= 0) sp[R.f_path * stride] = t0 << 16 | tlen;
  if (R.f_authority >= 0 && have_host) sp[R.f_authority * stride] = auth;
  return true;
}

// ---- structural masks of a wave's stage (data-parallel) ----------------
// Two bitmaps over the stage's bytes, built by all 64 lanes (32 bytes per
// lane per round): `special` = byte < 0x21 or DEL (SP, HTAB, CR, LF and every
// control byte: what ends a plain run of target or field-value bytes) and
// `nontchar` (not an RFC 7230 tchar: what ends a method or a header name).
// A lane then parses its head line by line with find-next-set over the
// bitmaps instead of byte loops.
__device__ __forceinline__ uint32_t pack4(uint32_t hi_bits) {  // bits 7/15/23/31 → bits 0..3
  return ((hi_bits >> 7) * 0x00204081u) >> 21 & 0xFu;
}
__device__ __forceinline__ uint32_t special4(uint32_t x) {
  const uint32_t lt = ~(((x & 0x7F7F7F7Fu) + 0x5F5F5F5Fu) | x) & 0x80808080u;  // byte < 0x21
  const uint32_t t = x ^ 0x7F7F7F7Fu;
  const uint32_t del = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;  // byte == 0x7F
  return pack4(lt | del);
}
__device__ __forceinline__ void build_masks(const lds_u8* stage, uint32_t slen, const lds_u8* tct, lds_u32* masks,
                                            uint32_t lane) {
  for (uint32_t w = lane; w * 32 < slen; w += 64) {
    const uint4 a = to_uint4(*(const lds_v4*)(stage + 32 * w));
    const uint4 b = to_uint4(*(const lds_v4*)(stage + 32 * w + 16));
    const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t sp = 0, nt = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sp |= special4(d[k]) << (4 * k);
#pragma unroll
      for (int j = 0; j < 4; ++j) nt |= (uint32_t)tct[(d[k] >> (8 * j)) & 0xFFu] << (4 * k + j);
    }
    masks[w] = sp;
    masks[kMaskWords + w] = nt;
  }
}
// First set bit at or after p (stage offsets), or lim when none before lim.
__device__ __forceinline__ uint32_t next_set(const lds_u32* m, uint32_t p, uint32_t lim) {
  uint32_t w = p >> 5;
  uint32_t x = m[w] & (0xFFFFFFFFu << (p & 31));
  while (!x) {
    if (32 * (w + 1) >= lim) return lim;
    x = m[++w];
  }
  return min(32 * w + (uint32_t)__builtin_ctz(x), lim);
}
__device__ __forceinline__ uint32_t sbyte(const lds_u8* st, uint32_t p) { return st[p]; }
__device__ __forceinline__ uint32_t squad(const lds_u8* st, uint32_t p) {
  const lds_u32* w4 = (const lds_u32*)(st + (p & ~3u));
  return __builtin_amdgcn_alignbyte(w4[1], w4[0], p & 3u);
}
__device__ __forceinline__ uint32_t lower4(uint32_t x) {  // ASCII A-Z → a-z, per byte (bytes < 0x80)
  const uint32_t y = x & 0x7F7F7F7Fu;
  const uint32_t ge_a = y + 0x3F3F3F3Fu, gt_z = y + 0x25252525u;  // bit 7: byte >= 'A' / byte > 'Z'
  return x | ((ge_a & ~gt_z & ~x & 0x80808080u) >> 2);
}
__device__ __forceinline__ uint32_t keep_bytes(uint32_t x, uint32_t nb) {
  return nb >= 4 ? x : x & ((1u << (8 * nb)) - 1u);
}

// The field a header name (stage bytes [k, k + nl)) is, or -1: the lowercase
// (length, first 8, last 8) key in R.nkeys (raw_name_key), the bytes between
// verified for longer names.
template <class Tabs>
__device__ __forceinline__ int field_of_key(const HttpRawDev& R, const Tabs& T, const lds_u8* st, uint32_t k,
                                            uint32_t nl) {
  uint32_t lo0 = lower4(keep_bytes(squad(st, k), nl)), lo1 = 0, hi0 = 0, hi1 = 0;
  if (nl > 4) lo1 = lower4(keep_bytes(squad(st, k + 4), nl - 4));
  if (nl > 8) {
    hi0 = lower4(squad(st, k + nl - 8));
    hi1 = lower4(squad(st, k + nl - 4));
  }
  uint32_t sl = raw_name_hash(nl, lo0, lo1, hi0, hi1) & R.nkmask;
  for (uint32_t probe = 0; probe <= R.nkmask; ++probe) {
    const uint32_t e0 = T.nkeys[8 * sl];
    if (e0 == 0) return -1;
    if (e0 == nl && T.nkeys[8 * sl + 1] == lo0 && T.nkeys[8 * sl + 2] == lo1 && T.nkeys[8 * sl + 3] == hi0 &&
        T.nkeys[8 * sl + 4] == hi1) {
      const uint32_t name_off = T.nkeys[8 * sl + 6];
      bool eq = true;
      for (uint32_t j = 8; j + 8 < nl && eq; ++j) eq = lower(sbyte(st, k + j)) == T.fnames[name_off + j];
      if (eq) return (int)T.nkeys[8 * sl + 5];
    }
    sl = (sl + 1) & R.nkmask;
  }
  return -1;
}

// parse_head over the stage with the structural masks: the head is stage
// bytes [hs, he).  Same results as parse_head (http_parse.cc semantics).
template <class Tabs>
__device__ __forceinline__ bool parse_head_masks(const HttpRawDev& R, const Tabs& T, const lds_u8* st,
                                                 const lds_u32* msp, const lds_u32* mnt, uint32_t hs, uint32_t he,
                                                 lds_u32* sp, uint32_t stride) {
  for (uint32_t f = 0; f < R.nfields; ++f) sp[f * stride] = kAbsentSpan;
  if (he - hs > kRawMaxHead) return false;
  const uint32_t m = next_set(mnt, hs, he);  // method: a tchar run, then SP
  if (m == hs || m >= he || sbyte(st, m) != ' ') return false;
  const uint32_t t0 = m + 1;
  const uint32_t te = next_set(msp, t0, he);  // request-target: plain bytes, then SP
  if (te == t0 || te >= he || sbyte(st, te) != ' ') return false;
  uint32_t k = te + 1;
  if (k + 10 > he) return false;  // "HTTP/" DIGIT "." DIGIT CRLF
  {
    const uint32_t q0 = squad(st, k), q1 = squad(st, k + 4), q2 = squad(st, k + 8);
    const uint32_t d1 = q1 >> 8 & 0xFFu, d2 = q1 >> 24;
    if (q0 != 0x50545448u || (q1 & 0xFFu) != '/' || d1 < '0' || d1 > '9' || (q1 >> 16 & 0xFFu) != '.' || d2 < '0' ||
        d2 > '9' || (q2 & 0xFFFFu) != 0x0A0Du)
      return false;
  }
  k += 10;
  bool have_host = false;
  uint32_t auth = kAbsentSpan;
  while (true) {
    if (k + 1 >= he) return false;  // no CRLF left: incomplete head
    if ((squad(st, k) & 0xFFFFu) == 0x0A0Du) break;  // empty line: end of head
    const uint32_t c = next_set(mnt, k, he);  // name: a tchar run, then ':'
    if (c == k || c >= he || sbyte(st, c) != ':') return false;
    const uint32_t nl = c - k;
    uint32_t v = c + 1, first = kAbsentSpan, lend = v, s;
    while (true) {  // field-value to CRLF: IS_HEADER_CHAR, OWS trimmed
      s = next_set(msp, v, he);
      if (s > v) {
        if (first == kAbsentSpan) first = v;
        lend = s;
      }
      if (s >= he) return false;
      const uint32_t x = sbyte(st, s);
      if (x == ' ' || x == '\t') {
        v = s + 1;
        continue;
      }
      if (x == '\r' && s + 1 < he && sbyte(st, s + 1) == '\n') break;
      return false;
    }
    const uint32_t span = first == kAbsentSpan ? ((s - hs) << 16) : ((first - hs) << 16 | (lend - first));
    const bool is_host = nl == 4 && lower4(squad(st, k)) == 0x74736F68u;  // "host"
    if (is_host) {
      if (!have_host) auth = span;  // the first value is the one the filter sees
      have_host = true;
    } else {
      const int f = field_of_key(R, T, st, k, nl);
      if (f >= 0 && sp[f * stride] == kAbsentSpan) sp[f * stride] = span;  // first value wins
    }
    k = s + 2;
  }
  if (R.f_method >= 0) sp[R.f_method * stride] = m - hs;
  if (R.f_path >= 0) sp[R.f_path * stride] = (t0 - hs) << 16 | (te - t0);
  if (R.f_authority >= 0 && have_host) sp[R.f_authority * stride] = auth;
  return true;
}

// ---- header lists (cg_http_pack input): "name\0value\0" pairs ----------
// http_pack.cc semantics: names compare case-insensitively (ASCII), the first
// value of a name wins, a value byte the codec rejects (or, proxylib
// snapshots, a raw byte <= 0x02 / a bad 0x03 escape pair) flags the request
// malformed; a pair cut short by the list's end has what it has.
__device__ __forceinline__ bool list_stop(uint32_t c, bool raw_values) {  // ends a plain run of value bytes
  return raw_values ? c <= 3 : ((c < 0x20 && c != 0x09) || c == 0x7F);  // both include the NUL terminator
}
__device__ __forceinline__ uint32_t zero4(uint32_t x) {  // bit per zero byte
  return pack4(~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u);
}
// masks: `stop` (list_stop, from the table tct) and `zero` (NUL)
__device__ __forceinline__ void build_masks_lists(const lds_u8* stage, uint32_t slen, const lds_u8* tct,
                                                  lds_u32* masks, uint32_t lane) {
  for (uint32_t w = lane; w * 32 < slen; w += 64) {
    const uint4 a = to_uint4(*(const lds_v4*)(stage + 32 * w));
    const uint4 b = to_uint4(*(const lds_v4*)(stage + 32 * w + 16));
    const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t st = 0, zr = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      zr |= zero4(d[k]) << (4 * k);
#pragma unroll
      for (int j = 0; j < 4; ++j) st |= (uint32_t)tct[(d[k] >> (8 * j)) & 0xFFu] << (4 * k + j);
    }
    masks[w] = st;
    masks[kMaskWords + w] = zr;
  }
}

// The value bytes [v, e) of a proxylib snapshot's list: false when one is a
// raw byte <= 0x02 or a 0x03 not followed by 0x10..0x14 (http_pack.cc).
template <class Byte, class NextStop>
__device__ __forceinline__ bool escapes_ok(uint32_t v, uint32_t e, Byte byte, NextStop next_stop) {
  bool ok = true;
  for (uint32_t s = next_stop(v, e); s < e;) {
    if (byte(s) <= 2) {
      ok = false;
      s = next_stop(s + 1, e);
      continue;
    }
    const uint32_t y = s + 1 < e ? byte(s + 1) : 0u;  // 0x03: an escape pair
    if (y < 0x10 || y > 0x14) ok = false;
    const uint32_t nx = s + (s + 1 < e ? 2u : 1u);
    s = nx < e ? next_stop(nx, e) : e;
  }
  return ok;
}

// A list inside the stage, bytes [hs, he), over its masks.
template <class Tabs>
__device__ __forceinline__ bool parse_list_masks(const HttpRawDev& R, const Tabs& T, const lds_u8* st,
                                                 const lds_u32* mstop, const lds_u32* mzero, uint32_t hs, uint32_t he,
                                                 lds_u32* sp, uint32_t stride) {
  for (uint32_t f = 0; f < R.nfields; ++f) sp[f * stride] = kAbsentSpan;
  bool ok = true;
  for (uint32_t k = hs; k < he;) {
    const uint32_t ne = next_set(mzero, k, he), nl = ne - k;
    const uint32_t v = ne < he ? ne + 1 : he;
    uint32_t e;
    if (!R.raw_values) {
      const uint32_t s = v < he ? next_set(mstop, v, he) : he;
      e = s;
      if (s < he && sbyte(st, s) != 0) {  // a byte the codec rejects
        ok = false;
        e = next_set(mzero, s, he);
      }
    } else {
      e = v < he ? next_set(mzero, v, he) : he;
      ok &= escapes_ok(
          v, e, [&](uint32_t x) { return sbyte(st, x); }, [&](uint32_t x, uint32_t lim) { return next_set(mstop, x, lim); });
    }
    const int f = nl ? field_of_key(R, T, st, k, nl) : R.f_empty;
    if (f >= 0 && sp[f * stride] == kAbsentSpan) sp[f * stride] = (v - hs) << 16 | (e - v);  // first value wins
    k = e < he ? e + 1 : he;
  }
  return ok;
}

// A list outside the stage, byte by byte.
template <class Tabs>
__device__ __forceinline__ bool parse_list_bytes(const HttpRawDev& R, const Tabs& T, HeadReader& hr, lds_u32* sp,
                                                 uint32_t stride) {
  for (uint32_t f = 0; f < R.nfields; ++f) sp[f * stride] = kAbsentSpan;
  const uint32_t n = hr.n;
  bool ok = true;
  for (uint32_t k = 0; k < n;) {
    uint32_t c = k, h = kRawFnvInit;
    for (uint32_t x; c < n && (x = hr.at(c)) != 0; ++c) h = raw_fnv(h, (uint8_t)lower(x));
    const uint32_t nl = c - k, v = c < n ? c + 1 : n;
    uint32_t e = v;
    while (e < n && hr.at(e) != 0) ++e;
    if (!R.raw_values) {
      for (uint32_t j = v; j < e; ++j)
        if (list_stop(hr.at(j), false)) ok = false;
    } else {
      ok &= escapes_ok(
          v, e, [&](uint32_t x) { return hr.at(x); },
          [&](uint32_t x, uint32_t lim) {
            while (x < lim && hr.at(x) > 3) ++x;
            return x;
          });
    }
    const int f = nl ? field_of(R, T, hr, h, nl, k) : R.f_empty;
    if (f >= 0 && sp[f * stride] == kAbsentSpan) sp[f * stride] = v << 16 | (e - v);
    k = e < n ? e + 1 : n;
  }
  return ok;
}

// Length of the walked string (http_pack.cc): values of the fields up to the
// last present one, each SEP-terminated (absent: 0x01), then REST (0x02) if
// any field after it is absent.
__device__ __forceinline__ uint32_t string_len(const HttpRawDev& R, const lds_u32* sp, uint32_t stride,
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

template <class Tabs>
__device__ __forceinline__ uint32_t lookup_prog(const HttpRawDev& R, const Tabs& T, uint32_t policy, bool ingress,
                                                uint32_t port) {
  if (policy >= R.npolicies) return kProgDeny;
  const uint32_t key = (policy << 17) | ((uint32_t)ingress << 16) | (port & 0xFFFF);
  uint32_t h = hash32(key) & R.phash_mask;
  for (uint32_t probe = 0; probe <= R.phash_mask; ++probe) {
    const uint32_t kk = T.phk[h];
    if (kk == key) return T.phv[h];
    if (kk == 0xFFFFFFFFu) break;
    h = (h + 1) & R.phash_mask;
  }
  return R.dflt[policy * 2 + (ingress ? 1 : 0)];
}

template <class Tabs>
__device__ __forceinline__ bool walked_t(const HttpRawDev& R, const Tabs& T, uint32_t prog) {
  return prog < R.nprogs && ((T.walk[prog >> 5] >> (prog & 31)) & 1u);
}
__device__ __forceinline__ bool walked(const HttpRawDev& R, uint32_t prog) {
  return prog < R.nprogs && !(R.progs[prog].flags & kProgAllowAll);
}

__device__ __forceinline__ uint32_t group_of(const HttpRawDev& R, uint32_t prog) {
  return prog < R.nprogs ? prog : R.nprogs + (prog == kProgAllow ? 0u : 1u);
}

// Dynamic LDS of the scan kernel: [spans: nfields × 256 u32][4 wave stages ×
// kStage bytes][4 wave mask pairs × 2 × kStage bits][tchar table: 256 B]
// [bucket counters: nkeys u32, when they fit (lds_keys)].
__device__ __forceinline__ lds_u8* wave_stage(lds_u32* lds, uint32_t F, uint32_t wave) {
  return (lds_u8*)(lds + F * kRawThreads) + wave * kStage;
}
__device__ __forceinline__ lds_u32* wave_masks(lds_u32* lds, uint32_t F, uint32_t wave) {
  return (lds_u32*)((lds_u8*)(lds + F * kRawThreads) + 4 * kStage) + wave * 2 * kMaskWords;
}
__device__ __forceinline__ lds_u8* tchar_table(lds_u32* lds, uint32_t F) { return (lds_u8*)wave_masks(lds, F, 4); }
__device__ __forceinline__ lds_u32* key_counters(lds_u32* lds, uint32_t F) { return (lds_u32*)(tchar_table(lds, F) + 256); }
// [name keys: 8 u32 per slot][field slots: 4 u32 per slot][names, u32
// words][program hash keys][values] after the key counters, when they fit
// (lds_tables): the lookups every header line and request makes, at LDS
// latency instead of L1/L2
struct RawTableWords {
  uint32_t nk, fs, fn, ph, wb;
};
__host__ __device__ __forceinline__ RawTableWords raw_table_words(const HttpRawDev& R) {
  return {8 * (R.nkmask + 1), 4 * (R.fmask + 1), (R.fnames_bytes + 3) / 4, R.phash_mask + 1, (R.nprogs + 31) / 32 + 1};
}
__host__ __device__ __forceinline__ uint32_t raw_tables_lds_words(const HttpRawDev& R) {
  const RawTableWords w = raw_table_words(R);
  return w.nk + w.fs + w.fn + 2 * w.ph + w.wb;
}
// The head of request i as a reader: in the stage if it lies inside it.
__device__ __forceinline__ HeadReader head_of(glb_u8* raw, const uint64_t* __restrict__ off, size_t i,
                                              const lds_u8* stage, uint64_t sbase, uint32_t slen) {
  const uint64_t a = off[i], b = off[i + 1];
  const uint32_t n = b > a ? (uint32_t)min<uint64_t>(b - a, 0xFFFFFFFFull) : 0u;
  const uint64_t ga = (uint64_t)(uintptr_t)(raw + a);
  const bool in = ga >= sbase && ga + n <= sbase + slen;
  return HeadReader(raw + a, n, stage + (in ? (uint32_t)(ga - sbase) : 0u), in);
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

// The walked string, uncoded (value bytes, SEP 0x00, absent 0x01, REST 0x02
// — the bytes the program's code map takes), into o.
__device__ __forceinline__ void emit_string(const HttpRawDev& R, HeadReader& hr, const lds_u32* sp, uint32_t stride,
                                            uint32_t last, Out16& o) {
  for (uint32_t f = 0; f < last; ++f) {
    const uint32_t s = sp[f * stride];
    if (s == kAbsentSpan) {
      o.put4(1u, 2);  // absent, SEP
      continue;
    }
    const uint32_t a = s >> 16, L = s & 0xFFFFu;
    for (uint32_t k = 0; k < L; k += 4) {  // a quad at a time
      const uint32_t q = hr.quad(a + k), nb = min(L - k, 4u);
      o.put4(nb == 4 ? q : q & ((1u << (8 * nb)) - 1), nb);
    }
    o.put(0u);  // SEP
  }
  if (last < R.nfields) o.put(2u);  // REST
}

// A request's record in the string buffer (16-byte aligned, request order):
// a 16-byte header {request index, remote identity, string length | flags
// << 24, program} and the uncoded walked string.  A head of h bytes yields at
// most h + 2F bytes of string (each absent field costs 2 bytes the head does
// not hold; the request line and the blank line hold 13 bytes no string
// does), so with a stride of cst >= 2F + 32 bytes per request the records
// never overlap.
__device__ __forceinline__ uint64_t rec_off(uint64_t head_rel, size_t i, uint32_t cst) {
  return ((head_rel + 15) & ~15ull) + (uint64_t)cst * i;
}

// ---- pass 1: parse, program, string length, bucket key, the request's
// record in the string buffer; per-block bucket counts (bcount[key * gridDim.x + block],
// lds_keys) or a global histogram.  kLists: header lists, not heads;
// kMasks: requests inside the stage parse over its structural bitmaps (else
// through HeadReader's dword steps).
// A lane's request inputs, loaded two iterations ahead of their use.
struct RawIn {
  uint32_t pol, ing, port;
  uint64_t a, b;  // off[i], off[i + 1]
};
__device__ __forceinline__ RawIn raw_in(const uint64_t* __restrict__ off, const uint32_t* __restrict__ policy,
                                        const uint8_t* __restrict__ ingress, const uint16_t* __restrict__ port,
                                        size_t i, size_t n) {
  const size_t j = i < n ? i : (n ? n - 1 : 0);  // unconditional loads (no branch around them)
  RawIn r;
  r.pol = i < n ? policy[j] : 0xFFFFFFFFu;
  r.ing = ingress[j];
  r.port = port[j];
  r.a = off[j];
  r.b = off[j + 1];
  if (i >= n) r.a = r.b;  // empty
  return r;
}
constexpr uint32_t kStageVecs = kStage / (64 * 16);  // 16-B loads per lane for a whole stage
// The stage of the wave whose lanes hold `in` (64 consecutive requests, lanes
// past n empty): its 16-B aligned blocks into registers.  Every block loaded
// holds at least one byte of the wave's heads, so no load leaves their pages.
struct StageRegs {
  uint4 v[kStageVecs];
  uint64_t base;
  uint32_t len;
};
__device__ __forceinline__ void stage_load(glb_u8* raw, const RawIn& in, uint32_t lane, StageRegs& S) {
  const uint64_t lo = __shfl(in.a, 0, 64);
  // the last lane's end (empty lanes past n repeat off[n])
  const uint64_t hi = __shfl(in.b, 63, 64);
  const uint64_t glo = (uint64_t)(uintptr_t)(raw + lo), ghi = (uint64_t)(uintptr_t)(raw + hi);
  const uint64_t a0 = glo & ~15ull;
  const uint32_t nb = hi > lo ? (uint32_t)min<uint64_t>((ghi - a0 + 15) & ~15ull, kStage) : 0u;
  S.base = a0;
  S.len = nb;
#pragma unroll
  for (uint32_t j = 0; j < kStageVecs; ++j) {
    const uint32_t o = (j * 64 + lane) * 16;
    const uint64_t a = o < nb ? a0 + o : a0;  // past the stage: a harmless repeat of the first block
    S.v[j] = nb ? to_uint4(*(glb_v4*)(uintptr_t)a) : make_uint4(0, 0, 0, 0);
  }
}
__device__ __forceinline__ void stage_store(const StageRegs& S, lds_u8* stage, uint32_t lane) {
#pragma unroll
  for (uint32_t j = 0; j < kStageVecs; ++j) *(lds_v4*)(stage + (j * 64 + lane) * 16) = to_v4(S.v[j]);
}

template <bool kLists, bool kMasks, bool kLdsTabs>
__global__ __launch_bounds__(kRawThreads) void raw_scan_kernel(HttpRawDev R, const uint8_t* __restrict__ raw_g,
                                                               const uint64_t* __restrict__ off, size_t n,
                                                               const uint32_t* __restrict__ policy,
                                                               const uint8_t* __restrict__ ingress,
                                                               const uint16_t* __restrict__ port,
                                                               uint32_t* __restrict__ counts, uint2* __restrict__ rinfo,
                                                               const uint32_t* __restrict__ remote,
                                                               uint8_t* __restrict__ sbuf, uint32_t cst,
                                                               unsigned long long* __restrict__ ovf_bytes,
                                                               uint32_t lds_keys) {
  extern __shared__ uint32_t lds_[];
  lds_u32* lds = (lds_u32*)lds_;
  glb_u8* raw = (glb_u8*)raw_g;
  const uint32_t F = max(R.nfields, 1u), wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  lds_u32* sp = lds + threadIdx.x;  // this lane's spans: sp[f * kRawThreads]
  lds_u8* stage = wave_stage(lds, F, wave);
  lds_u32* masks = wave_masks(lds, F, wave);
  lds_u8* tct = tchar_table(lds, F);
  lds_u32* lk = key_counters(lds, F);
  const uint32_t nk = (R.nprogs + 2) * kRawKeys;
  if (lds_keys)
    for (uint32_t k = threadIdx.x; k < nk; k += blockDim.x) lk[k] = 0;
  for (uint32_t b = threadIdx.x; b < 256; b += blockDim.x) tct[b] = kLists ? list_stop(b, R.raw_values) : !tchar(b);
  // the lookup tables: LDS copies when they fit (kLdsTabs), else HBM
  using Tabs = typename std::conditional<kLdsTabs, LdsTabs, GlbTabs>::type;
  Tabs T;
  if constexpr (kLdsTabs) {
    const RawTableWords w = raw_table_words(R);
    lds_u32* t = lk + (lds_keys ? nk : 0u);
    lds_u32* tfs = t + w.nk;
    lds_u32* tfn = tfs + w.fs;
    lds_u32* tpk = tfn + w.fn;
    lds_u32* tpv = tpk + w.ph;
    lds_u32* twb = tpv + w.ph;
    for (uint32_t k = threadIdx.x; k < w.nk; k += blockDim.x) t[k] = R.nkeys[k];
    for (uint32_t k = threadIdx.x; k < w.fs; k += blockDim.x) tfs[k] = R.fslots[k];
    for (uint32_t k = threadIdx.x; k < w.fn; k += blockDim.x) {
      uint32_t v = 0;
      for (uint32_t j = 0; j < 4; ++j)
        if (4 * k + j < R.fnames_bytes) v |= (uint32_t)R.fnames[4 * k + j] << (8 * j);
      tfn[k] = v;
    }
    for (uint32_t k = threadIdx.x; k < w.ph; k += blockDim.x) {
      tpk[k] = R.phash_keys[k];
      tpv[k] = R.phash_vals[k];
    }
    for (uint32_t k = threadIdx.x; k < w.wb; k += blockDim.x) twb[k] = R.walk_bits[k];
    T = LdsTabs{t, tfs, tpk, tpv, twb, (const lds_u8*)tfn};
  } else {
    T = GlbTabs{(glb_u32*)R.nkeys, (glb_u32*)R.fslots, (glb_u32*)R.phash_keys, (glb_u32*)R.phash_vals,
                (glb_u32*)R.walk_bits, (glb_u8*)R.fnames};
  }
  const uint64_t off0 = off[0];
  __syncthreads();
  // software pipeline per wave: iteration k parses stage k from LDS while the
  // stage of k + 1 is in flight into registers and the inputs of k + 2 load
  const size_t gstride = (size_t)gridDim.x * kRawThreads;
  size_t base = (size_t)blockIdx.x * kRawThreads;
  // (a wave with no requests skips the loop and meets the others at the flush)
  RawIn cur = raw_in(off, policy, ingress, port, base + wave * 64 + lane, n);
  RawIn nxt = raw_in(off, policy, ingress, port, base + gstride + wave * 64 + lane, n);
  StageRegs S;
  if (base + (size_t)wave * 64 < n) stage_load(raw, cur, lane, S);
  for (; base < n; base += gstride) {
    const size_t i0 = base + (size_t)wave * 64;
    if (i0 >= n) break;  // wave-uniform
    const size_t i = i0 + lane;
    const bool live = i < n;
    const RawIn nn = raw_in(off, policy, ingress, port, base + 2 * gstride + wave * 64 + lane, n);
    const uint32_t rem = remote[live ? i : 0];
    // stage k: registers → LDS (the previous iteration's reads are done)
    wave_sync();
    stage_store(S, stage, lane);
    const uint64_t sbase = S.base;
    const uint32_t slen = S.len;
    // stage k + 1 into registers, under this iteration's parse
    if (base + gstride < n) stage_load(raw, nxt, lane, S);
    wave_sync();
    if (kMasks) {
      if (kLists) build_masks_lists(stage, slen, tct, masks, lane);
      else build_masks(stage, slen, tct, masks, lane);
      wave_sync();
    }
    const uint32_t prog = live ? lookup_prog(R, T, cur.pol, cur.ing != 0, cur.port) : kProgDeny;
    if (live) {
      // every request but an unknown policy's is parsed: a head the codec
      // rejects is denied in any program (flagged malformed)
      const bool parse = prog != kProgDeny;
      uint32_t key = 0, len = 0, bad = 0;
      uint4* rec = reinterpret_cast<uint4*>(sbuf + rec_off(cur.a - off0, i, cst));
      if (parse) {
        const uint32_t hn = cur.b > cur.a ? (uint32_t)min<uint64_t>(cur.b - cur.a, 0xFFFFFFFFull) : 0u;
        const uint64_t ga = (uint64_t)(uintptr_t)(raw + cur.a);
        const bool in = ga >= sbase && ga + hn <= sbase + slen;
        HeadReader hr(raw + cur.a, hn, stage + (in ? (uint32_t)(ga - sbase) : 0u), in);
        // heads / lists inside the stage parse over its masks, the rest byte by byte
        const uint32_t hs = (uint32_t)(hr.lp - stage);
        bool ok;
        if (kLists) {
          if (hr.n > kFieldsMaxList) {  // spans would not fit: the call fails
            atomicOr(ovf_bytes, kRawListTooLong);
            ok = false;
          } else {
            ok = kMasks && hr.in
                     ? parse_list_masks(R, T, stage, masks, masks + kMaskWords, hs, hs + hr.n, sp, kRawThreads)
                     : parse_list_bytes(R, T, hr, sp, kRawThreads);
          }
        } else {
          ok = kMasks && hr.in
                   ? parse_head_masks(R, T, stage, masks, masks + kMaskWords, hs, hs + hr.n, sp, kRawThreads)
                   : parse_head(R, T, hr, sp, kRawThreads);
        }
        if (!ok) {
          bad = 1;
        } else if (walked_t(R, T, prog)) {
          uint32_t last;
          len = string_len(R, sp, kRawThreads, &last);
          key = len > CG_HTTP_SLOT_BYTES ? kRawKeys - 1 : (len + 15) / 16;
          Out16 o(rec + 1, 1);
          emit_string(R, hr, sp, kRawThreads, last, o);
          if (o.pos) o.flush();
          if (len > CG_HTTP_SLOT_BYTES) atomicAdd(ovf_bytes, (unsigned long long)((4 + len + 15) & ~15u));
        }
      }
      const uint32_t flags = (cur.ing ? CG_HTTP_F_INGRESS : 0u) | (bad ? CG_HTTP_F_MALFORMED : 0u) |
                             (len > CG_HTTP_SLOT_BYTES ? CG_HTTP_F_OVERFLOW : 0u);
      *rec = make_uint4((uint32_t)i, rem, len | flags << 24, prog);
      rinfo[i] = make_uint2(prog, len | bad << 31);
      const uint32_t k = group_of(R, prog) * kRawKeys + key;
      if (lds_keys) __hip_atomic_fetch_add(&lk[k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else atomicAdd(&counts[k], 1u);
    }
    cur = nxt;
    nxt = nn;
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

// ---- pass 2: a slot per request from its bucket's cursor — the block's
// LDS cursor per key (the key's first slot + this block's prefix, lds_keys:
// the same grid and request order as the scan), else a global cursor per key
__global__ __launch_bounds__(kRawThreads) void raw_rank_kernel(HttpRawDev R, size_t n,
                                                               const uint64_t* __restrict__ off, uint32_t cst,
                                                               const uint2* __restrict__ rinfo,
                                                               uint32_t* __restrict__ cursor,
                                                               const uint32_t* __restrict__ bbase, uint32_t lds_keys,
                                                               uint32_t* __restrict__ order) {
  extern __shared__ uint32_t lk[];  // the bucket cursors (lds_keys)
  const uint32_t nk = (R.nprogs + 2) * kRawKeys;
  if (lds_keys)
    for (uint32_t k = threadIdx.x; k < nk; k += blockDim.x) lk[k] = cursor[k] + bbase[(size_t)k * gridDim.x + blockIdx.x];
  const uint64_t off0 = off[0];
  __syncthreads();
  for (size_t base = (size_t)blockIdx.x * kRawThreads; base < n; base += (size_t)gridDim.x * kRawThreads) {
    const size_t i = base + threadIdx.x;
    if (i >= n) continue;
    const uint2 ri = rinfo[i];
    const uint32_t prog = ri.x, len = ri.y & 0x7FFFFFFFu;
    const bool walk = walked(R, prog) && !(ri.y >> 31);
    const uint32_t key = !walk ? 0u : len > CG_HTTP_SLOT_BYTES ? kRawKeys - 1 : (len + 15) / 16;
    const uint32_t k = group_of(R, prog) * kRawKeys + key;
    const uint32_t slot = lds_keys ? atomicAdd(&lk[k], 1u) : atomicAdd(&cursor[k], 1u);
    order[slot] = (uint32_t)(rec_off(off[i] - off0, i, cst) / 16);  // the request's record
  }
}

// Four string bytes through a code map in LDS.
__device__ __forceinline__ uint32_t code4(const uint8_t* lut, uint32_t q) {
  return (uint32_t)lut[q & 0xFFu] | (uint32_t)lut[(q >> 8) & 0xFFu] << 8 | (uint32_t)lut[(q >> 16) & 0xFFu] << 16 |
         (uint32_t)lut[q >> 24] << 24;
}

// ---- pass 3: tiles, a contiguous range per wave (so the run holding a
// tile advances instead of being searched).  The tile's records are gathered
// cooperatively: L = pow2 >= 1 + units lanes per record, lane `sub` of a
// record's group reading its 16-B chunk `sub` (0 = the header, c = string
// unit c - 1), so one load instruction touches 64 / L records' lines instead
// of 64; each lane class-codes its chunk through the program's code map
// (LDS, per wave) and stores it straight to its place in the tile (unit
// sub - 1 of slot s: whole 1 KiB units once the tile's passes are done).
// Header lanes write the meta word and order[slot] = request index, and copy
// strings past the slot into the overflow arena.
__global__ __launch_bounds__(kRawThreads) void raw_build_kernel(
    HttpRawDev R, const HttpRawRun* __restrict__ runs, uint32_t nruns, uint32_t ntiles, HttpTile* __restrict__ ttab,
    uint8_t* __restrict__ tiles, uint32_t* __restrict__ order, const uint8_t* __restrict__ sbuf,
    uint8_t* __restrict__ arena, unsigned long long* __restrict__ arena_cursor) {
  __shared__ __attribute__((aligned(16))) uint8_t s_lut[kRawThreads / 64][256];
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* lut = s_lut[wave];
  uint32_t lut_prog = 0xFFFFFFFFu;
  const uint4* rec16 = reinterpret_cast<const uint4*>(sbuf);
  const uint32_t nwaves = gridDim.x * (kRawThreads / 64), gw = blockIdx.x * (kRawThreads / 64) + wave;
  const uint32_t tpw = (ntiles + nwaves - 1) / nwaves;
  uint32_t t = gw * tpw;
  const uint32_t tend = min(ntiles, t + tpw);
  if (t >= tend) return;
  // the run holding t (runs ascending by t0, covering every tile)
  uint32_t lo = 0, hi = nruns;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (runs[mid].t0 <= t) lo = mid;
    else hi = mid;
  }
  uint32_t ri = lo;
  HttpRawRun run = runs[ri];
  uint32_t next_t0 = ri + 1 < nruns ? runs[ri + 1].t0 : 0xFFFFFFFFu;
  for (; t < tend; ++t) {
    while (t >= next_t0) {
      ++ri;
      run = runs[ri];
      next_t0 = ri + 1 < nruns ? runs[ri + 1].t0 : 0xFFFFFFFFu;
    }
    const uint32_t units = run.units;
    const uint32_t at = run.base + (t - run.t0) * (1 + 2 * units);
    uint8_t* tb = tiles + (size_t)at * 512;
    if (run.prog < R.nprogs && run.prog != lut_prog) {  // the program's code map (wave-uniform)
      wave_sync();  // earlier lookups done
      reinterpret_cast<uint32_t*>(lut)[lane] = reinterpret_cast<const uint32_t*>(R.codes + (size_t)run.prog * 256)[lane];
      wave_sync();
      lut_prog = run.prog;
    }
    const uint32_t r = order[(size_t)t * 64 + lane];  // the slot's record (16-B units), or padding
    const uint32_t L = units == 0 ? 1u : (units < 2 ? 2u : units < 4 ? 4u : units < 8 ? 8u : 16u);
    const uint32_t per = 64 / L, sub = lane & (L - 1), grp = lane & ~(L - 1);
    uint32_t m = 0;  // the longest slot string among this lane's header slots
    for (uint32_t pass = 0; pass < L; ++pass) {
      const uint32_t s = pass * per + lane / L;  // this lane's slot in this pass
      const uint32_t rs = (uint32_t)__shfl((int)r, (int)s, 64);
      const bool pad = rs == 0xFFFFFFFFu;
      uint4 x = make_uint4(0, 0, CG_HTTP_F_PAD << 24, 0);
      if (!pad && sub <= units) x = rec16[(size_t)rs + sub];
      // the record's header word (len | flags << 24), from its group's lane 0
      const uint32_t hz = (uint32_t)__shfl((int)x.z, (int)grp, 64);
      const uint32_t len = hz & 0xFFFFFFu, flags = hz >> 24;
      const bool ovf = flags & CG_HTTP_F_OVERFLOW;
      const uint32_t slen = (pad || ovf) ? 0u : len;
      if (sub == 0) {
        uint32_t aoff16 = 0;
        if (ovf) {
          const unsigned long long ao = atomicAdd(arena_cursor, (unsigned long long)((4 + len + 15) & ~15u));
          aoff16 = (uint32_t)(ao / 16);
          Out16 o(reinterpret_cast<uint4*>(arena + ao), 1);
          o.w0 = len;
          o.pos = 4;
          const uint32_t* s32 = reinterpret_cast<const uint32_t*>(rec16 + rs + 1);
          for (uint32_t k = 0; k < len; k += 4) {
            const uint32_t nb = min(len - k, 4u);
            const uint32_t c = code4(lut, s32[k / 4]);
            o.put4(nb == 4 ? c : c & ((1u << (8 * nb)) - 1u), nb);
          }
          if (o.pos) o.flush();
        }
        if (!pad) order[(size_t)t * 64 + s] = x.x;
        reinterpret_cast<uint2*>(tb)[s] = make_uint2(x.y, (aoff16 & 0xFFFFFFu) | flags << 24);
        m = max(m, slen);
      } else if (sub <= units) {
        // unit sub - 1 of slot s, zero past the string's end
        uint4 c = make_uint4(0, 0, 0, 0);
        const uint32_t u = sub - 1;
        if (16 * u < slen) {
          c = make_uint4(code4(lut, x.x), code4(lut, x.y), code4(lut, x.z), code4(lut, x.w));
          const uint32_t left = slen - 16 * u;  // the string's bytes in this unit
          if (left < 16) {
            const uint32_t m0 = left >= 4 ? 0xFFFFFFFFu : (1u << (8 * left)) - 1u;
            const uint32_t m1 = left >= 8 ? 0xFFFFFFFFu : left <= 4 ? 0u : (1u << (8 * (left - 4))) - 1u;
            const uint32_t m2 = left >= 12 ? 0xFFFFFFFFu : left <= 8 ? 0u : (1u << (8 * (left - 8))) - 1u;
            const uint32_t m3 = left <= 12 ? 0u : (1u << (8 * (left - 12))) - 1u;
            c = make_uint4(c.x & m0, c.y & m1, c.z & m2, c.w & m3);
          }
        }
        reinterpret_cast<uint4*>(tb + 512)[(size_t)u * 64 + s] = c;
      }
    }
    // the tile's tail: the longest string's bytes in its last unit
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    if (lane == 0) {
      const uint32_t tail = units ? m - 16 * (units - 1) : 0u;
      ttab[t] = HttpTile{at, units | tail << 16};
    }
  }
}

unsigned grid_for(size_t n, int cus, unsigned per_cu) {
  const size_t want = (n + kRawThreads - 1) / kRawThreads;
  return (unsigned)std::max<size_t>(1, std::min<size_t>(want, (size_t)cus * per_cu));
}

// LDS of the scan / emit kernels (see wave_stage, key_counters)
bool lds_tables_fit(const HttpRawDev& R) { return raw_tables_lds_words(R) * 4 <= 8 * 1024; }
size_t raw_lds(const HttpRawDev& R, bool lds_keys, bool lds_codes) {
  const size_t nk = ((size_t)R.nprogs + 2) * kRawKeys;
  return (size_t)std::max(R.nfields, 1u) * kRawThreads * 4 + 4 * (size_t)kStage + 4 * 2 * (kStage / 8) + 256 +
         (lds_keys ? nk * 4 : 0) + (lds_tables_fit(R) ? (size_t)raw_tables_lds_words(R) * 4 : 0) +
         (lds_codes ? (size_t)R.nprogs * 256 : 0) + 16;  // + slack: a quad read may pass the last stage by 7 bytes
}
// code maps in LDS only while small: a larger table costs workgroups per CU
// (occupancy) more than its global (L1-cached) lookups cost
bool lds_codes_fit(const HttpRawDev& R) { return (size_t)R.nprogs * 256 <= 4 * 1024; }

}  // namespace

size_t http_raw_grid(size_t n, int cus) { return grid_for(n, cus, 4); }

bool http_raw_lds_keys(const HttpRawDev& R) { return ((size_t)R.nprogs + 2) * kRawKeys * 4 <= 32 * 1024; }

int launch_http_raw_scan(const HttpRawDev& R, bool lists, const uint8_t* raw, const uint64_t* off, size_t n,
                         const uint32_t* policy, const uint8_t* ingress, const uint16_t* port, uint32_t* counts,
                         void* rinfo, const uint32_t* remote, uint8_t* sbuf, uint32_t cst,
                         unsigned long long* ovf_bytes, void* stream, int cus) {
  if (!n) return 0;
  const bool lk = http_raw_lds_keys(R);
  const size_t lds = raw_lds(R, lk, false);
  // CG_RAW_PARSE=bytes: HeadReader parsing for staged requests too (A/B)
  static const bool masks = [] {
    const char* e = getenv("CG_RAW_PARSE");
    return !(e && std::string(e) == "bytes");
  }();
  const bool tabs = lds_tables_fit(R);
  decltype(&raw_scan_kernel<false, false, false>) kern;
  if (lists)
    kern = masks ? (tabs ? raw_scan_kernel<true, true, true> : raw_scan_kernel<true, true, false>)
                 : (tabs ? raw_scan_kernel<true, false, true> : raw_scan_kernel<true, false, false>);
  else
    kern = masks ? (tabs ? raw_scan_kernel<false, true, true> : raw_scan_kernel<false, true, false>)
                 : (tabs ? raw_scan_kernel<false, false, true> : raw_scan_kernel<false, false, false>);
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(kern, dim3((unsigned)http_raw_grid(n, cus)), dim3(kRawThreads), lds, (hipStream_t)stream, R, raw,
                     off, n, policy, ingress, port, counts, (uint2*)rinfo, remote, sbuf, cst, ovf_bytes, (uint32_t)lk);
  return (int)hipGetLastError();
}

int launch_http_raw_prefix(const uint32_t* bcount, uint32_t nkeys, uint32_t nblk, uint32_t* bbase, uint32_t* hist,
                           void* stream) {
  if (!nkeys) return 0;
  hipLaunchKernelGGL(raw_prefix_kernel, dim3(nkeys), dim3(256), 0, (hipStream_t)stream, bcount, nblk, bbase, hist);
  return (int)hipGetLastError();
}

int launch_http_raw_rank(const HttpRawDev& R, size_t n, const uint64_t* off, uint32_t cst, const void* rinfo,
                         uint32_t* cursor, const uint32_t* bbase, uint32_t* order, void* stream, int cus) {
  if (!n) return 0;
  const bool lk = http_raw_lds_keys(R);
  const size_t lds = lk ? ((size_t)R.nprogs + 2) * kRawKeys * 4 : 0;
  hipLaunchKernelGGL(raw_rank_kernel, dim3((unsigned)http_raw_grid(n, cus)), dim3(kRawThreads), lds,
                     (hipStream_t)stream, R, n, off, cst, (const uint2*)rinfo, cursor, bbase, (uint32_t)lk, order);
  return (int)hipGetLastError();
}

int launch_http_raw_build(const HttpRawDev& R, const HttpRawRun* runs, uint32_t nruns, uint32_t ntiles,
                          HttpTile* ttab, uint8_t* tiles, uint32_t* order, const uint8_t* sbuf, uint8_t* arena,
                          unsigned long long* arena_cursor, void* stream, int cus) {
  if (!ntiles) return 0;
  const unsigned waves = kRawThreads / 64;
  const unsigned grid =
      (unsigned)std::max<size_t>(1, std::min<size_t>((ntiles + waves - 1) / waves, (size_t)cus * 8));
  hipLaunchKernelGGL(raw_build_kernel, dim3(grid), dim3(kRawThreads), 0, (hipStream_t)stream, R, runs, nruns, ntiles,
                     ttab, tiles, order, sbuf, arena, arena_cursor);
  return (int)hipGetLastError();
}

}  // namespace cg
