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
#include <map>
#include <mutex>
#include <tuple>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "../../include/cilium_gpu.h"
#include "dev_types.h"
#include "http_walk.h"
#include "raw_emit.h"
#include "kernels.h"

namespace cg {

namespace {

constexpr int kRawThreads = (int)kRawScanThreads;
constexpr uint32_t kRawWaves = kRawThreads / 64;

// CG_RAW_CLOCKS (experiment builds only, tools/exp_http.py raw_clocks): the
// scan's phases timed per wave with the shader clock; one wave prints its
// totals at the end
#ifdef CG_RAW_CLOCKS
#define RAW_CLK(v) v = clock64()
#define RAW_ACC(slot, a, b) clk[slot] += (b) - (a)
// inside parse_head_fast: time since the last mark into g_pclk[slot]
__device__ unsigned long long g_pclk[8];
#define RAW_PMARK(slot)                                                           \
  do {                                                                           \
    const uint64_t now_ = clock64();                                             \
    if (blockIdx.x == 7 && threadIdx.x == 64) g_pclk[slot] += now_ - pm_;        \
    pm_ = now_;                                                                  \
  } while (0)
#define RAW_PSTART uint64_t pm_ = clock64()
#else
#define RAW_CLK(v)
#define RAW_ACC(slot, a, b)
#define RAW_PMARK(slot)
#define RAW_PSTART
#endif
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
  P32 nkeys, fslots, phk, phv, walk, dflt;
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

// http_parser.h HTTP_METHOD_MAP (v2.8): the methods s_req_method accepts
// (case-sensitive; http_parse.cc known_method), in 64 slots of {bytes 0-3,
// bytes 4-7, bytes 8-10 | length << 24, 0} under a perfect hash of (bytes
// 0-3, length) — one 16-byte read and three compares per head.
constexpr const char* kMethodNames[] = {
    "DELETE", "GET",    "HEAD",     "POST",   "PUT",   "CONNECT",    "OPTIONS",    "TRACE",    "COPY",
    "LOCK",   "MKCOL",  "MOVE",     "PROPFIND", "PROPPATCH", "SEARCH", "UNLOCK",   "BIND",     "REBIND",
    "UNBIND", "ACL",    "REPORT",   "MKACTIVITY", "CHECKOUT", "MERGE", "M-SEARCH", "NOTIFY",   "SUBSCRIBE",
    "UNSUBSCRIBE", "PATCH", "PURGE", "MKCALENDAR", "LINK",  "UNLINK"};
constexpr uint32_t kMethodMaxLen = 11, kMethodSlots = 64;
constexpr uint32_t method_slot(uint32_t w0, uint32_t len) { return ((w0 + len * 0x9E3779B1u) * 0x00C93D79u) >> 26; }
struct MethodTab {
  uint32_t e[kMethodSlots][4];
  uint32_t collisions;
};
constexpr uint32_t cstr_len(const char* s) { return *s ? 1 + cstr_len(s + 1) : 0; }
constexpr uint32_t cstr_word(const char* s, uint32_t len, uint32_t at) {
  uint32_t w = 0;
  for (uint32_t j = 0; j < 4; ++j)
    if (at + j < len) w |= (uint32_t)(uint8_t)s[at + j] << (8 * j);
  return w;
}
constexpr MethodTab make_method_tab() {
  MethodTab t{};
  for (const char* m : kMethodNames) {
    const uint32_t n = cstr_len(m), w0 = cstr_word(m, n, 0);
    uint32_t* e = t.e[method_slot(w0, n)];
    t.collisions += e[2] != 0;
    e[0] = w0;
    e[1] = cstr_word(m, n, 4);
    e[2] = cstr_word(m, n, 8) | n << 24;
  }
  return t;
}
constexpr MethodTab kMethodTabHost = make_method_tab();
static_assert(kMethodTabHost.collisions == 0, "method_slot must place every method in its own slot");
__device__ const MethodTab kMethodTab = make_method_tab();
// the method's words (bytes past its length zero) against the table slot e
__device__ __forceinline__ bool method_known(uint4 e, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t len) {
  return len <= kMethodMaxLen && e.x == w0 && e.y == w1 && e.z == (w2 | len << 24);
}

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

// 6 KiB: 64 heads of ~70 B fit with room to spare (heads past the stage are
// read from HBM), and four waves' stages leave room for 3+ workgroups per CU
// (8 KiB: 1.69, 6 KiB: 2.01, 4 KiB: 1.12 G requests/s on config 5)
constexpr uint32_t kStage = 6144;
constexpr uint32_t kMaskWords = kStage / 32;  // u32 words per structural mask of a stage
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

// Content-Length (http_parser h_content_length) over the value's bytes from
// its first non-OWS byte a to its line end e: digits, then SP only, the
// value never past (ULLONG_MAX - 10) / 10 before a digit is appended.
template <class Byte>
__device__ __forceinline__ bool content_length_ok(uint32_t a, uint32_t e, Byte byte) {
  uint64_t cl = 0;
  uint32_t p = a;
  for (; p < e; ++p) {
    const uint32_t d = byte(p) - '0';
    if (d > 9u) break;
    if (cl > (~0ull - 10) / 10) return false;
    cl = cl * 10 + d;
  }
  if (p == a) return false;
  for (; p < e; ++p)
    if (byte(p) != ' ') return false;
  return true;
}
// "content-length" from a name's length and lowercased key words (first 8,
// last 8 bytes: bytes 0-7 and 6-13 of the 14)
__device__ __forceinline__ bool is_content_length(uint32_t nl, uint32_t lo0, uint32_t lo1, uint32_t hi0, uint32_t hi1) {
  return nl == 14 && lo0 == 0x746E6F63u && lo1 == 0x2D746E65u && hi0 == 0x656C2D74u && hi1 == 0x6874676Eu;
}
// Four target bytes all in 0x21-0x7E (strict normal_url_char; '?' and '#'
// are accepted as state changes)
__device__ __forceinline__ bool all_url(uint32_t q) { return all_plain(q) && !(q & 0x80808080u); }

// parse_head (http_parse.cc) for one head: the value span {start << 16 |
// length} of every field it sets in sp[f * stride] (kAbsentSpan otherwise);
// false = the codec or the connection manager stops the request before the
// filter (http_parse.cc's rules: leading CR / LF skipped, http_parser's
// methods, SP+, a '/' target of 0x21-0x7E bytes, HTTP/1.1, CR LF or a bare
// LF at every line end, Content-Length digits, Host required).
template <class Tabs>
__device__ __forceinline__ bool parse_head(const HttpRawDev& R, const Tabs& T, HeadReader& hr, lds_u32* sp,
                                           uint32_t stride) {
  for (uint32_t f = 0; f < R.nfields; ++f) sp[f * stride] = kAbsentSpan;
  const uint32_t n = hr.n;
  if (n > kRawMaxHead) return false;
  uint32_t k = 0;
  while (k < n && (hr.at(k) == '\r' || hr.at(k) == '\n')) ++k;  // s_start_req
  const uint32_t ms = k;
  while (k < n && tchar(hr.at(k))) ++k;  // method
  if (k == ms || k >= n || hr.at(k) != ' ') return false;
  const uint32_t mlen = k - ms;
  {
    uint32_t w[3] = {0, 0, 0};
    for (uint32_t j = 0; j < min(mlen, 12u); ++j) w[j >> 2] |= hr.at(ms + j) << (8 * (j & 3));
    const uint32_t* e = kMethodTab.e[method_slot(w[0], mlen)];
    if (!method_known(make_uint4(e[0], e[1], e[2], e[3]), w[0], w[1], w[2], mlen)) return false;
  }
  while (k < n && hr.at(k) == ' ') ++k;  // s_req_spaces_before_url
  const uint32_t t0 = k;
  while (k < n) {  // request-target
    if (k + 4 <= n && all_url(hr.quad(k))) {
      k += 4;
      continue;
    }
    const uint32_t c = hr.at(k);
    if (c <= 0x20 || c >= 0x7F) break;
    ++k;
  }
  if (k == t0 || hr.at(t0) != '/' || k >= n || hr.at(k) != ' ') return false;
  const uint32_t tlen = k - t0;
  ++k;
  if (k + 9 > n) return false;  // "HTTP/1.1" LF
  if (hr.at(k) != 'H' || hr.at(k + 1) != 'T' || hr.at(k + 2) != 'T' || hr.at(k + 3) != 'P' || hr.at(k + 4) != '/' ||
      hr.at(k + 5) != '1' || hr.at(k + 6) != '.' || hr.at(k + 7) != '1')
    return false;
  k += 8;
  if (hr.at(k) == '\n') {
    k += 1;
  } else if (hr.at(k) == '\r' && k + 1 < n && hr.at(k + 1) == '\n') {
    k += 2;
  } else {
    return false;
  }
  bool have_host = false, have_cl = false;
  uint32_t auth = kAbsentSpan;
  while (true) {
    if (k >= n) return false;  // no empty line: incomplete head
    {
      const uint32_t x0 = hr.at(k);
      if (x0 == '\n') break;  // empty line: end of head
      if (x0 == '\r') {
        if (k + 1 < n && hr.at(k + 1) == '\n') break;
        return false;
      }
    }
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
    uint32_t v = c + 1, first = kAbsentSpan, lend = v, nxt;
    while (true) {  // field-value up to the line end: IS_HEADER_CHAR, OWS trimmed
      if (v + 4 <= n && all_plain(hr.quad(v))) {
        if (first == kAbsentSpan) first = v;
        v += 4;
        lend = v;
        continue;
      }
      if (v >= n) return false;
      const uint32_t x = hr.at(v);
      if (x == '\n') {  // a bare LF ends the line
        nxt = v + 1;
        break;
      }
      if (x == '\r') {
        if (v + 1 < n && hr.at(v + 1) == '\n') {
          nxt = v + 2;
          break;
        }
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
    auto lw = [&](uint32_t at) { return lower(hr.at(at)); };
    const bool is_host = nl == 4 && lw(k) == 'h' && lw(k + 1) == 'o' && lw(k + 2) == 's' && lw(k + 3) == 't';
    if (is_host) {
      if (!have_host) auth = span;  // the first value is the one the filter sees
      have_host = true;
    } else {
      if (nl == 14 && first != kAbsentSpan) {  // h_content_length
        bool cl = true;
        for (uint32_t j = 0; j < 14 && cl; ++j) cl = lw(k + j) == (uint32_t)"content-length"[j];
        if (cl && (have_cl || !content_length_ok(first, v, [&](uint32_t p) { return hr.at(p); }))) return false;
        have_cl |= cl;
      }
      const int f = field_of(R, T, hr, h, nl, k);
      if (f >= 0 && sp[f * stride] == kAbsentSpan) sp[f * stride] = span;  // first value wins
    }
    k = nxt;
  }
  if (!have_host) return false;  // the connection manager answers 400 without Host
  if (R.f_method >= 0) sp[R.f_method * stride] = ms << 16 | mlen;
  if (R.f_path >= 0) sp[R.f_path * stride] = t0 << 16 | tlen;
  if (R.f_authority >= 0) sp[R.f_authority * stride] = auth;
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
  return pack4(lt | del | (x & 0x80808080u));  // bytes >= 0x80 end a target (strict URL bytes)
}
// 16 stage bytes per lane per round (rounds wave-uniform, so a lane's pair
// partner is always active): the half-words of a mask word come from lanes
// 2m and 2m + 1, joined by a DPP pair swap.  (32 bytes per lane left the
// last of three rounds a fifth full at config 5's ~4.5 KB stages.)
__device__ __forceinline__ uint32_t pair_swap(uint32_t x) {  // quad_perm [1, 0, 3, 2]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
}
template <class Classify>
__device__ __forceinline__ void build_masks16(const lds_u8* stage, uint32_t slen, lds_u32* masks, uint32_t lane,
                                              Classify classify) {
  for (uint32_t r = 0; r * 1024 < slen; ++r) {
    const uint32_t u = r * 64 + lane;  // this lane's 16-byte unit
    const uint4 a = to_uint4(*(const lds_v4*)(stage + 16 * u));
    uint32_t m0, m1;  // 16-bit masks of the unit
    classify(a, m0, m1);
    const uint32_t o0 = pair_swap(m0), o1 = pair_swap(m1);
    if (!(lane & 1u)) {
      masks[u >> 1] = m0 | o0 << 16;
      masks[kMaskWords + (u >> 1)] = m1 | o1 << 16;
    }
  }
}
__device__ __forceinline__ void build_masks(const lds_u8* stage, uint32_t slen, const lds_u8* tct, lds_u32* masks,
                                            uint32_t lane) {
  build_masks16(stage, slen, masks, lane, [&](const uint4& a, uint32_t& sp, uint32_t& nt) {
    const uint32_t d[4] = {a.x, a.y, a.z, a.w};
    sp = nt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sp |= special4(d[k]) << (4 * k);
#pragma unroll
      for (int j = 0; j < 4; ++j) nt |= (uint32_t)tct[(d[k] >> (8 * j)) & 0xFFu] << (4 * k + j);
    }
  });
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

// The special / nontchar bits of 128 stage bytes from `base` (a multiple of
// 32) in registers: a lane's find-next-set over its head is register work,
// the LDS masks are read past the window only (heads beyond ~100 bytes).
struct MaskWin {
  uint32_t s[4], n[4];  // mask words base / 32 .. + 3
  uint32_t base;
};
__device__ __forceinline__ MaskWin load_win(const lds_u32* msp, const lds_u32* mnt, uint32_t hs) {
  const uint32_t w = hs >> 5;
  MaskWin W;
  W.base = w << 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    W.s[j] = msp[w + j];
    W.n[j] = mnt[w + j];
  }
  return W;
}
// window word j (0..3; 0 past the window), selected without a branch
__device__ __forceinline__ uint32_t win_word(const uint32_t (&w)[4], uint32_t j) {
  return j == 0 ? w[0] : j == 1 ? w[1] : j == 2 ? w[2] : j == 3 ? w[3] : 0u;
}
// next_set over a window (p >= base): the 128 bits as two 64-bit halves in
// registers — the rest of p's half, then the high half — then the LDS mask
__device__ __forceinline__ uint32_t wnext(const uint32_t (&w)[4], uint32_t base, const lds_u32* m, uint32_t p,
                                          uint32_t lim) {
  const uint32_t r = p - base;
  const uint64_t lo = (uint64_t)w[1] << 32 | w[0], hi = (uint64_t)w[3] << 32 | w[2];
  const bool inlo = r < 64;
  const uint64_t a = r < 128 ? (inlo ? lo : hi) >> (r & 63) : 0ull;
  const uint64_t b = inlo ? hi : 0ull;
  if (a) return min(p + (uint32_t)__builtin_ctzll(a), lim);
  if (b) return min(base + 64 + (uint32_t)__builtin_ctzll(b), lim);
  // the first bit the window did not cover
  const uint32_t q = r < 128 ? base + 128 : p;
  return q >= lim ? lim : next_set(m, q, lim);
}
// the bit at p (p >= base)
__device__ __forceinline__ bool wbit(const uint32_t (&w)[4], uint32_t base, const lds_u32* m, uint32_t p) {
  const uint32_t r = p - base;
  return r < 128 ? (win_word(w, r >> 5) >> (r & 31)) & 1u : (m[p >> 5] >> (p & 31)) & 1u;
}

// The field of a header name from its key words (lowercased by the caller;
// lo1 / hi0 / hi1 zero where the name is shorter), or -1: R.nkeys
// (raw_name_key), the bytes between the first and last 8 verified for longer
// names.
// A name-key slot's 8 words as two 16-byte loads (one round trip, not one
// per compared word).
__device__ __forceinline__ void key_slot(const lds_u32* p, uint4& a, uint4& b) {
  a = to_uint4(*(const lds_v4*)p);
  b = to_uint4(*(const lds_v4*)(p + 4));
}
__device__ __forceinline__ void key_slot(glb_u32* p, uint4& a, uint4& b) {
  a = to_uint4(*(glb_v4*)p);
  b = to_uint4(*(glb_v4*)(p + 4));
}
template <class Tabs>
__device__ __forceinline__ int field_of_words(const HttpRawDev& R, const Tabs& T, const lds_u8* st, uint32_t k,
                                              uint32_t nl, uint32_t lo0, uint32_t lo1, uint32_t hi0, uint32_t hi1) {
  uint32_t sl = raw_name_hash(nl, lo0, lo1, hi0, hi1) & R.nkmask;
  for (uint32_t probe = 0; probe <= R.nkmask; ++probe) {
    uint4 a, b;  // {len, lo0, lo1, hi0}, {hi1, field, name offset, -}
    key_slot(T.nkeys + 8 * sl, a, b);
    if (a.x == 0) return -1;
    if (a.x == nl && a.y == lo0 && a.z == lo1 && a.w == hi0 && b.x == hi1) {
      bool eq = true;
      for (uint32_t j = 8; j + 8 < nl && eq; ++j) eq = lower(sbyte(st, k + j)) == T.fnames[b.z + j];
      if (eq) return (int)b.y;
    }
    sl = (sl + 1) & R.nkmask;
  }
  return -1;
}

// A parsed request: the value span {start - hs << 16 | length} of each field
// it sets, in sp[f * stride] for the bits of `present`, and the sum of their
// lengths (the walked string's length follows: walked_len).
struct Parsed {
  uint32_t present, vsum;
  __device__ __forceinline__ void set(lds_u32* sp, uint32_t stride, uint32_t f, uint32_t span) {
    sp[f * stride] = span;
    present |= 1u << f;
    vsum += span & 0xFFFFu;
  }
};
__device__ __forceinline__ uint32_t walked_len(const HttpRawDev& R, const Parsed& P, uint32_t* last_out) {
  const uint32_t last = P.present ? 32u - (uint32_t)__builtin_clz(P.present) : 0u;
  const uint32_t np = (uint32_t)__popc(P.present);
  *last_out = last;
  return P.vsum + np + 2u * (last - np) + (last < R.nfields ? 1u : 0u);
}

// parse_head (http_parse.cc semantics) for a head inside the stage, bytes
// [hs, he), over the structural masks.  Reads are issued in batches: the
// request line's delimiter bytes, method words and version in one round trip,
// then per header line its first bytes, the name's end byte and key words and
// the value's first two specials in one.  The leniencies of http_parser that
// cost a loop (CR / LF before the request line, more than one SP before the
// target) are found by bit tests on the masks and only then walked.
template <class Tabs>
__device__ __forceinline__ bool parse_head_fast(const HttpRawDev& R, const Tabs& T, const lds_u8* st,
                                                const lds_u32* msp, const lds_u32* mnt, const lds_u32* mtab,
                                                uint32_t hs, uint32_t he, lds_u32* sp, uint32_t stride, Parsed& P) {
  RAW_PSTART;
  P.present = P.vsum = 0;
  if (he - hs > kRawMaxHead) return false;
  const MaskWin W = load_win(msp, mnt, hs);
  auto nS = [&](uint32_t p) { return p >= he ? he : wnext(W.s, W.base, msp, p, he); };
  auto nN = [&](uint32_t p) { return p >= he ? he : wnext(W.n, W.base, mnt, p, he); };
  uint32_t ms = hs;  // s_start_req: CR / LF before the method are skipped
  if (hs < he && wbit(W.s, W.base, msp, hs))
    while (ms < he && (sbyte(st, ms) == '\r' || sbyte(st, ms) == '\n')) ++ms;
  const uint32_t m = nN(ms);  // method: a tchar run, then SP
  uint32_t t0 = m + 1;
  uint32_t te = nS(t0);  // request-target: plain bytes, then SP
  if (te == t0 && t0 < he) {  // a special first: more SP (s_req_spaces_before_url) or a rejected head
    while (t0 < he && sbyte(st, t0) == ' ') ++t0;
    te = nS(t0);
  }
  // SP at m; method words; '/' at t0; " HTTP/1.1" then CR LF or LF at te
  const uint32_t bm = sbyte(st, m), bt = sbyte(st, t0), q0 = squad(st, te), q1 = squad(st, te + 4),
                 q2 = squad(st, te + 8), a0 = squad(st, ms), a1 = squad(st, ms + 4), a2 = squad(st, ms + 8);
  const uint32_t ml = m - ms;
  const uint32_t w0 = keep_bytes(a0, ml), w1 = ml > 4 ? keep_bytes(a1, ml - 4) : 0u,
                 w2 = ml > 8 ? keep_bytes(a2, ml - 8) : 0u;
  const uint4 me = to_uint4(*(const lds_v4*)(mtab + 4 * method_slot(w0, ml)));
  const bool lf_only = (q2 >> 8 & 0xFFu) == '\n';
  uint32_t k = te + (lf_only ? 10u : 11u);
  if (m == ms || m >= he || te == t0 || k > he) return false;
  if (bm != ' ' || bt != '/' || q0 != 0x54544820u || q1 != 0x2E312F50u || (q2 & 0xFFu) != '1' ||
      (!lf_only && (q2 >> 8 & 0xFFFFu) != 0x0A0Du))
    return false;
  RAW_PMARK(0);  // window, request line
  bool have_host = false, have_cl = false;
  uint32_t auth = kAbsentSpan;
  while (true) {
    if (k >= he) return false;  // no empty line: incomplete head
    // a line starting with a special byte is the empty line (CR LF or a
    // bare LF) or a rejected head: one bit test, no searches
    if (wbit(W.s, W.base, msp, k)) {
      const uint32_t q = squad(st, k);
      if ((q & 0xFFu) == '\n' || ((q & 0xFFFFu) == 0x0A0Du && k + 1 < he)) break;  // empty line: end of head
      return false;
    }
    const uint32_t c = nN(k);       // name: a tchar run, then ':'
    const uint32_t s1 = nS(c + 1);  // the value's first special, and the one after it
    const uint32_t s2 = nS(s1 + 1);
    const uint32_t qk = squad(st, k), bc = sbyte(st, c), r1 = squad(st, k + 4), r2 = squad(st, c - 8),
                   r3 = squad(st, c - 4), q1 = squad(st, s1), q2 = squad(st, s2);
    RAW_PMARK(1);  // a line's searches and reads
    if (c == k || c >= he || bc != ':') return false;
    const uint32_t nl = c - k;
    // field-value to the line end: IS_HEADER_CHAR (bytes >= 0x80 are
    // specials of the mask that belong to the value), OWS trimmed
    uint32_t v = c + 1, first = kAbsentSpan, lend = v, s = s1, q = q1, nxt;
    for (uint32_t it = 0;; ++it) {
      if (s > v) {
        if (first == kAbsentSpan) first = v;
        lend = s;
      }
      if (s >= he) return false;
      const uint32_t x = q & 0xFFu;
      if (x == ' ' || x == '\t' || x >= 0x80) {
        if (x >= 0x80) {
          if (first == kAbsentSpan) first = s;
          lend = s + 1;
        }
        v = s + 1;
        if (it == 0) {
          s = s2;
          q = q2;
        } else {
          s = nS(v);
          q = squad(st, s);
        }
        continue;
      }
      if (x == '\n') {  // a bare LF ends the line
        nxt = s + 1;
        break;
      }
      if (x == '\r' && s + 1 < he && (q >> 8 & 0xFFu) == '\n') {
        nxt = s + 2;
        break;
      }
      return false;
    }
    RAW_PMARK(2);  // value loop
    const uint32_t span = first == kAbsentSpan ? ((s - hs) << 16) : ((first - hs) << 16 | (lend - first));
    // "host" in any case: OR-ing 0x20 lowers letters and maps no other
    // token byte onto one
    if (nl == 4 && (qk | 0x20202020u) == 0x74736F68u) {
      if (!have_host) auth = span;  // the first value is the one the filter sees
      have_host = true;
    } else {
      const uint32_t lo0 = lower4(keep_bytes(qk, nl));
      const uint32_t lo1 = nl > 4 ? lower4(keep_bytes(r1, nl - 4)) : 0u;
      const uint32_t hi0 = nl > 8 ? lower4(r2) : 0u, hi1 = nl > 8 ? lower4(r3) : 0u;
      if (is_content_length(nl, lo0, lo1, hi0, hi1) && first != kAbsentSpan) {  // h_content_length
        if (have_cl || !content_length_ok(first, s, [&](uint32_t p) { return sbyte(st, p); })) return false;
        have_cl = true;
      }
      const int f = field_of_words(R, T, st, k, nl, lo0, lo1, hi0, hi1);
      if (f >= 0 && !(P.present >> f & 1u)) P.set(sp, stride, (uint32_t)f, span);  // first value wins
    }
    k = nxt;
    RAW_PMARK(3);  // name key, span
  }
  RAW_PMARK(4);
  // the method (read above, under the header lines) and Host: the
  // connection manager answers 400 without Host
  if (!have_host || !method_known(me, w0, w1, w2, ml)) return false;
  if (R.f_method >= 0) P.set(sp, stride, (uint32_t)R.f_method, (ms - hs) << 16 | ml);
  if (R.f_path >= 0) P.set(sp, stride, (uint32_t)R.f_path, (t0 - hs) << 16 | (te - t0));
  if (R.f_authority >= 0) P.set(sp, stride, (uint32_t)R.f_authority, auth);
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
  build_masks16(stage, slen, masks, lane, [&](const uint4& a, uint32_t& st, uint32_t& zr) {
    const uint32_t d[4] = {a.x, a.y, a.z, a.w};
    st = zr = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      zr |= zero4(d[k]) << (4 * k);
#pragma unroll
      for (int j = 0; j < 4; ++j) st |= (uint32_t)tct[(d[k] >> (8 * j)) & 0xFFu] << (4 * k + j);
    }
  });
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
__device__ __forceinline__ bool parse_list_fast(const HttpRawDev& R, const Tabs& T, const lds_u8* st,
                                                const lds_u32* mstop, const lds_u32* mzero, uint32_t hs, uint32_t he,
                                                lds_u32* sp, uint32_t stride, Parsed& P) {
  P.present = P.vsum = 0;
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
    int f = R.f_empty;
    if (nl) {
      const uint32_t lo0 = lower4(keep_bytes(squad(st, k), nl));
      const uint32_t lo1 = nl > 4 ? lower4(keep_bytes(squad(st, k + 4), nl - 4)) : 0u;
      const uint32_t hi0 = nl > 8 ? lower4(squad(st, k + nl - 8)) : 0u, hi1 = nl > 8 ? lower4(squad(st, k + nl - 4)) : 0u;
      f = field_of_words(R, T, st, k, nl, lo0, lo1, hi0, hi1);
    }
    if (f >= 0 && !(P.present >> f & 1u)) P.set(sp, stride, (uint32_t)f, (v - hs) << 16 | (e - v));  // first value wins
    k = e < he ? e + 1 : he;
  }
  return ok;
}

// parse_list_fast with the first 128 bits of both masks in registers
// (MaskWin: s = stop, n = NUL): a short list's searches are register work,
// and a stop byte is told from a NUL by the NUL window, not a byte read.
// For header lists of HTTP snapshots (not raw_values).
template <class Tabs>
__device__ __forceinline__ bool parse_list_win(const HttpRawDev& R, const Tabs& T, const lds_u8* st,
                                               const lds_u32* mstop, const lds_u32* mzero, uint32_t hs, uint32_t he,
                                               lds_u32* sp, uint32_t stride, Parsed& P) {
  P.present = P.vsum = 0;
  const MaskWin W = load_win(mstop, mzero, hs);
  bool ok = true;
  for (uint32_t k = hs; k < he;) {
    const uint32_t ne = wnext(W.n, W.base, mzero, k, he), nl = ne - k;
    const uint32_t v = ne < he ? ne + 1 : he;
    const uint32_t s = v < he ? wnext(W.s, W.base, mstop, v, he) : he;
    uint32_t e = s;
    if (s < he && !wbit(W.n, W.base, mzero, s)) {  // a byte the codec rejects
      ok = false;
      e = wnext(W.n, W.base, mzero, s, he);
    }
    int f = R.f_empty;
    if (nl) {
      const uint32_t lo0 = lower4(keep_bytes(squad(st, k), nl));
      const uint32_t lo1 = nl > 4 ? lower4(keep_bytes(squad(st, k + 4), nl - 4)) : 0u;
      const uint32_t hi0 = nl > 8 ? lower4(squad(st, k + nl - 8)) : 0u, hi1 = nl > 8 ? lower4(squad(st, k + nl - 4)) : 0u;
      f = field_of_words(R, T, st, k, nl, lo0, lo1, hi0, hi1);
    }
    if (f >= 0 && !(P.present >> f & 1u)) P.set(sp, stride, (uint32_t)f, (v - hs) << 16 | (e - v));  // first value wins
    k = e < he ? e + 1 : he;
  }
  return ok;
}

// parse_list_win's result for ONE list [hs, he) computed by the whole wave
// (the ring's single-request calls, which would otherwise parse on one lane
// while 63 wait).  The pairs follow from the NULs alone: pair j's name ends
// at NUL 2j, its value [NUL 2j + 1, NUL 2j + 1) — the value's first stop byte
// is either a byte the codec rejects or that NUL, so the list is malformed
// iff a stop that is not a NUL lies where an odd number of NULs precede it.
// Lanes take the mask words: NUL counts scanned over the wave, their
// positions ranked into scr, the odd-parity regions by a prefix XOR of each
// word; then lane j decides pair j, the first pair of each field wins (by
// ballot, lowest lane first) and the spans go to sp0 (request 0's column).
// Returns false, having written nothing, when the list holds more than 127
// NULs (64+ pairs): the caller parses it on one lane.
constexpr uint32_t kCoopNuls = 127;
// (the ring's NUL ranks go after a single-request call's bytes in its data area)
static_assert(64 + kRingBlob + 16 + 4 * kCoopNuls <= kRingDataMax, "ring scratch for parse_list_coop");
template <class Tabs>
__device__ __forceinline__ bool parse_list_coop(const HttpRawDev& R, const Tabs& T, const lds_u8* st,
                                                const lds_u32* mstop, const lds_u32* mzero, uint32_t hs, uint32_t he,
                                                lds_u32* sp0, uint32_t stride, lds_u32* scr, uint32_t lane, Parsed& P,
                                                bool& ok) {
  const uint32_t w_lo = hs >> 5, w_end = he > hs ? ((he - 1) >> 5) + 1 : w_lo;
  uint32_t m = 0;       // NULs so far (wave-uniform)
  bool bad = false;     // a rejected byte inside a value (this lane's words)
  for (uint32_t w0 = w_lo; w0 < w_end; w0 += 64) {  // uniform
    const uint32_t w = w0 + lane;
    uint32_t z = 0, b = 0;
    if (w < w_end) {
      uint32_t keep = 0xFFFFFFFFu;
      if (w == w_lo) keep &= 0xFFFFFFFFu << (hs & 31);
      if (w == (he - 1) >> 5 && (he & 31)) keep &= (1u << (he & 31)) - 1u;
      z = mzero[w] & keep;
      b = mstop[w] & ~mzero[w] & keep;
    }
    // exclusive prefix of the NUL counts over the lanes
    const uint32_t c = (uint32_t)__popc(z);
    uint32_t inc = c;
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
      if (lane >= o) inc += y;
    }
    const uint32_t r0 = m + inc - c;
    m += (uint32_t)__shfl((int)inc, 63, 64);
    if (m > kCoopNuls) return false;  // uniform
    // odd-parity positions: NULs before them in the word (exclusive prefix
    // XOR of z) plus the parity carried in
    uint32_t px = z;
    px ^= px << 1;
    px ^= px << 2;
    px ^= px << 4;
    px ^= px << 8;
    px ^= px << 16;
    const uint32_t inside = (px ^ z) ^ ((r0 & 1u) ? 0xFFFFFFFFu : 0u);
    bad |= (b & inside) != 0;
    for (uint32_t r = r0; z; z &= z - 1, ++r) scr[r] = 32 * w + (uint32_t)__builtin_ctz(z);
  }
  ok = !__ballot(bad);
  wave_sync();  // the NUL positions
  // pair j: name [k, ne), value [v, e)
  const uint32_t j = lane;
  const bool has = j == 0 ? hs < he : (2 * j - 1 < m && scr[2 * j - 1] + 1 < he);
  int f = -1;
  uint32_t span = 0;
  if (has) {
    const uint32_t k = j ? scr[2 * j - 1] + 1 : hs;
    const uint32_t ne = 2 * j < m ? scr[2 * j] : he, nl = ne - k;
    const uint32_t v = ne < he ? ne + 1 : he;
    const uint32_t e = 2 * j + 1 < m ? scr[2 * j + 1] : he;
    f = R.f_empty;
    if (nl) {
      const uint32_t lo0 = lower4(keep_bytes(squad(st, k), nl));
      const uint32_t lo1 = nl > 4 ? lower4(keep_bytes(squad(st, k + 4), nl - 4)) : 0u;
      const uint32_t hi0 = nl > 8 ? lower4(squad(st, k + nl - 8)) : 0u, hi1 = nl > 8 ? lower4(squad(st, k + nl - 4)) : 0u;
      f = field_of_words(R, T, st, k, nl, lo0, lo1, hi0, hi1);
    }
    span = (v - hs) << 16 | (e - v);
  }
  // the first pair of each field wins: per field, the lowest lane naming it
  P.present = P.vsum = 0;
  for (unsigned long long left = __ballot(has && f >= 0); left;) {  // uniform
    const uint32_t l = (uint32_t)__builtin_ctzll(left);
    const int fl = __shfl(f, (int)l, 64);
    const uint32_t sl = (uint32_t)__shfl((int)span, (int)l, 64);
    left &= ~__ballot(has && f == fl);
    if (lane == 0) sp0[(uint32_t)fl * stride] = sl;
    P.present |= 1u << fl;
    P.vsum += sl & 0xFFFFu;
  }
  wave_sync();  // request 0's spans for lane 0
  return true;
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
  return T.dflt[policy * 2 + (ingress ? 1 : 0)];
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
// [method table: 64 × 16 B][bucket counters: nkeys u32, when they fit
// (lds_keys)].
__device__ __forceinline__ lds_u8* wave_stage(lds_u32* lds, uint32_t F, uint32_t wave) {
  return (lds_u8*)(lds + F * kRawThreads) + wave * kStage;
}
__device__ __forceinline__ lds_u32* wave_masks(lds_u32* lds, uint32_t F, uint32_t wave) {
  return (lds_u32*)((lds_u8*)(lds + F * kRawThreads) + kRawWaves * kStage) + wave * 2 * kMaskWords;
}
__device__ __forceinline__ lds_u8* tchar_table(lds_u32* lds, uint32_t F) { return (lds_u8*)wave_masks(lds, F, kRawWaves); }
// the method table (kMethodTab) follows the 256-byte tchar table
constexpr uint32_t kTctBytes = 256 + kMethodSlots * 16;
__device__ __forceinline__ lds_u32* method_table(lds_u32* lds, uint32_t F) { return (lds_u32*)(tchar_table(lds, F) + 256); }
__device__ __forceinline__ void stage_methods(lds_u32* mt) {
  for (uint32_t j = threadIdx.x; j < kMethodSlots * 4; j += blockDim.x) mt[j] = kMethodTab.e[j >> 2][j & 3];
}
__device__ __forceinline__ lds_u32* key_counters(lds_u32* lds, uint32_t F) { return (lds_u32*)(tchar_table(lds, F) + kTctBytes); }
// [name keys: 8 u32 per slot][field slots: 4 u32 per slot][names, u32
// words][program hash keys][values] after the key counters, when they fit
// (lds_tables): the lookups every header line and request makes, at LDS
// latency instead of L1/L2
// [default programs: 2 u32 per policy] — every table a lane reads inside the
// loop: one global load there would make the wave wait for the next stage's
// loads too (vmcnt counts in issue order)
struct RawTableWords {
  uint32_t nk, fs, fn, ph, wb, df;
};
__host__ __device__ __forceinline__ RawTableWords raw_table_words(const HttpRawDev& R) {
  // (the FNV field slots are not staged: only the deferred requests' byte
  // path looks names up through them, from global memory)
  return {8 * (R.nkmask + 1), 0, (R.fnames_bytes + 3) / 4, R.phash_mask + 1, (R.nprogs + 31) / 32 + 1,
          2 * R.npolicies};
}
__host__ __device__ __forceinline__ uint32_t raw_tables_lds_words(const HttpRawDev& R) {
  const RawTableWords w = raw_table_words(R);
  return w.nk + w.fs + w.fn + 2 * w.ph + w.wb + w.df;
}
// The scan's lookup tables (RawTableWords order) copied into LDS at t, or
// their global copies (GlbTabs); the caller's barrier follows.
__device__ __forceinline__ void stage_tables(const HttpRawDev& R, lds_u32* t, LdsTabs& T) {
  const RawTableWords w = raw_table_words(R);
  lds_u32* tfs = t + w.nk;
  lds_u32* tfn = tfs + w.fs;
  lds_u32* tpk = tfn + w.fn;
  lds_u32* tpv = tpk + w.ph;
  lds_u32* twb = tpv + w.ph;
  lds_u32* tdf = twb + w.wb;
  for (uint32_t k = threadIdx.x; k < w.nk; k += blockDim.x) t[k] = R.nkeys[k];
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
  for (uint32_t k = threadIdx.x; k < w.df; k += blockDim.x) tdf[k] = R.dflt[k];
  T = LdsTabs{t, tfs, tpk, tpv, twb, tdf, (const lds_u8*)tfn};
}
__device__ __forceinline__ void stage_tables(const HttpRawDev& R, lds_u32*, GlbTabs& T) {
  T = GlbTabs{(glb_u32*)R.nkeys, (glb_u32*)R.fslots, (glb_u32*)R.phash_keys, (glb_u32*)R.phash_vals,
              (glb_u32*)R.walk_bits, (glb_u32*)R.dflt, (glb_u8*)R.fnames};
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

// 16 bytes of the stage from byte p (any alignment): five dword reads (one
// round trip) and four byte aligns.
__device__ __forceinline__ uint4 sread16(const lds_u8* st, uint32_t p) {
  const lds_u32* w = (const lds_u32*)(st + (p & ~3u));
  const uint32_t r = p & 3u, a = w[0], b = w[1], c = w[2], d = w[3], e = w[4];
  return make_uint4(__builtin_amdgcn_alignbyte(b, a, r), __builtin_amdgcn_alignbyte(c, b, r),
                    __builtin_amdgcn_alignbyte(d, c, r), __builtin_amdgcn_alignbyte(e, d, r));
}
// Unaligned stores (the byte address of a string position): the hardware
// runs in unaligned mode (amdhsa), and one lane's stores to overlapping bytes
// land in program order, so each store may leave bytes past its end that a
// later store of the same string overwrites.
typedef unsigned int u32x4_u __attribute__((ext_vector_type(4), aligned(1)));
typedef unsigned int u32_u __attribute__((aligned(1)));
__device__ __forceinline__ void st16u(uint8_t* p, uint4 v) { *(u32x4_u*)p = u32x4_u{v.x, v.y, v.z, v.w}; }
__device__ __forceinline__ void st4u(uint8_t* p, uint32_t v) { *(u32_u*)p = v; }
// The walked string of a request parsed from the stage (emit_string's
// output) stored at out: its present fields in order, each value copied 16
// bytes at a time and followed by its SEP, each run of absent fields below
// the last present one as 0x01 SEP pairs.  Stores reach up to 15 bytes past
// the string (the record stride leaves room: http_raw.cc cst); the build
// reads the string's length only.
__device__ __forceinline__ void emit_direct(const HttpRawDev& R, const lds_u8* st, uint32_t hs, const lds_u32* sp,
                                            uint32_t stride, const Parsed& P, uint32_t last, uint8_t* out) {
  uint32_t f = 0, pos = 0;
  for (uint32_t rem = P.present; rem; rem &= rem - 1) {
    const uint32_t g = (uint32_t)__builtin_ctz(rem);
    for (; f + 2 <= g; f += 2, pos += 4) st4u(out + pos, 0x00010001u);  // two absent fields
    if (f < g) {
      st4u(out + pos, 1u);
      pos += 2;
    }
    const uint32_t sv = sp[g * stride], a = hs + (sv >> 16), L = sv & 0xFFFFu;
    // whole 16-byte chunks of stage bytes (the bytes past L are overwritten:
    // first by the SEP below, then by what follows it), then the SEP
    for (uint32_t k = 0; k < L; k += 16) st16u(out + pos + k, sread16(st, a + k));
    out[pos + L] = 0;  // SEP
    pos += L + 1;
    f = g + 1;
  }
  if (last < R.nfields) st4u(out + pos, 2u);  // REST
}

// A request's record in the string buffer (16-byte aligned, request order):
// a 16-byte header {request index, remote identity, string length | flags
// << 24, program} and the uncoded walked string.  A head of h bytes yields at
// most h + 2F bytes of string (each absent field costs 2 bytes the head does
// not hold; the request line and the blank line hold 13 bytes no string
// does; a list at most its own bytes + 2F + 1), so with a stride of cst >=
// 2F + 48 bytes per request the records never overlap, the 15 bytes the
// scan's last unaligned store may write past a string included; 128 more let
// the scan move a record to the next 128-B line start (see the scan).
__device__ __forceinline__ uint64_t rec_off(uint64_t head_rel, size_t i, uint32_t cst) {
  return ((head_rel + 15) & ~15ull) + (uint64_t)cst * i;
}

// ---- pass 1: parse, program, string length, bucket key, the request's
// record in the string buffer; per-block bucket counts (bcount[key * gridDim.x + block],
// lds_keys) or a global histogram.  kLists: header lists, not heads.
// Requests inside the wave's stage parse over its structural bitmaps;
// the others are deferred to raw_defer_kernel.
// A lane's request inputs, loaded two iterations ahead of their use.
struct RawIn {
  uint32_t pol, rem, ip;  // policy, remote identity, ingress | port << 8
  uint32_t len;           // head bytes (off[i + 1] - off[i], clamped)
  uint64_t a;             // off[i]
  __device__ __forceinline__ uint32_t ing() const { return ip & 0xFFu; }
  __device__ __forceinline__ uint32_t port() const { return ip >> 8; }
};
__device__ __forceinline__ RawIn raw_in(const uint64_t* __restrict__ off, const uint32_t* __restrict__ policy,
                                        const uint8_t* __restrict__ ingress, const uint16_t* __restrict__ port,
                                        const uint32_t* __restrict__ remote, size_t i, size_t n) {
  // unconditional loads, selects after them: a load skipped on some path
  // makes the compiler's wait for any older load a wait for every load
  // (vmcnt(0)), the next stage's included
  const size_t j = i < n ? i : (n ? n - 1 : 0);
  RawIn r;
  const uint32_t pol = policy[j];
  r.pol = i < n ? pol : 0xFFFFFFFFu;
  r.ip = (uint32_t)ingress[j] | (uint32_t)port[j] << 8;
  r.rem = remote[j];
  const uint64_t a = off[j], b = off[j + 1];
  r.a = i < n ? a : b;  // past n: empty at off[n]
  r.len = i < n && b > a ? (uint32_t)min<uint64_t>(b - a, 0xFFFFFFFFull) : 0u;
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
__device__ __forceinline__ void stage_load(glb_u8* raw, const RawIn& in, uint32_t lane, StageRegs& S,
                                           const uint64_t* safe) {
  const uint64_t lo = __shfl(in.a, 0, 64);
  // the last lane's end (empty lanes past n sit at off[n])
  const uint64_t hi = __shfl(in.a + in.len, 63, 64);
  const uint64_t glo = (uint64_t)(uintptr_t)(raw + lo), ghi = (uint64_t)(uintptr_t)(raw + hi);
  const uint64_t a0 = glo & ~15ull;
  const uint32_t nb = hi > lo ? (uint32_t)min<uint64_t>((ghi - a0 + 15) & ~15ull, kStage) : 0u;
  S.base = a0;
  S.len = nb;
  // every load issued (no branch around one, no select after one: either
  // makes the compiler wait for it here): past the stage a harmless repeat of
  // the first block; a wave without head bytes reads a block of off[] instead
  // (readable; nothing of an empty stage is parsed)
  const uint64_t src0 = nb ? a0 : ((uint64_t)(uintptr_t)safe & ~15ull);
#pragma unroll
  for (uint32_t j = 0; j < kStageVecs; ++j) {
    const uint32_t o = (j * 64 + lane) * 16;
    const uint64_t a = o < nb ? a0 + o : src0;
    S.v[j] = to_uint4(*(glb_v4*)(uintptr_t)a);
  }
}
__device__ __forceinline__ void stage_store(const StageRegs& S, lds_u8* stage, uint32_t lane) {
#pragma unroll
  for (uint32_t j = 0; j < kStageVecs; ++j) *(lds_v4*)(stage + (j * 64 + lane) * 16) = to_v4(S.v[j]);
}

// Bucket key of a request: walked string units (0..8) or the overflow key.
__device__ __forceinline__ uint32_t bucket_key(uint32_t len) {
  return len > CG_HTTP_SLOT_BYTES ? kRawKeys - 1 : (len + 15) / 16;
}

template <bool kLists, bool kLdsTabs>
__global__ __launch_bounds__(kRawThreads) void raw_scan_kernel(HttpRawDev R, const uint8_t* __restrict__ raw_g,
                                                               const uint64_t* __restrict__ off, size_t n,
                                                               const uint32_t* __restrict__ policy,
                                                               const uint8_t* __restrict__ ingress,
                                                               const uint16_t* __restrict__ port,
                                                               uint32_t* __restrict__ counts, uint2* __restrict__ rinfo,
                                                               const uint32_t* __restrict__ remote,
                                                               uint8_t* __restrict__ sbuf, uint32_t cst,
                                                               unsigned long long* __restrict__ ovf_bytes,
                                                               uint32_t lds_keys, uint32_t* __restrict__ dlist,
                                                               uint32_t* __restrict__ dcount) {
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
  const lds_u32* mtab = method_table(lds, F);
  if (!kLists) stage_methods(method_table(lds, F));
  // the lookup tables: LDS copies when they fit (kLdsTabs), else HBM
  using Tabs = typename std::conditional<kLdsTabs, LdsTabs, GlbTabs>::type;
  Tabs T;
  stage_tables(R, lk + (lds_keys ? (nk + 3u) & ~3u : 0u), T);  // 16-byte aligned (field_of_words' key slots)
  const uint64_t off0 = off[0];
  __syncthreads();
  // software pipeline per wave: iteration k parses stage k from LDS while the
  // stage of k + 1 is in flight into registers and the inputs of k + 2 load
  const size_t gstride = (size_t)gridDim.x * kRawThreads;
  size_t base = (size_t)blockIdx.x * kRawThreads;
  // (a wave with no requests skips the loop and meets the others at the flush)
  RawIn cur = raw_in(off, policy, ingress, port, remote, base + wave * 64 + lane, n);
  RawIn nxt = raw_in(off, policy, ingress, port, remote, base + gstride + wave * 64 + lane, n);
  StageRegs S;
  stage_load(raw, cur, lane, S, off);
#ifdef CG_RAW_CLOCKS
  uint64_t clk[8] = {0, 0, 0, 0, 0, 0, 0, 0}, c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0;
#endif
  for (; base < n; base += gstride) {
    const size_t i0 = base + (size_t)wave * 64;
    if (i0 >= n) break;  // wave-uniform
    RAW_CLK(c0);
    const size_t i = i0 + lane;
    const bool live = i < n;
    const RawIn nn = raw_in(off, policy, ingress, port, remote, base + 2 * gstride + wave * 64 + lane, n);
    // the program (LDS tables): done while the stage's loads and the previous
    // iteration's record stores drain (the stage store below waits for both)
    const uint32_t prog = live ? lookup_prog(R, T, cur.pol, cur.ing() != 0, cur.port()) : kProgDeny;
    // stage k: registers → LDS (the previous iteration's reads are done)
    wave_sync();
    stage_store(S, stage, lane);
    const uint64_t sbase = S.base;
    const uint32_t slen = S.len;
    // stage k + 1 into registers, under this iteration's parse
    stage_load(raw, nxt, lane, S, off);  // (past n: no bytes, nothing staged)
    wave_sync();
    RAW_CLK(c1);
    if (kLists) build_masks_lists(stage, slen, tct, masks, lane);
    else build_masks(stage, slen, tct, masks, lane);
    wave_sync();
    RAW_CLK(c2);
#ifdef CG_RAW_CLOCKS
    c3 = c4 = c2;
#endif
    // every request but an unknown policy's is parsed: a head the codec
    // rejects is denied in any program (flagged malformed)
    const uint32_t hn = cur.len;
    const uint64_t ga = (uint64_t)(uintptr_t)(raw + cur.a);
    const bool in = ga >= sbase && ga + hn <= sbase + slen;
    // a request outside the stage goes to raw_defer_kernel (one append per wave)
    const bool defer = live && prog != kProgDeny && !in;
    const unsigned long long dm = __ballot(defer);
    if (dm) {
      uint32_t dbase = 0;
      if (lane == (uint32_t)__builtin_ctzll(dm)) dbase = atomicAdd(dcount, (uint32_t)__popcll(dm));
      dbase = (uint32_t)__shfl((int)dbase, (int)__builtin_ctzll(dm), 64);
      if (defer) dlist[dbase + (uint32_t)__popcll(dm & ((1ull << lane) - 1))] = (uint32_t)i;
    }
    if (live && !defer) {
      uint32_t key = 0, len = 0, bad = 0;
      uint64_t rpos = rec_off(cur.a - off0, i, cst);  // the record's byte offset (16-B aligned)
      uint4* rec = reinterpret_cast<uint4*>(sbuf + rpos);
      if (prog != kProgDeny) {
        const uint32_t hs = (uint32_t)(ga - sbase);
        Parsed P;
        const bool ok = kLists ? (R.raw_values ? parse_list_fast(R, T, stage, masks, masks + kMaskWords, hs, hs + hn, sp, kRawThreads, P)
                                             : parse_list_win(R, T, stage, masks, masks + kMaskWords, hs, hs + hn, sp, kRawThreads, P))
                               : parse_head_fast(R, T, stage, masks, masks + kMaskWords, mtab, hs, hs + hn, sp, kRawThreads, P);
        RAW_CLK(c3);
        if (!ok) {
          bad = 1;
        } else if (walked_t(R, T, prog)) {
          uint32_t last;
          len = walked_len(R, P, &last);
          key = bucket_key(len);
          // a record the build reads (header + len rounded to 16) that would
          // straddle a 64-B sector (records up to 64 B) or a 128-B line
          // (up to 128 B) moves to the next one's start: the build gathers
          // one sector / line per record instead of two
          const uint32_t ext = 16 + ((len + 15) & ~15u), g = ext <= 64 ? 64u : 128u;
          if ((rpos & (g - 1)) + ext > g && ext <= 128) {
            rpos = (rpos + g - 1) & ~(uint64_t)(g - 1);
            rec = reinterpret_cast<uint4*>(sbuf + rpos);
          }
          emit_direct(R, stage, hs, sp, kRawThreads, P, last, reinterpret_cast<uint8_t*>(rec + 1));
          if (len > CG_HTTP_SLOT_BYTES) atomicAdd(ovf_bytes, (unsigned long long)((4 + len + 15) & ~15u));
          RAW_CLK(c4);
        }
      }
      const uint32_t flags = (cur.ing() ? CG_HTTP_F_INGRESS : 0u) | (bad ? CG_HTTP_F_MALFORMED : 0u) |
                             (len > CG_HTTP_SLOT_BYTES ? CG_HTTP_F_OVERFLOW : 0u);
      *rec = make_uint4((uint32_t)i, cur.rem, len | flags << 24, prog);
      const uint32_t k = group_of(R, prog) * kRawKeys + key;
      // for the rank: the bucket and the record (16-B units)
      rinfo[i] = make_uint2(k, (uint32_t)(rpos / 16));
      if (lds_keys) __hip_atomic_fetch_add(&lk[k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else atomicAdd(&counts[k], 1u);
    }
    cur = nxt;
    nxt = nn;
    RAW_CLK(c5);
    RAW_ACC(0, c0, c1);  // stage store (waits for the stage's loads)
    RAW_ACC(1, c1, c2);  // structural masks
    RAW_ACC(2, c2, c3);  // program lookup + parse
    RAW_ACC(3, c3, c4);  // string length + emission
    RAW_ACC(4, c4, c5);  // record header, rinfo, counters
    RAW_ACC(5, c0, c5);
#ifdef CG_RAW_CLOCKS
    clk[6] += 1;
#endif
  }
#ifdef CG_RAW_CLOCKS
  if (blockIdx.x == 7 && threadIdx.x == 64) {
    printf("raw_scan clocks (wave 1 of block 7, %llu iterations): stage %llu masks %llu parse %llu emit %llu tail %llu total %llu\n",
           (unsigned long long)clk[6], (unsigned long long)clk[0], (unsigned long long)clk[1], (unsigned long long)clk[2],
           (unsigned long long)clk[3], (unsigned long long)clk[4], (unsigned long long)clk[5]);
    printf("parse clocks: request line %llu, line reads %llu, values %llu, names %llu, end %llu\n", g_pclk[0], g_pclk[1],
           g_pclk[2], g_pclk[3], g_pclk[4]);
  }
#endif
  if (lds_keys) {
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nk; k += blockDim.x) counts[(size_t)k * gridDim.x + blockIdx.x] = lk[k];
  }
}

// ---- pass 1b: the requests the scan deferred (heads / lists not inside
// their wave's stage: long ones), one lane each, read byte by byte from HBM
// through HeadReader with the tables in global memory.  Their bucket counts
// go to the scan block that met them (nblk: the scan's grid), after it.
template <bool kLists>
__global__ __launch_bounds__(kRawThreads) void raw_defer_kernel(HttpRawDev R, const uint8_t* __restrict__ raw,
                                                                const uint64_t* __restrict__ off,
                                                                const uint32_t* __restrict__ policy,
                                                                const uint8_t* __restrict__ ingress,
                                                                const uint16_t* __restrict__ port,
                                                                uint32_t* __restrict__ counts, uint32_t nblk,
                                                                uint32_t lds_keys, uint2* __restrict__ rinfo,
                                                                const uint32_t* __restrict__ remote,
                                                                uint8_t* __restrict__ sbuf, uint32_t cst,
                                                                unsigned long long* __restrict__ ovf_bytes,
                                                                const uint32_t* __restrict__ dlist,
                                                                const uint32_t* __restrict__ dcount) {
  extern __shared__ uint32_t lds_[];
  lds_u32* sp = (lds_u32*)lds_ + threadIdx.x;
  const GlbTabs T{(glb_u32*)R.nkeys, (glb_u32*)R.fslots, (glb_u32*)R.phash_keys, (glb_u32*)R.phash_vals,
                  (glb_u32*)R.walk_bits, (glb_u32*)R.dflt, (glb_u8*)R.fnames};
  const uint32_t nd = *dcount;
  const uint64_t off0 = off[0];
  for (uint32_t j = blockIdx.x * kRawThreads + threadIdx.x; j < nd; j += gridDim.x * kRawThreads) {
    const size_t i = dlist[j];
    const uint64_t a = off[i], b = off[i + 1];
    const uint32_t hn = b > a ? (uint32_t)min<uint64_t>(b - a, 0xFFFFFFFFull) : 0u;
    const uint32_t prog = lookup_prog(R, T, policy[i], ingress[i] != 0, port[i]);
    HeadReader hr((glb_u8*)raw + a, hn, (const lds_u8*)0, false);
    uint32_t key = 0, len = 0, bad = 0;
    uint4* rec = reinterpret_cast<uint4*>(sbuf + rec_off(a - off0, i, cst));
    bool ok;
    if (kLists) {
      if (hn > kFieldsMaxList) {  // spans would not fit: the call fails
        atomicOr(ovf_bytes, kRawListTooLong);
        ok = false;
      } else {
        ok = parse_list_bytes(R, T, hr, sp, kRawThreads);
      }
    } else {
      ok = parse_head(R, T, hr, sp, kRawThreads);
    }
    if (!ok) {
      bad = 1;
    } else if (walked(R, prog)) {
      uint32_t last;
      len = string_len(R, sp, kRawThreads, &last);
      key = bucket_key(len);
      Out16 o(rec + 1, 1);
      emit_string(R, hr, sp, kRawThreads, last, o);
      if (o.pos) o.flush();
      if (len > CG_HTTP_SLOT_BYTES) atomicAdd(ovf_bytes, (unsigned long long)((4 + len + 15) & ~15u));
    }
    const uint32_t flags = (ingress[i] ? CG_HTTP_F_INGRESS : 0u) | (bad ? CG_HTTP_F_MALFORMED : 0u) |
                           (len > CG_HTTP_SLOT_BYTES ? CG_HTTP_F_OVERFLOW : 0u);
    *rec = make_uint4((uint32_t)i, remote[i], len | flags << 24, prog);
    const uint32_t k = group_of(R, prog) * kRawKeys + key;
    rinfo[i] = make_uint2(k, (uint32_t)(rec_off(a - off0, i, cst) / 16));
    // the scan's block of request i (grid-stride order, kRawThreads per block)
    if (lds_keys) atomicAdd(&counts[(size_t)k * nblk + (i / kRawThreads) % nblk], 1u);
    else atomicAdd(&counts[k], 1u);
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
// the same grid and request order as the scan), else a global cursor per
// key: order[slot] = the request's record.  rinfo[i] = {bucket, record in
// 16-B units} from the scan; kRankU requests per thread in flight.
constexpr uint32_t kRankU = 8;
__global__ __launch_bounds__(kRawThreads) void raw_rank_kernel(HttpRawDev R, size_t n,
                                                               const uint2* __restrict__ rinfo,
                                                               uint32_t* __restrict__ cursor,
                                                               const uint32_t* __restrict__ bbase, uint32_t lds_keys,
                                                               uint32_t* __restrict__ order) {
  extern __shared__ uint32_t lk[];  // the bucket cursors (lds_keys)
  const uint32_t nk = (R.nprogs + 2) * kRawKeys;
  if (lds_keys)
    for (uint32_t k = threadIdx.x; k < nk; k += blockDim.x) lk[k] = cursor[k] + bbase[(size_t)k * gridDim.x + blockIdx.x];
  __syncthreads();
  const size_t gs = (size_t)gridDim.x * kRawThreads;
  for (size_t base = (size_t)blockIdx.x * kRawThreads; base < n; base += kRankU * gs) {
    uint2 ri[kRankU];
#pragma unroll
    for (uint32_t u = 0; u < kRankU; ++u) {
      const size_t i = base + u * gs + threadIdx.x;
      ri[u] = rinfo[i < n ? i : n - 1];
    }
#pragma unroll
    for (uint32_t u = 0; u < kRankU; ++u) {
      if (base + u * gs + threadIdx.x >= n) continue;
      const uint32_t slot = lds_keys ? atomicAdd(&lk[ri[u].x], 1u) : atomicAdd(&cursor[ri[u].x], 1u);
      order[slot] = ri[u].y;
    }
  }
}

// Nontemporal 16-byte load / store (streaming data read or written once)
__device__ __forceinline__ uint4 ld_nt16(const uint4* p) {
  return to_uint4(__builtin_nontemporal_load(reinterpret_cast<const v4u32*>(p)));
}
__device__ __forceinline__ void st_nt16(uint4* p, uint4 v) {
  __builtin_nontemporal_store(to_v4(v), reinterpret_cast<v4u32*>(p));
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
  uint32_t rn = order[(size_t)t * 64 + lane];  // the next tile's slot records, one tile ahead
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
    const uint32_t r = rn;  // the slot's record (16-B units), or padding
    rn = order[(size_t)min(t + 1, tend - 1) * 64 + lane];
    const uint32_t L = units == 0 ? 1u : (units < 2 ? 2u : units < 4 ? 4u : units < 8 ? 8u : 16u);
    const uint32_t per = 64 / L, sub = lane & (L - 1), grp = lane & ~(L - 1);
    uint32_t m = 0;  // the longest slot string among this lane's header slots
    // slots at or past the group's end are padding (their order entries are
    // not initialised: written below)
    const uint32_t nreal = run.send > t * 64 ? min(run.send - t * 64, 64u) : 0u;
    // one pass: slot s = pass * per + lane / L; x = its chunk (raw load, ok =
    // a real slot and a chunk of the record)
    auto body = [&](uint32_t pass, uint32_t rs, bool ok, uint4 xr) {
      const uint32_t s = pass * per + lane / L;
      const bool pad = s >= nreal;
      const uint4 x = ok ? xr : make_uint4(0, 0, CG_HTTP_F_PAD << 24, 0);
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
        order[(size_t)t * 64 + s] = pad ? 0xFFFFFFFFu : x.x;
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
    };
    auto fetch = [&](uint32_t pass, uint32_t& rs, bool& ok, uint4& x) {
      const uint32_t s = pass * per + lane / L;
      rs = (uint32_t)__shfl((int)r, (int)s, 64);
      ok = s < nreal && sub <= units;
      x = rec16[ok ? (size_t)rs + sub : 0];  // unconditional: others read chunk 0
    };
    // two passes' chunks in flight: A holds pass p, B pass p + 1; each is
    // refilled (p + 2, p + 3) right after it is consumed
    uint32_t rsA = 0, rsB = 0;
    bool okA = false, okB = false;
    uint4 xA = make_uint4(0, 0, 0, 0), xB = xA;
    fetch(0, rsA, okA, xA);
    if (L > 1) fetch(1, rsB, okB, xB);
    for (uint32_t pass = 0; pass < L; pass += 2) {
      body(pass, rsA, okA, xA);
      if (pass + 2 < L) fetch(pass + 2, rsA, okA, xA);
      if (pass + 1 < L) {
        body(pass + 1, rsB, okB, xB);
        if (pass + 3 < L) fetch(pass + 3, rsB, okB, xB);
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

// ---- the device-layout path (CILIUM_GPU_RAW_LAYOUT=device, http_raw.cc) --
// The steps of the path above without its host round trips:
//   raw_scan_dl_kernel   parse as raw_scan_kernel, then the request takes a
//                        slot of its bucket (program group x string units)
//                        from a per-bucket counter and writes its class-coded
//                        string units, meta word and order entry straight
//                        into the tile-transposed batch http_kernel reads
//   raw_defer_dl_kernel  the same for requests outside their wave's stage
//   raw_seal_kernel      last tiles padded, chunk table grouped by program,
//                        batch header — the layout the host computes above
//   http_kernel          the verdicts, in request order through order[]
//   raw_walk_kernel      requests whose string passes the 128-byte slot:
//                        walked one lane each over the tables in HBM
// Dynamic LDS of raw_scan_dl_kernel: raw_scan_kernel's without the bucket
// counters (the lookup tables follow the tchar table).
__device__ __forceinline__ lds_u32* raw_tables(lds_u32* lds, uint32_t F) { return (lds_u32*)(tchar_table(lds, F) + kTctBytes); }

// ---- the walked string, class-coded, straight into its tile slot ---------
// http_pack.cc's string: the values of the fields up to the last present
// one, each SEP-terminated (an absent one: 0x01 SEP), then REST (0x02) when a
// later field is absent; every byte through the program's code map (identity
// for byte-mode programs).  Bytes gather in 16; each full unit is coded and
// stored to the slot's next string unit (1 KiB apart in the tile); in the
// last unit the bytes past the string stay zero (the walk's padding).

// The string of a request parsed from the stage (parse_head_fast /
// parse_list_fast spans, relative to hs) into o.
template <class Out>
__device__ __forceinline__ void emit_stage(const HttpRawDev& R, const lds_u8* st, uint32_t hs, const lds_u32* sp,
                                           uint32_t stride, const Parsed& P, uint32_t last, Out& o) {
  uint32_t f = 0;
  for (uint32_t rem = P.present; rem; rem &= rem - 1) {
    const uint32_t g = (uint32_t)__builtin_ctz(rem);
    for (; f + 2 <= g; f += 2) o.put4(0x00010001u, 4);  // two absent fields
    if (f < g) o.put4(1u, 2);
    const uint32_t sv = sp[g * stride], a = hs + (sv >> 16), L = sv & 0xFFFFu;
    for (uint32_t k = 0; k < L; k += 4) {  // a quad at a time
      const uint32_t nb = min(L - k, 4u);
      o.put4(keep_bytes(squad(st, a + k), nb), nb);
    }
    o.put(0u);  // SEP
    f = g + 1;
  }
  if (last < R.nfields) o.put(2u);  // REST
  o.finish();
}

// The string of a request parsed through a HeadReader (parse_head /
// parse_list_bytes spans, absolute, kAbsentSpan for absent fields) into o.
template <class Out>
__device__ __forceinline__ void emit_reader(const HttpRawDev& R, HeadReader& hr, const lds_u32* sp, uint32_t stride,
                                            uint32_t last, Out& o) {
  for (uint32_t f = 0; f < last; ++f) {
    const uint32_t s = sp[f * stride];
    if (s == kAbsentSpan) {
      o.put4(1u, 2);  // absent, SEP
      continue;
    }
    const uint32_t a = s >> 16, L = s & 0xFFFFu;
    for (uint32_t k = 0; k < L; k += 4) {
      const uint32_t nb = min(L - k, 4u);
      o.put4(keep_bytes(hr.quad(a + k), nb), nb);
    }
    o.put(0u);
  }
  if (last < R.nfields) o.put(2u);
  o.finish();
}

// ---- slots: the batch laid out on the device (dev_types.h RawLayoutDev) ---
// Every lane with `want` takes the next slot of its bucket key; the first
// slot of a chunk takes a chunk id and publishes it (never waiting first), the
// others wait for their chunk's id.  ok = false: the layout's bounds were
// passed or the chunk's id was not seen within L.spin polls (neither happens
// for the sizes http_raw.cc reserves; ctl[kRawCtlError] records it) — the
// lane's request is walked by raw_walk_kernel instead, and a slot it had
// taken in a chunk goes on the late list for raw_seal_kernel to pad.
struct RawSlot {
  uint8_t* tb;  // the tile's data
  uint32_t t, l;
  bool ok;
};
__device__ __forceinline__ RawSlot raw_slot(const RawLayoutDev& L, bool want, uint32_t key, uint32_t prog) {
  RawSlot r{nullptr, 0, 0, false};
  uint32_t s = 0;
  if (want) s = atomicAdd(&L.kcnt[(size_t)key * kRawCntStride], 1u);
  const uint32_t c = s >> L.cshift;
  if (want && (s & ((1u << L.cshift) - 1u)) == 0 && c < L.dpk) {  // publish the chunk
    const uint32_t id = atomicAdd(&L.ctl[kRawCtlChunks], 1u);
    const bool fits = id < L.maxchunks;
    if (fits) L.chunks[id] = HttpChunk{prog, id * L.ext, L.ext, key};
    else atomicOr(&L.ctl[kRawCtlError], 1u);
    __hip_atomic_store(&L.dir[(size_t)key * L.dpk + c], (unsigned long long)L.seq << 32 | (fits ? id : 0xFFFFFFFFu),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!want) return r;
  if (c >= L.dpk) {
    atomicOr(&L.ctl[kRawCtlError], 1u);
    return r;
  }
  const unsigned long long* e = &L.dir[(size_t)key * L.dpk + c];
  unsigned long long v = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t it = 0; (uint32_t)(v >> 32) != L.seq && it < L.spin; ++it) {
    __builtin_amdgcn_s_sleep(2);
    v = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const uint32_t id = (uint32_t)v;
  if ((uint32_t)(v >> 32) != L.seq) {  // not seen in time: the seal pads the slot
    atomicOr(&L.ctl[kRawCtlError], 2u);
    const uint32_t j = atomicAdd(&L.ctl[kRawCtlLate], 1u);
    L.late[j] = (unsigned long long)key << 32 | s;  // (one per slot taken: j < slots <= capacity)
    return r;
  }
  if (id == 0xFFFFFFFFu) return r;  // a chunk past maxchunks (bit 0 set): not in the chunk table
  r.t = id * L.ext + ((s >> 6) & (L.ext - 1u));
  r.l = s & 63u;
  r.tb = L.tiles + (size_t)r.t * (kRawTileGran * 512);
  r.ok = true;
  return r;
}

// One lane's request into its slot: meta word, order entry, the tile's data
// offset (slot 0) and, for walked strings, the units (emit) and the tile's
// tail (atomicMax on units | tail << 16, zeroed per sub-batch).
template <class Emit>
__device__ __forceinline__ void raw_fill(const RawLayoutDev& L, const RawSlot& sl, uint32_t i, uint32_t rem,
                                         uint32_t flags, uint32_t units, uint32_t len, Emit emit) {
  reinterpret_cast<uint2*>(sl.tb)[sl.l] = make_uint2(rem, flags << 24);
  L.order[(size_t)sl.t * 64 + sl.l] = i;
  if (sl.l == 0) L.ttab[sl.t].at = sl.t * kRawTileGran;
  if (units) {
    emit(reinterpret_cast<uint4*>(sl.tb + 512) + sl.l);
    atomicMax(&L.ttab[sl.t].units, units | (len - 16u * (units - 1u)) << 16);
  }
}

// Append the lanes with `take` to a request list (count at *cnt): one atomic
// per wave.
__device__ __forceinline__ void list_append(uint32_t* list, uint32_t* cnt, bool take, uint32_t i, uint32_t lane) {
  const unsigned long long m = __ballot(take);
  if (!m) return;
  const int first = __builtin_ctzll(m);
  uint32_t base = 0;
  if ((int)lane == first) base = atomicAdd(cnt, (uint32_t)__popcll(m));
  base = (uint32_t)__shfl((int)base, first, 64);
  if (take) list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = i;
}
// ---- the scan: parse, program, string, slot and tile ---------------------
// One lane per request, a wave's 64 heads (lists) staged in LDS: parse over
// the structural bitmaps, look the program up, and put the request straight
// into its slot of the device-built batch — class-coded string units, meta
// word, order entry.  A request whose walked string passes the slot
// (CG_HTTP_SLOT_BYTES) goes on the walk list; one outside its wave's stage on
// the deferred list (raw_defer_kernel).  kLists: header lists, not heads.
template <bool kLists, bool kLdsTabs>
__global__ __launch_bounds__(kRawThreads) void raw_scan_dl_kernel(HttpRawDev R, const uint8_t* __restrict__ raw_g,
                                                               const uint64_t* __restrict__ off, size_t n,
                                                               const uint32_t* __restrict__ policy,
                                                               const uint8_t* __restrict__ ingress,
                                                               const uint16_t* __restrict__ port,
                                                               const uint32_t* __restrict__ remote, RawLayoutDev L) {
  extern __shared__ uint32_t lds_[];
  lds_u32* lds = (lds_u32*)lds_;
  glb_u8* raw = (glb_u8*)raw_g;
  const uint32_t F = max(R.nfields, 1u), wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  lds_u32* sp = lds + threadIdx.x;  // this lane's spans: sp[f * kRawThreads]
  lds_u8* stage = wave_stage(lds, F, wave);
  lds_u32* masks = wave_masks(lds, F, wave);
  lds_u8* tct = tchar_table(lds, F);
  for (uint32_t b = threadIdx.x; b < 256; b += blockDim.x) tct[b] = kLists ? list_stop(b, R.raw_values) : !tchar(b);
  const lds_u32* mtab = method_table(lds, F);
  if (!kLists) stage_methods(method_table(lds, F));
  // the lookup tables: LDS copies when they fit (kLdsTabs), else HBM
  using Tabs = typename std::conditional<kLdsTabs, LdsTabs, GlbTabs>::type;
  Tabs T;
  stage_tables(R, raw_tables(lds, F), T);
  __syncthreads();
  // software pipeline per wave: iteration k parses stage k from LDS while the
  // stage of k + 1 is in flight into registers and the inputs of k + 2 load
  const size_t gstride = (size_t)gridDim.x * kRawThreads;
  size_t base = (size_t)blockIdx.x * kRawThreads;
  RawIn cur = raw_in(off, policy, ingress, port, remote, base + wave * 64 + lane, n);
  RawIn nxt = raw_in(off, policy, ingress, port, remote, base + gstride + wave * 64 + lane, n);
  StageRegs S;
  stage_load(raw, cur, lane, S, off);
  uint64_t clk[8] = {0, 0, 0, 0, 0, 0, 0, 0}, c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0;
  for (; base < n; base += gstride) {
    const size_t i0 = base + (size_t)wave * 64;
    if (i0 >= n) break;  // wave-uniform
    const size_t i = i0 + lane;
    const bool live = i < n;
    RAW_CLK(c0);
    const RawIn nn = raw_in(off, policy, ingress, port, remote, base + 2 * gstride + wave * 64 + lane, n);
    const uint32_t prog = live ? lookup_prog(R, T, cur.pol, cur.ing() != 0, cur.port()) : kProgDeny;
    // stage k: registers → LDS (the previous iteration's reads are done)
    wave_sync();
    stage_store(S, stage, lane);
    const uint64_t sbase = S.base;
    const uint32_t slen = S.len;
    // stage k + 1 into registers, under this iteration's parse
    stage_load(raw, nxt, lane, S, off);  // (past n: no bytes, nothing staged)
    wave_sync();
    RAW_CLK(c1);
    if (kLists) build_masks_lists(stage, slen, tct, masks, lane);
    else build_masks(stage, slen, tct, masks, lane);
    wave_sync();
    RAW_CLK(c2);
    // every request but an unknown policy's is parsed: a head the codec
    // rejects is denied in any program (flagged malformed)
    const uint32_t hn = cur.len;
    const uint64_t ga = (uint64_t)(uintptr_t)(raw + cur.a);
    const bool in = ga >= sbase && ga + hn <= sbase + slen;
    const bool defer = live && prog != kProgDeny && !in;
    list_append(L.dlist, &L.ctl[kRawCtlDefer], defer, (uint32_t)i, lane);
    const uint32_t hs = (uint32_t)(ga - sbase);
    uint32_t flags = cur.ing() ? CG_HTTP_F_INGRESS : 0u, units = 0, len = 0, last = 0;
    bool walk = false;
    Parsed P;
    P.present = P.vsum = 0;
    if (live && !defer && prog != kProgDeny) {
      const bool ok = kLists ? (R.raw_values ? parse_list_fast(R, T, stage, masks, masks + kMaskWords, hs, hs + hn, sp, kRawThreads, P)
                                             : parse_list_win(R, T, stage, masks, masks + kMaskWords, hs, hs + hn, sp, kRawThreads, P))
                             : parse_head_fast(R, T, stage, masks, masks + kMaskWords, mtab, hs, hs + hn, sp, kRawThreads, P);
      if (!ok) {
        flags |= CG_HTTP_F_MALFORMED;
      } else if (walked_t(R, T, prog)) {
        len = walked_len(R, P, &last);
        if (len > CG_HTTP_SLOT_BYTES) walk = true;
        else units = (len + 15) / 16;
      }
    }
    RAW_CLK(c3);
    const bool want = live && !defer && !walk;
    const RawSlot sl = raw_slot(L, want, raw_vkey(L, group_of(R, prog) * kRawUnits + units, blockIdx.x), prog);
    RAW_CLK(c4);
    walk |= want && !sl.ok;
    list_append(L.walk, &L.ctl[kRawCtlWalk], walk, (uint32_t)i, lane);
    if (want && sl.ok) {
      raw_fill(L, sl, (uint32_t)i, cur.rem, flags, units, len, [&](uint4* dst) {
        TileOut<false> o(dst, nullptr);  // raw bytes: http_kernel codes them
        emit_stage(R, stage, hs, sp, kRawThreads, P, last, o);
      });
    }
    RAW_CLK(c5);
    RAW_ACC(0, c0, c1);  // program lookup, stage store (waits for the stage's loads)
    RAW_ACC(1, c1, c2);  // structural masks
    RAW_ACC(2, c2, c3);  // parse, walked length
    RAW_ACC(3, c3, c4);  // slot (atomic, directory)
    RAW_ACC(4, c4, c5);  // lists, emission
    RAW_ACC(5, c0, c5);
#ifdef CG_RAW_CLOCKS
    clk[6] += 1;
#endif
    (void)c6;
    cur = nxt;
    nxt = nn;
  }
#ifdef CG_RAW_CLOCKS
  if (blockIdx.x == 7 && threadIdx.x == 64) {
    printf("raw_scan_dl clocks (wave 1 of block 7, %llu iterations): stage %llu masks %llu parse %llu slot %llu emit %llu total %llu\n",
           (unsigned long long)clk[6], (unsigned long long)clk[0], (unsigned long long)clk[1], (unsigned long long)clk[2],
           (unsigned long long)clk[3], (unsigned long long)clk[4], (unsigned long long)clk[5]);
    printf("parse clocks: request line %llu, line reads %llu, values %llu, names %llu, end %llu\n", g_pclk[0], g_pclk[1],
           g_pclk[2], g_pclk[3], g_pclk[4]);
  }
#else
  (void)clk;
#endif
}

// ---- the deferred requests (heads / lists not inside their wave's stage:
// long ones), one lane each, read from HBM through HeadReader with the tables
// in global memory, into their slots as the scan does.
template <bool kLists>
__global__ __launch_bounds__(kRawThreads) void raw_defer_dl_kernel(HttpRawDev R, const uint8_t* __restrict__ raw,
                                                                const uint64_t* __restrict__ off,
                                                                const uint32_t* __restrict__ policy,
                                                                const uint8_t* __restrict__ ingress,
                                                                const uint16_t* __restrict__ port,
                                                                const uint32_t* __restrict__ remote, RawLayoutDev L) {
  extern __shared__ uint32_t lds_[];
  lds_u32* sp = (lds_u32*)lds_ + threadIdx.x;
  const GlbTabs T{(glb_u32*)R.nkeys, (glb_u32*)R.fslots, (glb_u32*)R.phash_keys, (glb_u32*)R.phash_vals,
                  (glb_u32*)R.walk_bits, (glb_u32*)R.dflt, (glb_u8*)R.fnames};
  const uint32_t nd = L.ctl[kRawCtlDefer], lane = threadIdx.x & 63;
  const uint32_t gs = gridDim.x * kRawThreads;
  for (uint32_t base = blockIdx.x * kRawThreads; base < nd; base += gs) {  // uniform per workgroup
    const uint32_t j = base + threadIdx.x;
    const bool live = j < nd;
    const uint32_t i = live ? L.dlist[j] : 0u;
    const uint64_t a = off[i], b = off[i + 1];
    const uint32_t hn = b > a ? (uint32_t)min<uint64_t>(b - a, 0xFFFFFFFFull) : 0u;
    const uint32_t prog = live ? lookup_prog(R, T, policy[i], ingress[i] != 0, port[i]) : kProgDeny;
    HeadReader hr((glb_u8*)raw + a, hn, (const lds_u8*)0, false);
    uint32_t flags = ingress[i] ? CG_HTTP_F_INGRESS : 0u, units = 0, len = 0, last = 0;
    bool walk = false;
    if (live) {
      // a list's spans are 16-bit offsets: longer lists (past Envoy's 60 KiB
      // header limit) are rejected
      const bool ok = kLists ? hn <= kFieldsMaxList && parse_list_bytes(R, T, hr, sp, kRawThreads)
                             : parse_head(R, T, hr, sp, kRawThreads);
      if (!ok) {
        flags |= CG_HTTP_F_MALFORMED;
      } else if (walked(R, prog)) {
        len = string_len(R, sp, kRawThreads, &last);
        if (len > CG_HTTP_SLOT_BYTES) walk = true;
        else units = (len + 15) / 16;
      }
    }
    const bool want = live && !walk;
    const RawSlot sl = raw_slot(L, want, raw_vkey(L, group_of(R, prog) * kRawUnits + units, blockIdx.x), prog);
    walk |= want && !sl.ok;
    list_append(L.walk, &L.ctl[kRawCtlWalk], walk, i, lane);
    if (want && sl.ok) {
      raw_fill(L, sl, i, remote[i], flags, units, len, [&](uint4* dst) {
        TileOut<false> o(dst, nullptr);  // raw bytes: http_kernel codes them
        emit_reader(R, hr, sp, kRawThreads, last, o);
      });
    }
  }
}

// ---- each key's last chunk gets its tile count and its last tile's free
// slots become padding (meta PAD, order 0xFFFFFFFF, zero units): one wave per
// (key, stripe), one lane per slot (coalesced stores).  Then the late slots
// (taken, never filled: their requests are walked): every chunk id is
// published by now, so each becomes padding in place — meta PAD (no
// counters), order 0xFFFFFFFF (no verdict), and the tile's data offset when
// it is the tile's slot 0 (whose lane writes it otherwise).
constexpr uint32_t kPadThreads = 256;
__global__ __launch_bounds__(kPadThreads) void raw_pad_kernel(RawLayoutDev L) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t k = blockIdx.x * (kPadThreads / 64) + (threadIdx.x >> 6);  // wave-uniform
  if (k < L.nkeys) {
    const uint32_t cnt = L.kcnt[(size_t)k * kRawCntStride];
    const uint32_t c = cnt ? (cnt - 1) >> L.cshift : 0u;
    if (cnt && c < L.dpk) {
      const unsigned long long v = L.dir[(size_t)k * L.dpk + c];
      const uint32_t id = (uint32_t)v;
      if ((uint32_t)(v >> 32) == L.seq && id < L.maxchunks) {
        const uint32_t used = cnt - (c << L.cshift), nt = (used + 63) >> 6;
        if (lane == 0) L.chunks[id].ntiles = nt;
        const uint32_t t = id * L.ext + nt - 1, units = (k / L.stripes) % kRawUnits;
        uint8_t* tb = L.tiles + (size_t)t * (kRawTileGran * 512);
        if (lane >= used - (nt - 1) * 64) {
          reinterpret_cast<uint2*>(tb)[lane] = make_uint2(0, CG_HTTP_F_PAD << 24);
          L.order[(size_t)t * 64 + lane] = 0xFFFFFFFFu;
          for (uint32_t u = 0; u < units; ++u) reinterpret_cast<uint4*>(tb + 512)[u * 64 + lane] = make_uint4(0, 0, 0, 0);
        }
      }
    }
  }
  const uint32_t nlate = L.ctl[kRawCtlLate];
  for (uint32_t j = blockIdx.x * kPadThreads + threadIdx.x; j < nlate; j += gridDim.x * kPadThreads) {
    const unsigned long long x = L.late[j];
    const uint32_t kk = (uint32_t)(x >> 32), sl = (uint32_t)x, c = sl >> L.cshift;
    const unsigned long long v = L.dir[(size_t)kk * L.dpk + c];
    const uint32_t id = (uint32_t)v;
    if ((uint32_t)(v >> 32) != L.seq || id >= L.maxchunks) continue;  // not in the chunk table
    const uint32_t t = id * L.ext + ((sl >> 6) & (L.ext - 1u)), l = sl & 63u;
    uint8_t* tb = L.tiles + (size_t)t * (kRawTileGran * 512);
    reinterpret_cast<uint2*>(tb)[l] = make_uint2(0, CG_HTTP_F_PAD << 24);
    L.order[(size_t)t * 64 + l] = 0xFFFFFFFFu;
    if (l == 0) L.ttab[t].at = t * kRawTileGran;
  }
}

// ---- the batch's tables, one workgroup (after raw_pad_kernel): the chunk
// table, grouped by program (so a workgroup's run of chunks shares the
// staged program block), and the header go to the front of the batch.
constexpr uint32_t kSealThreads = 1024;
__global__ __launch_bounds__(kSealThreads) void raw_seal_kernel(HttpRawDev R, RawLayoutDev L, uint8_t* __restrict__ batch,
                                                                uint32_t epoch, uint64_t ttab_off, uint64_t tiles_off,
                                                                uint64_t total_bytes, uint32_t sort) {
  extern __shared__ uint32_t sh[];  // [group counts][group cursors] (sort)
  const uint32_t G = R.nprogs + 2, tid = threadIdx.x;
  const uint32_t nch = min(L.ctl[kRawCtlChunks], L.maxchunks);
  HttpChunk* dst = reinterpret_cast<HttpChunk*>(batch + sizeof(HttpBatchHeader));
  auto group = [&](uint32_t prog) { return prog < R.nprogs ? prog : R.nprogs + (prog == kProgAllow ? 0u : 1u); };
  if (sort) {
    uint32_t* cntg = sh;
    uint32_t* cur = sh + G;
    for (uint32_t g = tid; g < G; g += kSealThreads) cntg[g] = 0;
    __syncthreads();
    for (uint32_t id = tid; id < nch; id += kSealThreads) atomicAdd(&cntg[group(L.chunks[id].prog)], 1u);
    __syncthreads();
    if (tid == 0) {
      uint32_t run = 0;
      for (uint32_t g = 0; g < G; ++g) {
        cur[g] = run;
        run += cntg[g];
      }
    }
    __syncthreads();
    for (uint32_t id = tid; id < nch; id += kSealThreads) {
      const HttpChunk ch = L.chunks[id];
      dst[atomicAdd(&cur[group(ch.prog)], 1u)] = HttpChunk{ch.prog, ch.first_tile, ch.ntiles, 0};
    }
  } else {
    for (uint32_t id = tid; id < nch; id += kSealThreads) {
      const HttpChunk ch = L.chunks[id];
      dst[id] = HttpChunk{ch.prog, ch.first_tile, ch.ntiles, 0};
    }
  }
  if (tid == 0) {
    HttpBatchHeader h{};
    h.magic = kBatchMagic;
    h.epoch = epoch;
    h.nchunks = nch;
    h.ntiles = L.maxchunks * L.ext;
    h.tiles_off = tiles_off;
    h.nslots = (uint64_t)h.ntiles * 64;
    h.ttab_off = ttab_off;
    h.total_bytes = total_bytes;
    h.arena_bytes = 0;
    *reinterpret_cast<HttpBatchHeader*>(batch) = h;
  }
}

// ---- the walk list: requests whose walked string passes the slot (and any
// the layout could not take), one lane each — re-parsed from HBM, the string
// built on the fly through the program's code map and walked over the
// program's tables in global memory; the verdict, its counters and rule hit
// as http_kernel gives them (kernels_http.hip http_tiles).
// blk / lut: the program's block and code map (global memory, or LDS copies
// for a rebased program: the persistent ring stages them).
__device__ __forceinline__ uint32_t walk_request_at(const HttpDev& T, const HttpRawDev& R, const HttpProg& pg,
                                                    const uint32_t* blk, const uint8_t* lut, HeadReader& hr,
                                                    const lds_u32* sp, uint32_t stride, uint32_t remote) {
  using namespace walk;
  const bool rebased = pg.flags & kProgRebased;
  uint32_t last;
  (void)string_len(R, sp, stride, &last);
  const uint32_t row = remote_row(blk, pg, remote), W = pg.mask_words;
  uint32_t hit = kNoHit;
  for (uint32_t pi = 0; pi < pg.part_count; ++pi) {
    const HttpPart pt = T.parts[pg.part_begin + pi];
    const bool cls = pt.mode == kPartClass;
    const uint32_t* cells = rebased ? blk : T.cells + pt.walk_off;
    uint32_t st = pt.start;
    auto stp = [&](uint32_t b) {
      const uint32_t x = lut[b];
      st = cls ? step<true>(cells, pt.dead, st, x) : step<false>(cells, pt.dead, st, x);
    };
    for (uint32_t f = 0; f < last && st != pt.dead; ++f) {
      const uint32_t s = sp[f * stride];
      if (s == kAbsentSpan) {
        stp(1u);
      } else {
        const uint32_t a = s >> 16, len = s & 0xFFFFu;
        for (uint32_t k = 0; k < len && st != pt.dead; ++k) stp(hr.at(a + k));
      }
      stp(0u);
    }
    if (last < R.nfields) stp(2u);
    const uint32_t lab = cls ? state_label<true>(cells, st) : state_label<false>(cells, st);
    if (lab != 0xFFFFu) hit = min(hit, first_meet(blk, pt.acc_off + lab * 2 * W, row, W));
  }
  if (pg.flags & kProgHasAlways) hit = min(hit, first_meet(blk, pg.always_off, row, W));
  return hit;
}

// One parsed request's verdict with its counters and rule hit, as
// http_kernel gives them: no policy for the port → allowed when the codec
// accepted it; unknown policy → denied; an allow-all scope → allowed
// (counted); else the walk (cilium_network_policy.h:129-138,187-191).
__device__ __forceinline__ uint32_t decide_request(const HttpDev& HT, const HttpRawDev& R, uint32_t prog, bool ok,
                                                   const uint32_t* blk, const uint8_t* lut, HeadReader& hr,
                                                   const lds_u32* sp, uint32_t stride, uint32_t remote) {
  uint32_t v = 0;
  if (prog == kProgAllow) {
    v = ok;
  } else if (prog < R.nprogs) {
    const HttpProg pg = HT.progs[prog];
    if (pg.flags & kProgAllowAll) {
      v = ok;
      if (ok) atomicAdd(&HT.counters[2 * prog], 1ull);
    } else if (ok) {
      const uint32_t hit = walk_request_at(HT, R, pg, blk ? blk : HT.cells + pg.cell_begin,
                                           lut ? lut : R.codes + (size_t)prog * 256, hr, sp, stride, remote);
      v = hit != walk::kNoHit;
      atomicAdd(&HT.counters[2 * prog + (v ? 0 : 1)], 1ull);
      if (v) atomicAdd(&HT.rule_hits[pg.rule_base + hit], 1ull);
    }
  }
  return v;
}

template <bool kLists>
__global__ __launch_bounds__(kRawThreads) void raw_walk_kernel(HttpDev HT, HttpRawDev R, const uint8_t* __restrict__ raw,
                                                               const uint64_t* __restrict__ off,
                                                               const uint32_t* __restrict__ policy,
                                                               const uint8_t* __restrict__ ingress,
                                                               const uint16_t* __restrict__ port,
                                                               const uint32_t* __restrict__ remote, RawLayoutDev L,
                                                               uint8_t* __restrict__ out) {
  extern __shared__ uint32_t lds_[];
  lds_u32* sp = (lds_u32*)lds_ + threadIdx.x;
  const GlbTabs T{(glb_u32*)R.nkeys, (glb_u32*)R.fslots, (glb_u32*)R.phash_keys, (glb_u32*)R.phash_vals,
                  (glb_u32*)R.walk_bits, (glb_u32*)R.dflt, (glb_u8*)R.fnames};
  const uint32_t nw = L.ctl[kRawCtlWalk];
  for (uint32_t j = blockIdx.x * kRawThreads + threadIdx.x; j < nw; j += gridDim.x * kRawThreads) {
    const uint32_t i = L.walk[j];
    const uint64_t a = off[i], b = off[i + 1];
    const uint32_t hn = b > a ? (uint32_t)min<uint64_t>(b - a, 0xFFFFFFFFull) : 0u;
    const uint32_t prog = lookup_prog(R, T, policy[i], ingress[i] != 0, port[i]);
    HeadReader hr((glb_u8*)raw + a, hn, (const lds_u8*)0, false);
    const bool ok = prog == kProgDeny ? false
                    : kLists          ? hn <= kFieldsMaxList && parse_list_bytes(R, T, hr, sp, kRawThreads)
                                      : parse_head(R, T, hr, sp, kRawThreads);
    out[i] = (uint8_t)decide_request(HT, R, prog, ok, nullptr, nullptr, hr, sp, kRawThreads, remote[i]);
  }
}
// ---- the persistent verdict ring (ring.cc; dev_types.h HttpRingDev) ------
// One wave per workgroup, resident: lane j polls the doorbell of slot
// blockIdx.x + j * nwg ({seq, done} in one system-scope acquire load over the
// bus).  A ready slot's inputs and lists come into LDS with 16-byte loads;
// each request is decided as raw_walk_kernel decides it (program lookup, the
// list parse, decide_request), with the program's block and code map staged
// in LDS when every request of the slot shares one rebased program that fits
// (kept across slots: Envoy's calls on one listener repeat the program).
// The verdicts go back into the slot and `done` is published with a
// system-scope release after them.  Every wave exits: on the host's stop
// word, or when workgroup 0 sees no call for idle_ticks or the launch pass
// life_ticks (it raises the exit word in device memory; each wave serves
// what is ready one last time and leaves) — ring.cc relaunches on the next
// call.
constexpr uint32_t kRingThreads = 64;
bool lds_tables_fit(const HttpRawDev& R);
// device memory of a launch: the exit word, the wall clock of the last call
// served, slots served (read by cg_http_ring_stats)
struct RingState {
  uint32_t exit, pad;
  unsigned long long last, served;
};

// Polls are relaxed system-scope loads (straight to host memory, no cache
// maintenance): an acquire at system scope invalidates the L2 (buffer_inv
// sc0 sc1), and 64 polling waves doing that without pause capped the ring
// at ~0.6 M round trips/s for the whole chip.  A slot seen ready is followed
// by one acquire fence before its data is read.
__device__ __forceinline__ uint32_t sys_load32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long sys_load64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The program block (and code map) of p into LDS by LDS-DMA: every 1 KiB
// piece's global_load_lds_dwordx4 issued back to back (no registers held),
// then one wait — a 64-KB block in about one memory round trip, not eight.
__device__ __forceinline__ void ring_stage(const HttpDev& HT, const HttpRawDev& R, const HttpProg& pg, uint32_t p,
                                           lds_u32* cells, lds_u32* cmap, uint32_t lane) {
  const uint32_t* src = HT.cells + pg.cell_begin;
  const uint32_t n = pg.cell_count;
  uint32_t done = 0;
  if ((((uintptr_t)src) & 15) == 0) {
    const uint32_t n4 = n / 4;  // 16-byte units
    for (uint32_t c0 = 0; c0 < n4; c0 += kRingThreads)
      if (c0 + lane < n4)  // (the last piece's lanes past the block write nothing)
        __builtin_amdgcn_global_load_lds((const void*)(src + 4 * (c0 + lane)),
                                         (__attribute__((address_space(3))) void*)(cells + 4 * c0), 16, 0, 0);
    done = 4 * n4;
  }
  for (uint32_t c = done + lane; c < n; c += kRingThreads) cells[c] = src[c];
  for (uint32_t c = lane; c < 64; c += kRingThreads) cmap[c] = reinterpret_cast<const uint32_t*>(R.codes + (size_t)p * 256)[c];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA'd pieces have landed
}

// The structural masks of a call's lists (list_stop / NUL, as the list
// scan's build_masks_lists) over its blob in LDS: 16 bytes per lane per
// round, mask m1 at kRingMaskWords past m0.
constexpr uint32_t kRingMaskWords = kRingBlob / 32;
__device__ __forceinline__ void ring_masks(const lds_u8* blob, uint32_t bytes, const lds_u8* tct, lds_u32* masks,
                                           uint32_t lane) {
  for (uint32_t r = 0; r * 1024 < bytes; ++r) {
    const uint32_t u = r * 64 + lane;
    const uint4 a = to_uint4(*(const lds_v4*)(blob + 16 * u));
    const uint32_t d[4] = {a.x, a.y, a.z, a.w};
    uint32_t m0 = 0, m1 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      m1 |= zero4(d[k]) << (4 * k);
#pragma unroll
      for (int j = 0; j < 4; ++j) m0 |= (uint32_t)tct[(d[k] >> (8 * j)) & 0xFFu] << (4 * k + j);
    }
    const uint32_t o0 = pair_swap(m0), o1 = pair_swap(m1);
    if (!(lane & 1u) && (u >> 1) < kRingMaskWords) {  // (the last round's units past the blob: bits past it)
      masks[u >> 1] = m0 | o0 << 16;
      masks[kRingMaskWords + (u >> 1)] = m1 | o1 << 16;
    }
  }
}
// The walked string (http_pack.cc: the fields' values up to the last
// present one, each SEP-terminated, ABSENT for a missing one, REST when a
// later field is missing) walked straight from the parsed spans in the
// call's LDS blob: four bytes per two LDS reads and a byte align (squad),
// the next four bytes and their codes loaded ahead of this four's steps, so
// only the cell load is on the chain.  Cells and codes are LDS pointers
// when the program is staged (ds_read, not flat loads).
__device__ __forceinline__ uint32_t ring_cell(const lds_u32* cells, uint32_t byte_off) {
  return *(const lds_u32*)((const lds_u8*)cells + byte_off);
}
__device__ __forceinline__ uint32_t ring_cell(const uint32_t* cells, uint32_t byte_off) {
  return *(const uint32_t*)((const uint8_t*)cells + byte_off);
}
template <bool kCls, class CellP>
__device__ __forceinline__ uint32_t ring_step(CellP cells, uint32_t dead, uint32_t st, uint32_t x) {
  // walk::comb_step / comb_step_cls on the typed pointer
  const uint32_t e = ring_cell(cells, kCls ? st + x : (st << 2) + (x << 2));
  const uint32_t dflt = max(st, dead);
  uint32_t nx;
  asm("v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:WORD_0 src1_sel:DWORD\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_sdwa %0, %3, %1, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
      : "=v"(nx)
      : "v"(e), "v"(st), "v"(dflt)
      : "vcc");
  return nx;
}
template <bool kCls, class CellP, class CodeP>
__device__ __forceinline__ uint32_t ring_run(const HttpRawDev& R, CellP cells, uint32_t dead, uint32_t st, CodeP lut,
                                             const lds_u8* blob, uint32_t hs, const lds_u32* sp, const Parsed& P,
                                             uint32_t last) {
  const uint32_t c_sep = lut[0], c_abs = lut[1];
  uint32_t f = 0;
  for (uint32_t rem = P.present; rem && st != dead; rem &= rem - 1) {
    const uint32_t g = (uint32_t)__builtin_ctz(rem);
    for (; f < g && st != dead; ++f) {
      st = ring_step<kCls>(cells, dead, st, c_abs);
      st = st == dead ? st : ring_step<kCls>(cells, dead, st, c_sep);
    }
    const uint32_t sv = sp[g * kRingThreads], a = hs + (sv >> 16), L = sv & 0xFFFFu;
    uint32_t w = squad(blob, a), k = 0;
    // whole quads unguarded (the dead state is absorbing: a step from it
    // stays there, as http_kernel's unguarded unit walk relies on), then the
    // last 1-3 bytes
    for (; k + 4 <= L && st != dead; k += 4) {
      const uint32_t wn = squad(blob, a + k + 4);  // (past the value: unused)
      uint32_t x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = lut[(w >> (8 * j)) & 0xFFu];
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) st = ring_step<kCls>(cells, dead, st, x[j]);
      w = wn;
    }
    for (uint32_t j = 0; k + j < L && st != dead; ++j) st = ring_step<kCls>(cells, dead, st, (uint32_t)lut[(w >> (8 * j)) & 0xFFu]);
    st = st == dead ? st : ring_step<kCls>(cells, dead, st, c_sep);
    f = g + 1;
  }
  if (last < R.nfields && st != dead) st = ring_step<kCls>(cells, dead, st, (uint32_t)lut[2]);  // REST
  return st;
}
// walk::remote_row / state_label / first_meet over a typed block pointer
// (LDS when staged: ds_read, not flat loads).
__device__ __forceinline__ uint4 ring_q(const lds_u32* p) { return to_uint4(*(const lds_v4*)p); }
__device__ __forceinline__ uint4 ring_q(const uint32_t* p) { return *(const uint4*)p; }
__device__ __forceinline__ uint32_t ring_w(const lds_u32* p) { return *p; }
__device__ __forceinline__ uint32_t ring_w(const uint32_t* p) { return *p; }
__device__ __forceinline__ uint32_t ring_h(const lds_u32* p, uint32_t i) { return ((const CG_LDS uint16_t*)p)[i]; }
__device__ __forceinline__ uint32_t ring_h(const uint32_t* p, uint32_t i) { return ((const uint16_t*)p)[i]; }
template <class CellP>
__device__ __forceinline__ uint32_t ring_remote_row(CellP blk, const HttpProg& pg, uint32_t remote) {
  if (pg.flags & kProgRemoteDirect) {
    const uint32_t d = remote - pg.rdir_base;
    const bool in = d < pg.rdir_len;
    const uint32_t v = ring_h(blk + pg.rdir_off, in ? d : 0);
    return in ? v : pg.default_remote;
  }
  const uint32_t h = rtab_hash(remote);
  const CellP b1 = blk + pg.rtab_off + kRtabBucketCells * rtab_b1h(h, pg.rtab_nb);
  const CellP b2 = blk + pg.rtab_off + kRtabBucketCells * rtab_b2h(h, pg.rtab_nb);
  const uint4 k1 = ring_q(b1), k2 = ring_q(b2), r1 = ring_q(b1 + 4), r2 = ring_q(b2 + 4);
  uint32_t row = pg.default_remote;
  row = k1.x == remote ? r1.x : row;
  row = k1.y == remote ? r1.y : row;
  row = k1.z == remote ? r1.z : row;
  row = k1.w == remote ? r1.w : row;
  row = k2.x == remote ? r2.x : row;
  row = k2.y == remote ? r2.y : row;
  row = k2.z == remote ? r2.z : row;
  row = k2.w == remote ? r2.w : row;
  return row;
}
template <class CellP>
__device__ __forceinline__ uint32_t ring_first_meet(CellP blk, uint32_t a, uint32_t row, uint32_t W) {
  for (uint32_t w = 0; w < W; ++w) {
    const unsigned long long x = ((unsigned long long)ring_w(blk + a + 2 * w + 1) << 32 | ring_w(blk + a + 2 * w)) &
                                 ((unsigned long long)ring_w(blk + row + 2 * w + 1) << 32 | ring_w(blk + row + 2 * w));
    if (x) return w * 64 + (uint32_t)__builtin_ctzll(x);
  }
  return walk::kNoHit;
}
// walk_request_at from the parsed spans over the program's block and code
// map at blk / lut (LDS, staged, or global memory); pt0: its first part.
template <class CellP, class CodeP>
__device__ __forceinline__ uint32_t walk_spans_at(const HttpDev& T, const HttpRawDev& R, const HttpProg& pg,
                                                  const HttpPart& pt0, CellP blk, CodeP lut, const lds_u8* blob,
                                                  uint32_t hs, const lds_u32* sp, const Parsed& P, uint32_t last,
                                                  uint32_t remote) {
  const uint32_t row = ring_remote_row(blk, pg, remote), W = pg.mask_words;
  uint32_t hit = walk::kNoHit;
  for (uint32_t pi = 0; pi < pg.part_count; ++pi) {
    const HttpPart pt = pi ? T.parts[pg.part_begin + pi] : pt0;
    const bool cls = pt.mode == kPartClass;
    // (a program walked from global memory without a rebased block reads its
    // cells at their place in the table)
    CellP cells = blk;  // (staged programs are rebased)
    if constexpr (std::is_same<CellP, const uint32_t*>::value)
      if (!(pg.flags & kProgRebased)) cells = T.cells + pt.walk_off;
    const uint32_t st = cls ? ring_run<true>(R, cells, pt.dead, pt.start, lut, blob, hs, sp, P, last)
                            : ring_run<false>(R, cells, pt.dead, pt.start, lut, blob, hs, sp, P, last);
    const uint32_t lab = (cls ? ring_cell(cells, st - 4) : ring_cell(cells, 4 * (st - 1))) >> 16;
    if (lab != 0xFFFFu) hit = min(hit, ring_first_meet(blk, pt.acc_off + lab * 2 * W, row, W));
  }
  if (pg.flags & kProgHasAlways) hit = min(hit, ring_first_meet(blk, pg.always_off, row, W));
  return hit;
}

template <class Tabs>
__device__ __forceinline__ void ring_serve(const HttpDev& HT, const HttpRawDev& R, const Tabs& T, const HttpRingDev& G,
                                           uint32_t s, uint32_t seq, lds_u8* in, lds_u32* sp, lds_u32* cells,
                                           lds_u32* cmap, lds_u32* masks, const lds_u8* tct, uint32_t& staged,
                                           HttpProg& spg, HttpPart& spt, uint32_t lane) {
  uint8_t* hs = G.slots + (size_t)s * kRingSlotBytes;     // the request
  uint8_t* ho = G.reply + (size_t)s * G.reply_stride;      // the reply (host memory)
  // (atomic loads: vector memory, never a cached scalar read of the slot)
  uint32_t* hw = reinterpret_cast<uint32_t*>(hs);
  uint32_t* ow = reinterpret_cast<uint32_t*>(ho);
  // the answered seq in the request slot (what the poll compares the
  // doorbell with; the same word as `done` when the slots are one)
  if (ho != hs && lane == 0) __hip_atomic_store(hw + 1, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (G.echo == 1) {  // transport experiment: no work at all
    if (lane == 0) __hip_atomic_store(ow + 1, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the slot's data after its doorbell
  uint32_t stamp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t cyc0 = 0;
  if (G.trace) {
    stamp[0] = (uint32_t)wall_clock64();
    cyc0 = clock64();
  }
  // the call's first KiB is loaded with its size words, not after them (one
  // round trip over the bus for a small call), the rest once they are known
  const uint8_t* src = hs + kRingData;
  const uint4 first = to_uint4(*(const glb_v4*)(src + lane * 16));
  const uint32_t n = min(__hip_atomic_load(hw + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), kRingReqs);
  const uint32_t bytes = min(__hip_atomic_load(hw + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), kRingBlob);
  const RingLayout L = ring_layout(n);
  const uint32_t total = (L.blob + bytes + 15) & ~15u;
  *(lds_v4*)(in + lane * 16) = to_v4(first);
  for (uint32_t o0 = kRingThreads * 16 + lane * 16; o0 < total; o0 += kRingThreads * 16 * 4) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      v[u] = to_uint4(*(const glb_v4*)(src + min(o0 + u * kRingThreads * 16, total - 16)));
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (o0 + u * kRingThreads * 16 < total) *(lds_v4*)(in + o0 + u * kRingThreads * 16) = to_v4(v[u]);
  }
  wave_sync();
  const lds_u32* pol = (const lds_u32*)in;
  const lds_u32* rem = (const lds_u32*)(in + L.rem);
  const CG_LDS uint16_t* prt = (const CG_LDS uint16_t*)(in + L.port);
  const lds_u8* ing = in + L.ing;
  const lds_u32* off = (const lds_u32*)(in + L.off);
  const lds_u8* blob = in + L.blob;
  ring_masks(blob, bytes, tct, masks, lane);
  wave_sync();
  if (G.trace) stamp[1] = (uint32_t)wall_clock64();
  if (G.echo == 2) {  // transport experiment: the data in, no decision
    wave_sync();
    if (lane == 0) __hip_atomic_store(ow + 1, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  for (uint32_t b = 0; b < n; b += kRingThreads) {  // uniform
    const uint32_t i = b + lane;
    const bool live = i < n;
    const uint32_t prog = live ? lookup_prog(R, T, pol[i], ing[i] != 0, prt[i]) : kProgDeny;
    // one program for every live lane: its block (and code map) in LDS
    const uint32_t p0 = (uint32_t)__shfl((int)prog, 0, kRingThreads);
    const bool same = !__ballot(live && prog != p0);
    bool lds = false;
    if (same && p0 < R.nprogs) {
      // the staged program's record and first part stay in registers (a
      // copy and a uniform branch: `c ? spg : HT.progs[p0]` selects between
      // two addresses, which put spg in scratch and cost a flat load per call)
      HttpProg pg = spg;
      if (staged != p0) pg = HT.progs[p0];
      lds = !(pg.flags & kProgAllowAll) && (pg.flags & kProgRebased) && pg.cell_count <= G.lds_cells;
      if (lds && staged != p0) {
        wave_sync();
        ring_stage(HT, R, pg, p0, cells, cmap, lane);
        spg = pg;
        spt = HT.parts[pg.part_begin];
        staged = p0;
        wave_sync();
      }
    }
    if (G.trace && b == 0) stamp[2] = (uint32_t)wall_clock64();
    // a single-request call: its list parsed by the whole wave
    Parsed P0{};
    bool ok0 = false, coop = false;
    if (n == 1 && !R.raw_values) {  // uniform
      const uint32_t a0 = min(off[0], bytes), e0 = min(max(off[1], a0), bytes);
      if (p0 != kProgDeny && e0 - a0 <= kFieldsMaxList)
        coop = parse_list_coop(R, T, blob, masks, masks + kRingMaskWords, a0, e0, sp - lane, kRingThreads,
                               (lds_u32*)(in + total), lane, P0, ok0);
    }
    uint32_t v = 0;
    if (live) {
      const uint32_t a = min(off[i], bytes), e = min(max(off[i + 1], a), bytes);
      // the list over the call's masks (parse_list_fast), then decide_request
      // with the walk over the emitted string
      Parsed P = P0;
      const bool ok = coop ? ok0
                           : prog != kProgDeny && e - a <= kFieldsMaxList &&
                                 (R.raw_values ? parse_list_fast(R, T, blob, masks, masks + kRingMaskWords, a, e, sp,
                                                                 kRingThreads, P)
                                               : parse_list_win(R, T, blob, masks, masks + kRingMaskWords, a, e, sp,
                                                                kRingThreads, P));
      if (G.trace && i == 0) stamp[4] = stamp[5] = (uint32_t)wall_clock64();
      const uint32_t* blk = lds ? (const uint32_t*)cells : nullptr;
      const uint8_t* lut = lds ? (const uint8_t*)cmap : nullptr;
      if (prog == kProgAllow) {
        v = ok;
      } else if (prog < R.nprogs) {
        HttpProg pg = spg;
        if (!lds) pg = HT.progs[prog];
        if (pg.flags & kProgAllowAll) {
          v = ok;
          if (ok) atomicAdd(&HT.counters[2 * prog], 1ull);
        } else if (ok) {
          uint32_t last;
          (void)walked_len(R, P, &last);
          const uint32_t* bk = blk ? blk : HT.cells + pg.cell_begin;
          const uint8_t* lt = lut ? lut : R.codes + (size_t)prog * 256;
          HttpPart pt0 = spt;
          if (!lds) pt0 = HT.parts[pg.part_begin];
          const uint32_t hit = lds ? walk_spans_at(HT, R, pg, pt0, (const lds_u32*)cells, (const lds_u8*)cmap, blob, a,
                                                   sp, P, last, rem[i])
                                   : walk_spans_at(HT, R, pg, pt0, bk, lt, blob, a, sp, P, last, rem[i]);
          v = hit != walk::kNoHit;
          atomicAdd(&HT.counters[2 * prog + (v ? 0 : 1)], 1ull);
          if (v) atomicAdd(&HT.rule_hits[pg.rule_base + hit], 1ull);
        }
      }
      ho[kRingOut + i] = (uint8_t)v;
    }
  }
  if (G.trace) stamp[6] = (uint32_t)wall_clock64();
  wave_sync();
  if (G.trace) {
    stamp[7] = (uint32_t)wall_clock64();
    // request 0's parse / emit stamps are lane 0's (0 when it took another way)
    stamp[3] = (uint32_t)__shfl((int)stamp[4], 0, kRingThreads);
    stamp[4] = (uint32_t)__shfl((int)stamp[5], 0, kRingThreads);
    stamp[3] = stamp[3] ? stamp[3] : stamp[2];
    stamp[4] = stamp[4] ? stamp[4] : stamp[3];
    stamp[5] = stamp[6];
    stamp[6] = stamp[7];
    const uint32_t cyc = (uint32_t)(clock64() - cyc0);  // shader clock cycles over the serve
    if (lane <= kRingStamps) {
      uint32_t x = lane == kRingStamps ? cyc : stamp[0];
      for (uint32_t j = 1; j < kRingStamps; ++j) x = lane == j ? stamp[j] : x;
      ow[kRingStampAt + lane] = x;
    }
  }
  // the verdicts (and the counters, stamps) before `done`: one release, then
  // a relaxed store of the word (a release store would write the L2 back a
  // second time)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  wave_sync();
  if (lane == 0) __hip_atomic_store(ow + 1, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool kLdsTabs>
__global__ __launch_bounds__(kRingThreads) void http_ring_kernel(HttpDev HT, HttpRawDev R, HttpRingDev G,
                                                                 RingState* __restrict__ st) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_ring_[];
  lds_u32* lds = (lds_u32*)lds_ring_;
  const uint32_t F = max(R.nfields, 1u), lane = threadIdx.x;
  // LDS: [call data: kRingDataMax][spans: F x 64][code map: 64 words]
  // [list masks: 2 x kRingMaskWords][stop table: 64 words][lookup tables,
  // kLdsTabs][program block: G.lds_cells]
  lds_u8* in = (lds_u8*)lds;
  lds_u32* sp = lds + kRingDataMax / 4 + lane;
  lds_u32* cmap = lds + kRingDataMax / 4 + F * kRingThreads;
  lds_u32* masks = cmap + 64;
  lds_u8* tct = (lds_u8*)(masks + 2 * kRingMaskWords);
  lds_u32* tabs = (lds_u32*)(tct + 256);
  for (uint32_t b = lane; b < 256; b += kRingThreads) tct[b] = list_stop(b, R.raw_values);
  using Tabs = typename std::conditional<kLdsTabs, LdsTabs, GlbTabs>::type;
  Tabs T;
  stage_tables(R, tabs, T);
  lds_u32* cells = tabs + ((kLdsTabs ? raw_tables_lds_words(R) : 0u) + 3u & ~3u);  // 16-byte aligned
  wave_sync();
  const uint32_t wg = blockIdx.x;
  const uint32_t per = G.nslots > wg ? (G.nslots - wg + G.nwg - 1) / G.nwg : 0u;  // slots of this workgroup
  const bool mine = lane < per;
  const uint32_t my = wg + lane * G.nwg;
  const unsigned long long* hdr =
      reinterpret_cast<const unsigned long long*>(G.slots + (size_t)(mine ? my : 0) * kRingSlotBytes);
  const uint64_t t0 = wall_clock64();
  uint32_t staged = 0xFFFFFFFFu;
  HttpProg spg{};
  HttpPart spt{};
  for (uint32_t it = 0, last_pass = 0;; ++it) {
    const unsigned long long sd = mine ? sys_load64(hdr) : 0ull;
    const uint32_t seq = (uint32_t)sd, done = (uint32_t)(sd >> 32);
    unsigned long long m = __ballot(mine && seq != done);
    const bool busy = m != 0;
    if (busy && lane == 0)
      __hip_atomic_store(&st->last, (unsigned long long)wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (m) {
      const uint32_t j = (uint32_t)__builtin_ctzll(m);
      m &= m - 1;
      ring_serve(HT, R, T, G, wg + j * G.nwg, (uint32_t)__shfl((int)seq, (int)j, kRingThreads), in, sp, cells, cmap,
                 masks, tct, staged, spg, spt, lane);
      if (lane == 0) atomicAdd(&st->served, 1ull);
    }
    if (last_pass) break;
    // idle, or every 32nd busy pass: the stop word, idle and life bounds
    // (workgroup 0 decides for all), so a launch under steady load ends too
    if (busy && (it & 31)) continue;
    const uint64_t now = wall_clock64();
    if (wg == 0 && lane == 0) {
      const unsigned long long lw = __hip_atomic_load(&st->last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t since = lw > t0 ? lw : t0;
      // (another workgroup may have stamped a call after this one read `now`:
      // since > now is not idle)
      if (sys_load32(&G.ctl[kRingStop]) || (now > since && now - since > G.idle_ticks) || now - t0 > G.life_ticks)
        __hip_atomic_store(&st->exit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint32_t ex = __hip_atomic_load(&st->exit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // past life + idle every wave leaves without the exit word (a bound
    // that does not depend on workgroup 0)
    const bool out = ex || now - t0 > G.life_ticks + G.idle_ticks;
    if (__shfl((int)out, 0, kRingThreads)) {
      last_pass = 1;  // serve what is ready one more time, then leave
      continue;
    }
    if (!busy) __builtin_amdgcn_s_sleep(4);
  }
}

// The device's constant-rate counter, for ring.cc to measure its rate.
__global__ void ring_clock_kernel(unsigned long long* out) {
  if (threadIdx.x == 0) *out = (unsigned long long)wall_clock64();
}

int launch_http_ring_impl(const HttpDev& HT, const HttpRawDev& R, const HttpRingDev& G, void* state, void* stream) {
  const size_t lds = ring_lds_bytes(R, G.lds_cells, G.lds_tabs != 0);
  const auto k = G.lds_tabs ? http_ring_kernel<true> : http_ring_kernel<false>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(k, dim3(G.nwg), dim3(kRingThreads), lds, (hipStream_t)stream, HT, R, G, (RingState*)state);
  return (int)hipGetLastError();
}

unsigned grid_for(size_t n, int cus, unsigned per_cu) {
  const size_t want = (n + kRawThreads - 1) / kRawThreads;
  return (unsigned)std::max<size_t>(1, std::min<size_t>(want, (size_t)cus * per_cu));
}

// LDS of the scan / emit kernels (see wave_stage, key_counters)
bool lds_tables_fit(const HttpRawDev& R) { return raw_tables_lds_words(R) * 4 <= 8 * 1024; }
size_t raw_lds(const HttpRawDev& R, bool lds_keys, bool lds_codes) {
  const size_t nk = ((size_t)R.nprogs + 2) * kRawKeys;
  return (size_t)std::max(R.nfields, 1u) * kRawThreads * 4 + kRawWaves * (size_t)kStage + kRawWaves * 2 * (kStage / 8) + kTctBytes +
         (lds_keys ? nk * 4 : 0) + (lds_tables_fit(R) ? (size_t)raw_tables_lds_words(R) * 4 : 0) +
         (lds_codes ? (size_t)R.nprogs * 256 : 0) + 16 + 12;  // + slack: a quad read may pass the last stage by 7 bytes; the tables' alignment
}
// code maps in LDS only while small: a larger table costs workgroups per CU
// (occupancy) more than its global (L1-cached) lookups cost
bool lds_codes_fit(const HttpRawDev& R) { return (size_t)R.nprogs * 256 <= 4 * 1024; }

using ScanKernel = decltype(&raw_scan_kernel<false, false>);
ScanKernel scan_kernel_for(const HttpRawDev& R, bool lists) {
  const bool tabs = lds_tables_fit(R);
  if (lists) return tabs ? raw_scan_kernel<true, true> : raw_scan_kernel<true, false>;
  return tabs ? raw_scan_kernel<false, true> : raw_scan_kernel<false, false>;
}

using DlScanKernel = decltype(&raw_scan_dl_kernel<false, false>);
DlScanKernel dl_scan_kernel_for(const HttpRawDev& R, bool lists) {
  const bool tabs = lds_tables_fit(R);
  if (lists) return tabs ? raw_scan_dl_kernel<true, true> : raw_scan_dl_kernel<true, false>;
  return tabs ? raw_scan_dl_kernel<false, true> : raw_scan_dl_kernel<false, false>;
}

}  // namespace

// One resident round of scan workgroups: as many per CU as the scan's LDS
// and registers allow (a grid past that runs a second, mostly idle round:
// 4 requested per CU with 3 resident took 2 rounds of 475 stages per wave).
size_t http_raw_grid(const HttpRawDev& R, bool lists, size_t n, int cus) {
  const ScanKernel kern = scan_kernel_for(R, lists);
  const size_t lds = raw_lds(R, http_raw_lds_keys(R), false);
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, size_t>, int> occ;
  int dev = 0;
  (void)hipGetDevice(&dev);
  int per_cu = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = occ.find({dev, (const void*)kern, lds});
    if (it == occ.end()) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kern, kRawThreads, lds) != hipSuccess || nb < 1)
        nb = 1;
      it = occ.emplace(std::make_tuple(dev, (const void*)kern, lds), nb).first;
    }
    per_cu = it->second;
  }
  return grid_for(n, cus, (unsigned)per_cu);
}

bool http_raw_lds_keys(const HttpRawDev& R) { return ((size_t)R.nprogs + 2) * kRawKeys * 4 <= 32 * 1024; }

int launch_http_raw_scan(const HttpRawDev& R, bool lists, const uint8_t* raw, const uint64_t* off, size_t n,
                         const uint32_t* policy, const uint8_t* ingress, const uint16_t* port, uint32_t* counts,
                         void* rinfo, const uint32_t* remote, uint8_t* sbuf, uint32_t cst,
                         unsigned long long* ovf_bytes, uint32_t* dlist, uint32_t* dcount, void* stream, int cus) {
  if (!n) return 0;
  const bool lk = http_raw_lds_keys(R);
  const size_t lds = raw_lds(R, lk, false);
  const ScanKernel kern = scan_kernel_for(R, lists);
  const unsigned grid = (unsigned)http_raw_grid(R, lists, n, cus);
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kRawThreads), lds, (hipStream_t)stream, R, raw, off, n, policy, ingress,
                     port, counts, (uint2*)rinfo, remote, sbuf, cst, ovf_bytes, (uint32_t)lk, dlist, dcount);
  // the deferred requests (their count stays on the device: a small grid
  // that exits at once when there are none)
  const size_t dlds = (size_t)std::max(R.nfields, 1u) * kRawThreads * 4;
  const auto dk = lists ? raw_defer_kernel<true> : raw_defer_kernel<false>;
  (void)hipFuncSetAttribute((const void*)dk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(dk, dim3((unsigned)std::max(1, cus) * 2), dim3(kRawThreads), dlds, (hipStream_t)stream, R, raw, off,
                     policy, ingress, port, counts, grid, (uint32_t)lk, (uint2*)rinfo, remote, sbuf, cst, ovf_bytes,
                     (const uint32_t*)dlist, (const uint32_t*)dcount);
  return (int)hipGetLastError();
}

int launch_http_raw_prefix(const uint32_t* bcount, uint32_t nkeys, uint32_t nblk, uint32_t* bbase, uint32_t* hist,
                           void* stream) {
  if (!nkeys) return 0;
  hipLaunchKernelGGL(raw_prefix_kernel, dim3(nkeys), dim3(256), 0, (hipStream_t)stream, bcount, nblk, bbase, hist);
  return (int)hipGetLastError();
}

int launch_http_raw_rank(const HttpRawDev& R, bool lists, size_t n, const void* rinfo, uint32_t* cursor,
                         const uint32_t* bbase, uint32_t* order, void* stream, int cus) {
  if (!n) return 0;
  const bool lk = http_raw_lds_keys(R);
  const size_t lds = lk ? ((size_t)R.nprogs + 2) * kRawKeys * 4 : 0;
  hipLaunchKernelGGL(raw_rank_kernel, dim3((unsigned)http_raw_grid(R, lists, n, cus)), dim3(kRawThreads), lds,
                     (hipStream_t)stream, R, n, (const uint2*)rinfo, cursor, bbase, (uint32_t)lk, order);
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

// As http_raw_grid, for raw_scan_dl_kernel.
size_t http_raw_dl_grid(const HttpRawDev& R, bool lists, size_t n, int cus) {
  const DlScanKernel kern = dl_scan_kernel_for(R, lists);
  const size_t lds = raw_lds(R, false, false);
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, size_t>, int> occ;
  int dev = 0;
  (void)hipGetDevice(&dev);
  int per_cu = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = occ.find({dev, (const void*)kern, lds});
    if (it == occ.end()) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kern, kRawThreads, lds) != hipSuccess || nb < 1)
        nb = 1;
      it = occ.emplace(std::make_tuple(dev, (const void*)kern, lds), nb).first;
      if (getenv("CILIUM_GPU_DEBUG"))
        fprintf(stderr, "[cilium-gpu] raw_scan_dl_kernel<%d>: %zu B of LDS per workgroup, %d workgroups per CU\n",
                (int)lists, lds, nb);
    }
    per_cu = it->second;
  }
  // (CILIUM_GPU_RAW_SCAN_WG: fewer workgroups per CU, for measurements)
  if (const char* v = getenv("CILIUM_GPU_RAW_SCAN_WG")) per_cu = std::max(1, std::min(per_cu, atoi(v)));
  return grid_for(n, cus, (unsigned)per_cu);
}

int launch_http_raw_dl_scan(const HttpRawDev& R, bool lists, const uint8_t* raw, const uint64_t* off, size_t n,
                         const uint32_t* policy, const uint8_t* ingress, const uint16_t* port, const uint32_t* remote,
                         const RawLayoutDev& L, void* stream, int cus) {
  if (!n) return 0;
  const size_t lds = raw_lds(R, false, false);
  const DlScanKernel kern = dl_scan_kernel_for(R, lists);
  const unsigned grid = (unsigned)http_raw_dl_grid(R, lists, n, cus);
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kRawThreads), lds, (hipStream_t)stream, R, raw, off, n, policy, ingress,
                     port, remote, L);
  // the deferred requests (their count stays on the device: a small grid
  // that exits at once when there are none)
  const size_t dlds = (size_t)std::max(R.nfields, 1u) * kRawThreads * 4;
  const auto dk = lists ? raw_defer_dl_kernel<true> : raw_defer_dl_kernel<false>;
  (void)hipFuncSetAttribute((const void*)dk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(dk, dim3((unsigned)std::max(1, cus) * 2), dim3(kRawThreads), dlds, (hipStream_t)stream, R, raw, off,
                     policy, ingress, port, remote, L);
  return (int)hipGetLastError();
}

bool http_raw_seal_sorts(const HttpRawDev& R) { return ((size_t)R.nprogs + 2) * 8 <= 64 * 1024; }

int launch_http_raw_seal(const HttpRawDev& R, const RawLayoutDev& L, void* batch, uint32_t epoch, uint64_t ttab_off,
                         uint64_t tiles_off, uint64_t total_bytes, void* stream) {
  const bool sort = http_raw_seal_sorts(R);
  const size_t lds = sort ? ((size_t)R.nprogs + 2) * 8 : 0;
  (void)hipFuncSetAttribute((const void*)raw_seal_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const unsigned pad_grid = std::max(1u, (L.nkeys + kPadThreads / 64 - 1) / (kPadThreads / 64));
  hipLaunchKernelGGL(raw_pad_kernel, dim3(pad_grid), dim3(kPadThreads), 0, (hipStream_t)stream, L);
  hipLaunchKernelGGL(raw_seal_kernel, dim3(1), dim3(kSealThreads), lds, (hipStream_t)stream, R, L, (uint8_t*)batch,
                     epoch, ttab_off, tiles_off, total_bytes, (uint32_t)sort);
  return (int)hipGetLastError();
}

size_t ring_lds_bytes(const HttpRawDev& R, uint32_t cells, bool tabs) {
  return kRingDataMax + (size_t)std::max(R.nfields, 1u) * kRingThreads * 4 + 256 + 8 * kRingMaskWords + 256 +
         (tabs ? (size_t)raw_tables_lds_words(R) * 4 + 12 : 0) + (size_t)cells * 4;
}
bool ring_tables_small(const HttpRawDev& R) { return lds_tables_fit(R); }
int ring_clock(unsigned long long* d_out, void* stream) {
  hipLaunchKernelGGL(ring_clock_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_out);
  return (int)hipGetLastError();
}
size_t http_ring_state_bytes() { return sizeof(RingState); }
int launch_http_ring(const HttpDev& HT, const HttpRawDev& R, const HttpRingDev& G, void* state, void* stream) {
  return launch_http_ring_impl(HT, R, G, state, stream);
}

int launch_http_raw_walk(const HttpDev& T, const HttpRawDev& R, bool lists, const uint8_t* raw, const uint64_t* off,
                         const uint32_t* policy, const uint8_t* ingress, const uint16_t* port, const uint32_t* remote,
                         const RawLayoutDev& L, uint8_t* out, void* stream, int cus) {
  const size_t lds = (size_t)std::max(R.nfields, 1u) * kRawThreads * 4;
  const auto wk = lists ? raw_walk_kernel<true> : raw_walk_kernel<false>;
  (void)hipFuncSetAttribute((const void*)wk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(wk, dim3((unsigned)std::max(1, cus) * 2), dim3(kRawThreads), lds, (hipStream_t)stream, T, R, raw,
                     off, policy, ingress, port, remote, L, out);
  return (int)hipGetLastError();
}

}  // namespace cg
