// kernels_http.hip — HTTP L7 verdict kernel (gfx950).
//
// NetworkPolicyMap::Allowed (envoy/cilium_network_policy.h:223-237) for every
// slot of a program-grouped batch (http_pack.cc).  One workgroup takes one
// chunk of ≤ kChunkTiles tiles of a single program: it stages the program's
// block — comb-packed DFA (comb.h), accept-label table, PNPR masks and the
// remote-identity table — into
// LDS, then each wavefront walks 64 requests at a time, one lane per request.
// Records are tile-transposed, so each of a wave's 16-byte unit loads is one
// contiguous 1 KiB read; the DFA walk touches only LDS (one ds_read_b32 per
// byte).  The walk is latency-bound (a dependent LDS read per byte), so the
// common path streams a wave's tiles: the next tile's first units load while
// the current tile walks, and units within a tile load two ahead.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>

#include "../../include/cilium_gpu.h"
#include "dev_types.h"
#include "http_walk.h"
#include "kernels.h"

namespace cg {

namespace {

using namespace walk;

constexpr int kWave = 64;
constexpr int kHttpThreads = 1024;
constexpr int kTilesPerWave = 1;  // strings walked per lane at a time
constexpr int kHttpWaves = 8;     // waves per SIMD http_kernel is built for (64 VGPRs)
constexpr uint32_t kDealRun = 4;  // consecutive chunks per workgroup turn
// Runs of chunks are taken from a per-launch ticket counter (dynamic
// dealing): chunk costs vary with their tiles' string lengths, and a static
// deal lets the unluckiest workgroup set the kernel's tail.
constexpr bool kDynamicDeal = true;

__device__ __forceinline__ uint32_t get_byte(const uint4& w, int k) {
  const uint32_t word = (k < 4) ? w.x : (k < 8) ? w.y : (k < 12) ? w.z : w.w;
  return (word >> ((k & 3) * 8)) & 0xFFu;
}


// Class-mode step on byte B of word w, block at LDS address 0 (the fast
// path): four VALU.  Written out because the compiler adds the dynamic-LDS
// base (0) as an operand and then splits the byte select from the add.
template <int B>
__device__ __forceinline__ uint32_t lds_cls_step(uint32_t dead, uint32_t st, uint32_t w) {
  uint32_t e, d, nx;
#define CG_CLS_STEP(b)                                                                                   \
  asm volatile("v_add_u32_sdwa %0, %3, %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" b \
               "\n\tds_read_b32 %0, %0\n\t"                                                              \
               "v_max_u32 %1, %5, %3\n\t"                                                                \
               "s_waitcnt lgkmcnt(0)\n\t"                                                                \
               "v_cmp_eq_u32_sdwa vcc, %0, %3 src0_sel:WORD_0 src1_sel:DWORD\n\t"                       \
               "s_nop 1\n\t"                                                                             \
               "v_cndmask_b32_sdwa %2, %1, %0, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "  \
               "src1_sel:WORD_1"                                                                        \
               : "=&v"(e), "=&v"(d), "=v"(nx)                                                           \
               : "v"(st), "v"(w), "s"(dead)                                                             \
               : "vcc")
  if (B == 0) CG_CLS_STEP("BYTE_0");
  else if (B == 1) CG_CLS_STEP("BYTE_1");
  else if (B == 2) CG_CLS_STEP("BYTE_2");
  else CG_CLS_STEP("BYTE_3");
#undef CG_CLS_STEP
  return nx;
}

template <int I>
__device__ __forceinline__ uint32_t lds_cls_step16(uint32_t dead, uint32_t st, const uint4& u) {
  const uint32_t w = I < 4 ? u.x : I < 8 ? u.y : I < 12 ? u.z : u.w;
  return lds_cls_step<I & 3>(dead, st, w);
}

// 16 raw string bytes → their class codes through the program's code map,
// staged in LDS at byte address cm (raw-byte batches, launch_http codes):
// one ds_read_u8 per byte, eight in flight per wait, each word joined by
// three shift-ors (every address in its own register) — none of it on the walk's dependent chain.  (D16 loads
// into the two halves of one register cannot both be in flight: the second
// merges the register's value from before the first completes.)
__device__ __forceinline__ uint32_t lds_code2w(uint32_t cm, uint32_t w0, uint32_t w1, uint32_t& r1) {
  uint32_t b0, b1, b2, b3, b4, b5, b6, b7, a0, a1, a2, a3, a4, a5, a6, a7;
#define CG_TC_ADDR(T, W, B) "v_add_u32_sdwa " T ", %16, " W " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" B "\n\t"
  asm volatile(CG_TC_ADDR("%8", "%17", "BYTE_0") CG_TC_ADDR("%9", "%17", "BYTE_1") CG_TC_ADDR("%10", "%17", "BYTE_2")
                   CG_TC_ADDR("%11", "%17", "BYTE_3") CG_TC_ADDR("%12", "%18", "BYTE_0")
                       CG_TC_ADDR("%13", "%18", "BYTE_1") CG_TC_ADDR("%14", "%18", "BYTE_2")
                           CG_TC_ADDR("%15", "%18", "BYTE_3")
               "ds_read_u8 %0, %8\n\t"
               "ds_read_u8 %1, %9\n\t"
               "ds_read_u8 %2, %10\n\t"
               "ds_read_u8 %3, %11\n\t"
               "ds_read_u8 %4, %12\n\t"
               "ds_read_u8 %5, %13\n\t"
               "ds_read_u8 %6, %14\n\t"
               "ds_read_u8 %7, %15\n\t"
               "s_waitcnt lgkmcnt(0)\n\t"
               "v_lshl_or_b32 %0, %1, 8, %0\n\t"
               "v_lshl_or_b32 %2, %3, 8, %2\n\t"
               "v_lshl_or_b32 %4, %5, 8, %4\n\t"
               "v_lshl_or_b32 %6, %7, 8, %6\n\t"
               "v_lshl_or_b32 %0, %2, 16, %0\n\t"
               "v_lshl_or_b32 %4, %6, 16, %4"
               : "=&v"(b0), "=&v"(b1), "=&v"(b2), "=&v"(b3), "=&v"(b4), "=&v"(b5), "=&v"(b6), "=&v"(b7),
                 "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(a4), "=&v"(a5), "=&v"(a6), "=&v"(a7)
               : "v"(cm), "v"(w0), "v"(w1));
#undef CG_TC_ADDR
  r1 = b4;
  return b0;
}
__device__ __forceinline__ uint4 lds_transcode(uint32_t cm, const uint4& u) {
  uint4 r;
  r.x = lds_code2w(cm, u.x, u.y, r.y);
  r.z = lds_code2w(cm, u.z, u.w, r.w);
  return r;
}

// Two independent walks (two requests of a lane) stepped together: both LDS
// reads are in flight before the one wait, so a wave's dependent chain costs
// one LDS round trip per TWO bytes walked.  Same VALU count as two single
// steps; the compare/select pairs share VCC in sequence (two wait states
// after each compare, filled by the default targets' max).
template <int B>
__device__ __forceinline__ void lds_cls_step2(uint32_t dead, uint32_t& sa, uint32_t wa, uint32_t& sb, uint32_t wb) {
  uint32_t ea, eb, da, db, na, nb;
#define CG_CLS_STEP2(b)                                                                                  \
  asm volatile("v_add_u32_sdwa %0, %6, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" b  \
               "\n\tv_add_u32_sdwa %1, %7, %9 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" b \
               "\n\tds_read_b32 %0, %0\n\t"                                                             \
               "ds_read_b32 %1, %1\n\t"                                                                  \
               "s_waitcnt lgkmcnt(0)\n\t"                                                                \
               "v_cmp_eq_u32_sdwa vcc, %0, %6 src0_sel:WORD_0 src1_sel:DWORD\n\t"                        \
               "v_max_u32 %2, %10, %6\n\t"                                                              \
               "v_max_u32 %3, %10, %7\n\t"                                                              \
               "v_cndmask_b32_sdwa %4, %2, %0, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "    \
               "src1_sel:WORD_1\n\t"                                                                    \
               "v_cmp_eq_u32_sdwa vcc, %1, %7 src0_sel:WORD_0 src1_sel:DWORD\n\t"                        \
               "s_nop 1\n\t"                                                                             \
               "v_cndmask_b32_sdwa %5, %3, %1, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "    \
               "src1_sel:WORD_1"                                                                          \
               : "=&v"(ea), "=&v"(eb), "=&v"(da), "=&v"(db), "=&v"(na), "=&v"(nb)                         \
               : "v"(sa), "v"(sb), "v"(wa), "v"(wb), "s"(dead)                                            \
               : "vcc")
  if (B == 0) CG_CLS_STEP2("BYTE_0");
  else if (B == 1) CG_CLS_STEP2("BYTE_1");
  else if (B == 2) CG_CLS_STEP2("BYTE_2");
  else CG_CLS_STEP2("BYTE_3");
#undef CG_CLS_STEP2
  sa = na;
  sb = nb;
}

template <int I>
__device__ __forceinline__ void lds_cls_step2x16(uint32_t dead, uint32_t& sa, const uint4& ua, uint32_t& sb,
                                                 const uint4& ub) {
  const uint32_t wa = I < 4 ? ua.x : I < 8 ? ua.y : I < 12 ? ua.z : ua.w;
  const uint32_t wb = I < 4 ? ub.x : I < 8 ? ub.y : I < 12 ? ub.z : ub.w;
  lds_cls_step2<I & 3>(dead, sa, wa, sb, wb);
}

// Where verdicts go: out[slot] (slot order), or — for a batch built on the
// device from raw requests (kernels_http_raw.hip) — out[order[slot]]
// (request order; padding slots, order 0xFFFFFFFF, write nothing).
// With `rule` set (cg_http_verdicts_rules_*), the request's first matching
// rule goes beside it: the per-rule counter index it adds to
// (HttpProg.rule_base + hit, cg_http_rule_info order) or 0xFFFFFFFF when no
// rule allows it — the access-log attribution of pkg/proxy/accesslog/
// record.go:36-47 and the policy trace of pkg/policy/policy.go:29-70.
struct VOut {
  uint8_t* __restrict__ out;
  const uint32_t* __restrict__ order;
  uint32_t* __restrict__ rule;
  uint32_t nout;  // requests (order entries past it write nothing)
  __device__ __forceinline__ void put(size_t slot, uint32_t v, uint32_t r_idx = 0xFFFFFFFFu) const {
    if (order) {
      const uint32_t r = order[slot];
      if (r < nout) {
        out[r] = (uint8_t)v;
        if (rule) rule[r] = r_idx;
      }
    } else {
      out[slot] = (uint8_t)v;
      if (rule) rule[slot] = r_idx;
    }
  }
};

// Records longer than a slot live in the overflow arena: byte loop.
template <bool kCls>
__device__ __forceinline__ uint32_t walk_arena(const uint32_t* __restrict__ cells, uint32_t dead, uint32_t st,
                                              const uint8_t* __restrict__ arena, uint32_t aoff, uint32_t len) {
  for (uint32_t p = 0; p < len && st != dead; ++p) st = step<kCls>(cells, dead, st, arena[aoff + p]);
  return st;
}

// A tile's meta block (8 bytes per lane: remote identity, overflow arena
// offset / 16 | flags << 24) and its string units (unit u ≥ 1 of lane l at
// units[(u - 1) * 64 + l]).
// `half`: the tile's last unit is a half unit (kTileHalfLast: 8 bytes per
// lane; its other 8 bytes read as zero padding).
struct TileRef {
  const uint2* meta;
  const uint4* units;
  bool half;
};
__device__ __forceinline__ TileRef tile_ref(const uint8_t* __restrict__ tiles, const HttpTile& tt) {
  const uint8_t* base = tiles + (size_t)tt.at * 512;
  return {reinterpret_cast<const uint2*>(base), reinterpret_cast<const uint4*>(base + kWave * CG_HTTP_META_BYTES),
          tile_half(tt)};
}

// String unit u (1-based) of a tile holding `units` whole units (the
// generic walker's tiles: cg_http_pack gives half last units only to
// one-part LDS programs, and http_chunks denies a half tile that reaches
// another walker); past them a lane re-reads the tile's last unit, or its
// meta block when it has none (bytes it never walks within its string) —
// never beyond the tile.
__device__ __forceinline__ uint4 tile_unit(const TileRef& tr, uint32_t units, uint32_t u, uint32_t lane) {
  if (units == 0) return reinterpret_cast<const uint4*>(tr.meta)[lane & 31];
  return tr.units[(min(u, units) - 1) * kWave + lane];
}

// Streaming loads for the one-part walkers: a tile's units and meta are read
// once, so they go nontemporal and leave L2 to the tile table, the program
// blocks and the arena (config 5, same box and run: 71.1 G/s against 68.5
// with plain loads, 70.2 with only the in-walk unit loads nontemporal).
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_nt __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  const u32x4_nt x = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(p));
  return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ uint2 ld_nt(const uint2* p) {
  const u32x2_nt x = __builtin_nontemporal_load(reinterpret_cast<const u32x2_nt*>(p));
  return make_uint2(x.x, x.y);
}
// unit k of lane l, nontemporal: 16 bytes, or 8 and zeros from a half unit
__device__ __forceinline__ uint4 ld_nt_unit(const TileRef& tr, uint32_t k, uint32_t l, bool half) {
  if (half) {
    const uint2 v = ld_nt(reinterpret_cast<const uint2*>(tr.units + k * kWave) + l);
    return make_uint4(v.x, v.y, 0u, 0u);
  }
  return ld_nt(tr.units + k * kWave + l);
}

// The overflow string of a lane whose meta word is m (arena entry: u32 length,
// bytes).  An entry reaching past the batch's arena (arena_bytes, from its
// header) ends in the dead state: the request is denied.
template <bool kCls>
__device__ __forceinline__ uint32_t walk_overflow(const uint32_t* __restrict__ cells, uint32_t dead, uint32_t st,
                                                 const uint8_t* __restrict__ arena, uint64_t arena_bytes, uint2 m,
                                                 bool ov) {
  if (!ov) return st;
  const uint64_t aoff = (uint64_t)(m.y & 0xFFFFFFu) * 16u;
  if (aoff + 4 > arena_bytes) return dead;
  const uint32_t len = *reinterpret_cast<const uint32_t*>(arena + aoff);
  if (aoff + 4 + len > arena_bytes) return dead;
  return walk_arena<kCls>(cells, dead, st, arena, (uint32_t)aoff + 4, len);
}

// The first-match hits of a wave's 64 requests (hit = rule bit, or kNoHit),
// called by the whole wave: lanes hold requests in the packer's string order,
// so equal hits come in runs; each run's first lane adds the run length —
// into the workgroup's LDS counters when the program's rules fit them, else
// into global memory.  One atomic per run instead of 64 same-address ones.
__device__ __forceinline__ void count_hits(const HttpDev& T, const HttpProg& pg, uint32_t hit, uint32_t* s_hits,
                                           uint32_t lane) {
  // the previous lane's hit: one DPP wave shift (lane 0 gets ~hit, a head)
  const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)~hit, (int)hit, 0x138 /* wave_shr:1 */, 0xF, 0xF,
                                                              false);
  const bool head = prev != hit;
  const unsigned long long heads = __ballot(head);
  if (head && hit != kNoHit) {
    const unsigned long long later = heads >> lane >> 1;  // heads of the runs after this one
    const uint32_t len = later ? (uint32_t)__builtin_ctzll(later) + 1u : 64u - lane;
    if (s_hits && pg.nrules <= kLdsRuleHits) atomicAdd(&s_hits[hit], len);
    else atomicAdd(&T.rule_hits[pg.rule_base + hit], (unsigned long long)len);
  }
}

// K tiles of a program (tile j takes part only if valid[j]): walk every
// part, OR the verdicts.  blk = the program's block (LDS copy or global);
// parts walk blk when rebased, else their own cells in T.cells.  Each lane
// walks K independent strings, interleaved byte by byte, so one lane's LDS
// reads overlap; units load one ahead and the walk ends once no lane is
// alive inside its string.
// Raw-byte batches on this path (programs walked from global memory): the
// class codes of a unit from the program's map in global memory.
__device__ __forceinline__ uint4 glb_transcode(const uint8_t* __restrict__ m, const uint4& u) {
  auto w = [&](uint32_t x) {
    return (uint32_t)m[x & 255] | (uint32_t)m[(x >> 8) & 255] << 8 | (uint32_t)m[(x >> 16) & 255] << 16 |
           (uint32_t)m[x >> 24] << 24;
  };
  return make_uint4(w(u.x), w(u.y), w(u.z), w(u.w));
}

template <int K>
__device__ __forceinline__ void http_tiles(const HttpDev& T, const HttpProg& pg, uint32_t prog,
                                           const uint32_t* __restrict__ blk, bool rebased,
                                           const uint8_t* __restrict__ tiles, const HttpTile* __restrict__ ttab,
                                           const uint32_t (&tile)[K],
                                           const bool (&valid)[K], const uint8_t* __restrict__ arena,
                                           uint64_t arena_bytes, VOut out, uint32_t lane, uint32_t& n_allow,
                                           uint32_t& n_deny, uint32_t* s_hits, const uint8_t* __restrict__ codes) {
  TileRef tr[K];
  uint2 meta[K];
  uint32_t row[K];
  uint32_t units = 0, tu[K];  // string units: of the K tiles (the longest, wave-uniform), of each
  bool counted[K], overflow[K];
  uint32_t hit[K];
  bool any_overflow = false;
  const uint32_t W = pg.mask_words;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const HttpTile tt = ttab[tile[j]];
    tr[j] = tile_ref(tiles, tt);
    // (a half last unit never reaches this walker from cg_http_pack: such a
    // tile is denied unwalked, its units never read as whole ones)
    const bool half = tile_half(tt);
    tu[j] = valid[j] && !half ? tile_units(tt) : 0u;
    units = max(units, tu[j]);
    meta[j] = tr[j].meta[lane];
    const uint32_t flags = meta[j].y >> 24;
    counted[j] = valid[j] && !half && !(flags & (CG_HTTP_F_PAD | CG_HTTP_F_MALFORMED));
    overflow[j] = counted[j] && (flags & CG_HTTP_F_OVERFLOW);
    any_overflow |= overflow[j];
    row[j] = remote_row(blk, pg, meta[j].x);
    hit[j] = kNoHit;
  }
  any_overflow = __any(any_overflow);
  for (uint32_t pi = 0; pi < pg.part_count; ++pi) {
    const HttpPart pt = T.parts[pg.part_begin + pi];
    const bool cls = pt.mode == kPartClass;  // uniform
    const uint32_t* __restrict__ cells = rebased ? blk : T.cells + pt.walk_off;
    uint32_t st[K];
#pragma unroll
    for (int j = 0; j < K; ++j) st[j] = pt.start;
    if (units) {
      // a tile stores tu[j] string units; past them (K > 1) a lane re-reads
      // its tile's last unit, which cannot change its verdict
      uint4 cur[K];
#pragma unroll
      for (int j = 0; j < K; ++j) cur[j] = tile_unit(tr[j], tu[j], 1, lane);
      for (uint32_t u = 0; u < units; ++u) {
        const bool more = u + 1 < units;
        uint4 nxt[K];
#pragma unroll
        for (int j = 0; j < K; ++j) nxt[j] = cur[j];
        if (more) {
#pragma unroll
          for (int j = 0; j < K; ++j) nxt[j] = tile_unit(tr[j], tu[j], u + 2, lane);
        }
        if (cls) {
          if (codes) {  // uniform: a raw-byte batch
#pragma unroll
            for (int j = 0; j < K; ++j) cur[j] = glb_transcode(codes + (size_t)prog * 256, cur[j]);
          }
#pragma unroll
          for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int j = 0; j < K; ++j) st[j] = comb_step_cls(cells, pt.dead, st[j], get_byte(cur[j], k));
          }
        } else {
#pragma unroll
          for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int j = 0; j < K; ++j) st[j] = comb_step(cells, pt.dead, st[j], get_byte(cur[j], k));
          }
        }
        bool alive = false;
#pragma unroll
        for (int j = 0; j < K; ++j) alive |= st[j] != pt.dead;
        if (!more || !__any(alive)) break;
#pragma unroll
        for (int j = 0; j < K; ++j) cur[j] = nxt[j];
      }
    }
    if (any_overflow) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint32_t sa =
            cls ? walk_overflow<true>(cells, pt.dead, pt.start, arena, arena_bytes, meta[j], overflow[j])
                : walk_overflow<false>(cells, pt.dead, pt.start, arena, arena_bytes, meta[j], overflow[j]);
        if (overflow[j]) st[j] = sa;
      }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t lab =
          counted[j] ? (cls ? state_label<true>(cells, st[j]) : state_label<false>(cells, st[j])) : 0xFFFFu;
      if (lab != 0xFFFFu) hit[j] = min(hit[j], first_meet(blk, pt.acc_off + lab * 2 * W, row[j], W));
    }
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (counted[j] && (pg.flags & kProgHasAlways)) hit[j] = min(hit[j], first_meet(blk, pg.always_off, row[j], W));
    const bool verdict = counted[j] && hit[j] != kNoHit;
    count_hits(T, pg, verdict ? hit[j] : kNoHit, s_hits, lane);
    if (valid[j]) out.put((size_t)tile[j] * kWave + lane, verdict, verdict ? pg.rule_base + hit[j] : kNoHit);
    n_allow += counted[j] && verdict;
    n_deny += counted[j] && !verdict;
  }
}

// The first string units of a wave's NEXT tile (and its meta block), loaded
// while the current tile walks: the walk is VALU-bound and a tile's loads
// would otherwise be waited for at its start, so each wave keeps the next
// tile's head in flight under the current walk.  kPre units (4 VGPRs each)
// bound the registers this costs at 8 waves per SIMD.
constexpr int kPre = 1;
#define NT_META(p) ld_nt(p)
#define NT_PRE(p) ld_nt(p)
struct TilePre {
  uint2 meta;
  uint4 u[kPre];
};
// The lane index recomputed where a tile address needs it (volatile: not
// CSE'd with the kernel's copy, which the register allocator otherwise
// spills at 64 VGPRs and reloads per tile — a scratch load that made the
// next tile's prefetch wait for this tile's unit loads).
__device__ __forceinline__ uint32_t lane_now() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

__device__ __forceinline__ void tile_prefetch(const TileRef& tr, uint32_t units, uint32_t, TilePre& p) {
  const uint32_t lane = lane_now();
  p.meta = NT_META(tr.meta + lane);
#pragma unroll
  for (int k = 0; k < kPre; ++k) {  // stays inside the tile (see tile_unit)
    const uint32_t kk = min(k + 1u, units) - 1;
    if (units == 0) p.u[k] = NT_PRE(reinterpret_cast<const uint4*>(tr.meta) + (lane & 31));
    else p.u[k] = ld_nt_unit(tr, kk, lane, tr.half && kk + 1 == units);
  }
}

// One tile of a one-part program whose block `blk` is in LDS, its string
// units count N known up front (tile table): straight-line code.  The tile's
// meta and first kPre units arrive prefetched (cur); the rest load at its
// start, then the next tile's head is issued (has_next) — so a wave pays a
// memory latency only for a tile's later units, which the walk of its first
// ones covers.  The remote-identity lookup reads the LDS block after the
// walk, only for lanes that reached an accepting state.  No early exit:
// lanes whose string ended (or died) keep stepping through zero padding or
// the dead state, which cannot change their verdict.
template <int N, bool kCls, bool kRaw, bool kHalf>
__device__ __forceinline__ void http_tile_n(const HttpDev& T, const HttpProg& pg, const HttpPart& pt,
                                            uint32_t prog, const uint32_t* __restrict__ blk, const TileRef tr,
                                            const TilePre& cur, bool has_next, const TileRef trn, uint32_t nunits,
                                            uint32_t tail, TilePre& nxt, uint32_t t, const uint8_t* __restrict__ arena,
                                            uint64_t arena_bytes, VOut out, uint32_t lane,
                                            uint32_t& n_allow, uint32_t& n_deny, uint32_t* s_hits, uint32_t cm) {
  const uint2 meta = cur.meta;
  // a rolling window of kWin units: unit k + kWin loads when unit k starts
  // walking (16 dependent steps cover its latency), so long tiles hold
  // kWin units in registers, not N
  constexpr int kWin = N < 4 ? (N > 0 ? N : 1) : 4;
  uint4 unit[kWin];
#pragma unroll
  for (int k = 0; k < kWin && k < N; ++k)
    unit[k] = k < kPre ? cur.u[k < kPre ? k : 0] : ld_nt_unit(tr, k, lane_now(), kHalf && k == N - 1);
  if (has_next) tile_prefetch(trn, nunits, lane, nxt);
  __builtin_amdgcn_sched_barrier(0);
  const uint32_t flags = meta.y >> 24;
  const bool counted = !(flags & (CG_HTTP_F_PAD | CG_HTTP_F_MALFORMED));
  const bool overflow = counted && (flags & CG_HTTP_F_OVERFLOW);
  const uint32_t dead = pt.dead;
  uint32_t st = pt.start;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    // raw-byte batches: the unit's bytes through the code map (class mode)
    const uint4 u = kRaw && kCls ? lds_transcode(cm, unit[k % kWin]) : unit[k % kWin];
    if (k + kWin < N) unit[k % kWin] = ld_nt_unit(tr, k + kWin, lane_now(), kHalf && k + kWin == N - 1);
    // the last unit: only the 4-byte groups holding some lane's string
    // (tail, wave-uniform), the rest is padding
    const bool last = k == N - 1;
    if (kCls) {
      st = lds_cls_step16<0>(dead, st, u);
      st = lds_cls_step16<1>(dead, st, u);
      st = lds_cls_step16<2>(dead, st, u);
      st = lds_cls_step16<3>(dead, st, u);
      if (!last || tail > 4) {
        st = lds_cls_step16<4>(dead, st, u);
        st = lds_cls_step16<5>(dead, st, u);
        st = lds_cls_step16<6>(dead, st, u);
        st = lds_cls_step16<7>(dead, st, u);
      }
      if (!last || tail > 8) {
        st = lds_cls_step16<8>(dead, st, u);
        st = lds_cls_step16<9>(dead, st, u);
        st = lds_cls_step16<10>(dead, st, u);
        st = lds_cls_step16<11>(dead, st, u);
      }
      if (!last || tail > 12) {
        st = lds_cls_step16<12>(dead, st, u);
        st = lds_cls_step16<13>(dead, st, u);
        st = lds_cls_step16<14>(dead, st, u);
        st = lds_cls_step16<15>(dead, st, u);
      }
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (last && g > 0 && tail <= 4u * g) break;
#pragma unroll
        for (int i = 4 * g; i < 4 * g + 4; ++i) st = step<kCls>(blk, dead, st, get_byte(u, i));
      }
    }
  }
  if (__any(overflow)) {
    const uint32_t sa = walk_overflow<kCls>(blk, dead, pt.start, arena, arena_bytes, meta, overflow);
    if (overflow) st = sa;
  }
  uint32_t hit = kNoHit;
  if (counted) {
    const uint32_t lab = state_label<kCls>(blk, st);
    const bool always = pg.flags & kProgHasAlways;
    if (lab != 0xFFFFu || always) {
      const uint32_t row = remote_row(blk, pg, meta.x);
      if (lab != 0xFFFFu) hit = first_meet(blk, pt.acc_off + mul24(lab, 2 * pg.mask_words), row, pg.mask_words);
      if (always) hit = min(hit, first_meet(blk, pg.always_off, row, pg.mask_words));
    }
  }
  const bool verdict = hit != kNoHit;
  count_hits(T, pg, hit, s_hits, lane);
  out.put((size_t)t * kWave + lane, verdict, verdict ? pg.rule_base + hit : kNoHit);
  n_allow += counted && verdict;
  n_deny += counted && !verdict;
}

// ---- two tiles per wave, one request of each per lane (kPairTiles) --------
// A lane walks the requests of tiles ta and tb together (lds_cls_step2): two
// LDS reads in flight per wait.  The pair is walked over N = the longer
// tile's string units; a lane of the shorter tile re-reads its tile's last
// unit past its end (tile_unit), which cannot change its verdict.
// Off: measured at 8 waves per SIMD (64 VGPRs) it spills and loses (§3.1);
// kept for a 4-waves-per-SIMD build (kHttpWaves = 4), where the second
// chain stands in for the halved occupancy.
constexpr bool kPairTiles = false;

__device__ __forceinline__ uint4 pair_unit(const TileRef& tr, uint32_t units, uint32_t k) {
  const uint32_t lane = lane_now();
  if (units == 0) return ld_nt(reinterpret_cast<const uint4*>(tr.meta) + (lane & 31));
  const uint32_t kk = min(k + 1u, units) - 1u;
  return ld_nt_unit(tr, kk, lane, tr.half && kk + 1 == units);
}

// The verdict of one lane's request after the walk (as http_tile_n's).
__device__ __forceinline__ void pair_verdict(const HttpDev& T, const HttpProg& pg, const HttpPart& pt,
                                             const uint32_t* __restrict__ blk, uint2 meta, uint32_t st,
                                             const uint8_t* __restrict__ arena, uint64_t arena_bytes, uint32_t t,
                                             VOut out, uint32_t lane, uint32_t& n_allow, uint32_t& n_deny,
                                             uint32_t* s_hits) {
  const uint32_t flags = meta.y >> 24;
  const bool counted = !(flags & (CG_HTTP_F_PAD | CG_HTTP_F_MALFORMED));
  const bool overflow = counted && (flags & CG_HTTP_F_OVERFLOW);
  if (__any(overflow)) {
    const uint32_t sa = walk_overflow<true>(blk, pt.dead, pt.start, arena, arena_bytes, meta, overflow);
    if (overflow) st = sa;
  }
  uint32_t hit = kNoHit;
  if (counted) {
    const uint32_t lab = state_label<true>(blk, st);
    const bool always = pg.flags & kProgHasAlways;
    if (lab != 0xFFFFu || always) {
      const uint32_t row = remote_row(blk, pg, meta.x);
      if (lab != 0xFFFFu) hit = first_meet(blk, pt.acc_off + mul24(lab, 2 * pg.mask_words), row, pg.mask_words);
      if (always) hit = min(hit, first_meet(blk, pg.always_off, row, pg.mask_words));
    }
  }
  const bool verdict = hit != kNoHit;
  count_hits(T, pg, hit, s_hits, lane);
  out.put((size_t)t * kWave + lane, verdict, verdict ? pg.rule_base + hit : kNoHit);
  n_allow += counted && verdict;
  n_deny += counted && !verdict;
}

template <int N, bool kRaw>
__device__ __forceinline__ void http_pair_n(const HttpDev& T, const HttpProg& pg, const HttpPart& pt,
                                            const uint32_t* __restrict__ blk, const TileRef ra, const TileRef rb,
                                            uint32_t ua, uint32_t ub, const TilePre& ca, const TilePre& cb,
                                            bool has_next, bool next_pair, const TileRef rna, const TileRef rnb,
                                            uint32_t nua, uint32_t nub, TilePre& xa, TilePre& xb, uint32_t tail,
                                            uint32_t ta, uint32_t tb, const uint8_t* __restrict__ arena,
                                            uint64_t arena_bytes, VOut out, uint32_t lane, uint32_t& n_allow,
                                            uint32_t& n_deny, uint32_t* s_hits, uint32_t cm) {
  // a rolling window of kW units per chain: unit k + kW loads when unit k
  // starts walking
  constexpr int kW = N < 2 ? (N > 0 ? N : 1) : 2;
  uint4 wa[kW], wb[kW];
#pragma unroll
  for (int k = 0; k < kW && k < N; ++k) {
    wa[k] = k == 0 ? ca.u[0] : (pair_unit(ra, ua, k));
    wb[k] = k == 0 ? cb.u[0] : (pair_unit(rb, ub, k));
  }
  if (has_next) {
    tile_prefetch(rna, nua, lane, xa);
    if (next_pair) tile_prefetch(rnb, nub, lane, xb);
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint32_t dead = pt.dead;
  uint32_t sa = pt.start, sb = pt.start;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint4 a = kRaw ? lds_transcode(cm, wa[k % kW]) : wa[k % kW];
    const uint4 b = kRaw ? lds_transcode(cm, wb[k % kW]) : wb[k % kW];
    if (k + kW < N) {
      wa[k % kW] = (pair_unit(ra, ua, k + kW));
      wb[k % kW] = (pair_unit(rb, ub, k + kW));
    }
    const bool last = k == N - 1;
    lds_cls_step2x16<0>(dead, sa, a, sb, b);
    lds_cls_step2x16<1>(dead, sa, a, sb, b);
    lds_cls_step2x16<2>(dead, sa, a, sb, b);
    lds_cls_step2x16<3>(dead, sa, a, sb, b);
    if (!last || tail > 4) {
      lds_cls_step2x16<4>(dead, sa, a, sb, b);
      lds_cls_step2x16<5>(dead, sa, a, sb, b);
      lds_cls_step2x16<6>(dead, sa, a, sb, b);
      lds_cls_step2x16<7>(dead, sa, a, sb, b);
    }
    if (!last || tail > 8) {
      lds_cls_step2x16<8>(dead, sa, a, sb, b);
      lds_cls_step2x16<9>(dead, sa, a, sb, b);
      lds_cls_step2x16<10>(dead, sa, a, sb, b);
      lds_cls_step2x16<11>(dead, sa, a, sb, b);
    }
    if (!last || tail > 12) {
      lds_cls_step2x16<12>(dead, sa, a, sb, b);
      lds_cls_step2x16<13>(dead, sa, a, sb, b);
      lds_cls_step2x16<14>(dead, sa, a, sb, b);
      lds_cls_step2x16<15>(dead, sa, a, sb, b);
    }
  }
  pair_verdict(T, pg, pt, blk, ca.meta, sa, arena, arena_bytes, ta, out, lane, n_allow, n_deny, s_hits);
  pair_verdict(T, pg, pt, blk, cb.meta, sb, arena, arena_bytes, tb, out, lane, n_allow, n_deny, s_hits);
}

template <int N, bool kCls, bool kRaw>
__device__ __forceinline__ void http_tile_n(const HttpDev& T, const HttpProg& pg, const HttpPart& pt,
                                            uint32_t prog, const uint32_t* __restrict__ blk, const TileRef tr,
                                            const TilePre& cur, bool has_next, const TileRef trn, uint32_t nunits,
                                            uint32_t tail, TilePre& nxt, uint32_t t, const uint8_t* __restrict__ arena,
                                            uint64_t arena_bytes, VOut out, uint32_t lane,
                                            uint32_t& n_allow, uint32_t& n_deny, uint32_t* s_hits, uint32_t cm);

// A wave's tiles of a class-mode one-part program in pairs (t, t + nw), then
// (t + 2nw, t + 3nw), ...; a last lone tile goes through http_tile_n.
template <bool kRaw>
__device__ __forceinline__ void one_part_pairs(const HttpDev& T, const HttpProg& pg, const HttpPart& pt, uint32_t prog,
                                               const uint32_t* __restrict__ lcells, const uint8_t* __restrict__ tiles,
                                               const HttpTile* __restrict__ ttab, uint32_t t, uint32_t tend,
                                               uint32_t nw, const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                               VOut out, uint32_t lane, uint32_t& n_allow, uint32_t& n_deny,
                                               uint32_t* s_hits, uint32_t cm) {
  HttpTile ta = ttab[t];
  HttpTile tb = ttab[t + nw < tend ? t + nw : t];
  TileRef ra = tile_ref(tiles, ta), rb = tile_ref(tiles, tb);
  TilePre pa, pb;
  tile_prefetch(ra, tile_units(ta), lane, pa);
  tile_prefetch(rb, tile_units(tb), lane, pb);
  for (; t < tend; t += 2 * nw) {
    const uint32_t tn = t + 2 * nw;
    const bool has_next = tn < tend, next_pair = tn + nw < tend;
    const HttpTile tna = ttab[has_next ? tn : t], tnb = ttab[next_pair ? tn + nw : (has_next ? tn : t)];
    const TileRef rna = tile_ref(tiles, tna), rnb = tile_ref(tiles, tnb);
    TilePre xa = pa, xb = pb;
    if (t + nw >= tend) {  // a lone last tile (wave-uniform)
      switch (tile_units(ta)) {
#define CG_TILE_1(n)                                                                                               \
  case n:                                                                                                          \
    if (!kRaw && tile_half(ta))                                                                                    \
      http_tile_n<n, true, kRaw, true>(T, pg, pt, prog, lcells, ra, pa, false, ra, 0, tile_tail(ta), xa, t, arena,  \
                                       arena_bytes, out, lane, n_allow, n_deny, s_hits, cm);                      \
    else                                                                                                           \
      http_tile_n<n, true, kRaw, false>(T, pg, pt, prog, lcells, ra, pa, false, ra, 0, tile_tail(ta), xa, t, arena, \
                                        arena_bytes, out, lane, n_allow, n_deny, s_hits, cm);                     \
    break;
        CG_TILE_1(0) CG_TILE_1(1) CG_TILE_1(2) CG_TILE_1(3) CG_TILE_1(4) CG_TILE_1(5) CG_TILE_1(6) CG_TILE_1(7)
        default: CG_TILE_1(8)
#undef CG_TILE_1
      }
      break;
    }
    const uint32_t ua = tile_units(ta), ub = tile_units(tb), n = max(ua, ub);
    // the last unit's 4-byte groups holding a string byte of a tile that
    // reaches it (a shorter tile re-reads an earlier unit there: skippable)
    const uint32_t tail = max(ua == n ? tile_tail(ta) : 0u, ub == n ? tile_tail(tb) : 0u);
    switch (n) {  // wave-uniform
#define CG_PAIR_N(k)                                                                                              \
  case k:                                                                                                         \
    http_pair_n<k, kRaw>(T, pg, pt, lcells, ra, rb, ua, ub, pa, pb, has_next, next_pair, rna, rnb,              \
                         tile_units(tna), tile_units(tnb), xa, xb, tail, t, t + nw, arena, arena_bytes, out, lane, \
                         n_allow, n_deny, s_hits, cm);                                                            \
    break;
      CG_PAIR_N(0) CG_PAIR_N(1) CG_PAIR_N(2) CG_PAIR_N(3) CG_PAIR_N(4) CG_PAIR_N(5) CG_PAIR_N(6) CG_PAIR_N(7)
      default:
        http_pair_n<8, kRaw>(T, pg, pt, lcells, ra, rb, ua, ub, pa, pb, has_next, next_pair, rna, rnb,
                             tile_units(tna), tile_units(tnb), xa, xb, tail, t, t + nw, arena, arena_bytes, out, lane,
                             n_allow, n_deny, s_hits, cm);
#undef CG_PAIR_N
    }
    ta = tna;
    tb = tnb;
    ra = rna;
    rb = rnb;
    pa = xa;
    pb = xb;
  }
}

// A wave's tiles t, t + nw, ... < tend of a one-part program whose block is
// in LDS: each tile's walk specialized on its string units (wave-uniform).
template <bool kCls, bool kRaw>
__device__ __forceinline__ void one_part_tiles(const HttpDev& T, const HttpProg& pg, const HttpPart& pt, uint32_t prog,
                                               const uint32_t* __restrict__ lcells, const uint8_t* __restrict__ tiles,
                                               const HttpTile* __restrict__ ttab, uint32_t t, uint32_t tend,
                                               uint32_t nw, const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                               VOut out, uint32_t lane, uint32_t& n_allow,
                                               uint32_t& n_deny, uint32_t* s_hits, uint32_t cm) {
  if (t >= tend) return;
  if (kPairTiles && kCls) {
    one_part_pairs<kRaw>(T, pg, pt, prog, lcells, tiles, ttab, t, tend, nw, arena, arena_bytes, out, lane, n_allow,
                         n_deny, s_hits, cm);
    return;
  }
  HttpTile tt = ttab[t];
  TileRef tb = tile_ref(tiles, tt);
  TilePre pre;
  tile_prefetch(tb, tile_units(tt), lane, pre);
  for (; t < tend; t += nw) {
    const bool has_next = t + nw < tend;
    const HttpTile ttn = ttab[has_next ? t + nw : t];
    const TileRef tbn = tile_ref(tiles, ttn);
    TilePre nxt = pre;
    switch (tile_units(tt)) {  // wave-uniform
#define CG_TILE_N(n)                                                                                                \
  case n:                                                                                                           \
    if (!kRaw && n > 0 && tile_half(tt))                                                                            \
      http_tile_n<n, kCls, kRaw, true>(T, pg, pt, prog, lcells, tb, pre, has_next, tbn, tile_units(ttn), tile_tail(tt), \
                                       nxt, t, arena, arena_bytes, out, lane, n_allow, n_deny, s_hits, cm);          \
    else                                                                                                            \
      http_tile_n<n, kCls, kRaw, false>(T, pg, pt, prog, lcells, tb, pre, has_next, tbn, tile_units(ttn), tile_tail(tt), \
                                        nxt, t, arena, arena_bytes, out, lane, n_allow, n_deny, s_hits, cm);         \
    break;
      CG_TILE_N(0) CG_TILE_N(1) CG_TILE_N(2) CG_TILE_N(3) CG_TILE_N(4) CG_TILE_N(5) CG_TILE_N(6) CG_TILE_N(7)
      default: CG_TILE_N(8)
#undef CG_TILE_N
    }
    tt = ttn;
    tb = tbn;
    pre = nxt;
  }
}

// End of a workgroup's run of chunks of program `prog`: wave totals are
// summed in LDS, then one thread adds them to the global counters, and the
// program's LDS rule-hit counters go to global memory (and are cleared).
// Ends with every wave past a barrier, so the caller may restage lcells.
__device__ __forceinline__ void flush_counts(const HttpDev& T, uint32_t prog, uint32_t& n_allow, uint32_t& n_deny,
                                             uint32_t lane, uint32_t* s_cnt, uint32_t* s_hits) {
  const bool real = prog < T.nprogs;  // uniform
  if (real) {
    for (int o = 32; o > 0; o >>= 1) {
      n_allow += __shfl_down(n_allow, o, kWave);
      n_deny += __shfl_down(n_deny, o, kWave);
    }
    if (lane == 0) {
      atomicAdd(&s_cnt[0], n_allow);
      atomicAdd(&s_cnt[1], n_deny);
    }
  }
  n_allow = n_deny = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (real && s_cnt[0]) atomicAdd(&T.counters[2 * prog], (unsigned long long)s_cnt[0]);
    if (real && s_cnt[1]) atomicAdd(&T.counters[2 * prog + 1], (unsigned long long)s_cnt[1]);
    s_cnt[0] = s_cnt[1] = 0;
  }
  if (real && s_hits) {
    const uint32_t base = T.progs[prog].rule_base, nr = T.progs[prog].nrules;
    if (nr <= kLdsRuleHits)
      for (uint32_t i = threadIdx.x; i < nr; i += blockDim.x) {
        const uint32_t c = s_hits[i];
        if (c) {
          atomicAdd(&T.rule_hits[base + i], (unsigned long long)c);
          s_hits[i] = 0;
        }
      }
  }
}

// Workgroups take chunks round-robin.  kGlobal = false: chunks of trivial
// programs and of programs whose block fits the workgroup's LDS share, which
// is staged when the program changes; kGlobal = true: the remaining chunks
// (programs too large for LDS), walked from global memory — a separate kernel
// so the rare path does not set the common one's register budget.
// kRaw: the batch's strings are raw bytes (device-layout raw batches), coded
// through `codes` (per program 256 bytes) as they walk: a class-mode
// program's map is staged in LDS after its block, at byte address cm.
template <bool kGlobal, bool kRaw>
__device__ __forceinline__ void http_chunks(const HttpDev& T, const uint8_t* __restrict__ batch, size_t nslots,
                                            const uint8_t* __restrict__ arena, VOut out,
                                            uint32_t* lcells, uint32_t* s_cnt, uint32_t* s_hits,
                                            uint32_t* __restrict__ deal, const uint8_t* __restrict__ codes) {
  const HttpBatchHeader* H = reinterpret_cast<const HttpBatchHeader*>(batch);
  const uint32_t magic = H->magic, epoch = H->epoch, nchunks = H->nchunks, ntiles = H->ntiles;
  const uint64_t toff = H->tiles_off, arena_bytes = H->arena_bytes;
  if (magic != kBatchMagic || epoch != T.epoch || (size_t)ntiles * kWave > nslots) {
    // packed against another snapshot (or not a batch): deny every slot
    if (kGlobal) return;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (size_t)gridDim.x * blockDim.x)
      out.put(i, 0);
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&T.counters[2 * T.nprogs], 1ULL);
    return;
  }
  const HttpChunk* chunks = reinterpret_cast<const HttpChunk*>(batch + sizeof(HttpBatchHeader));
  const HttpTile* ttab = reinterpret_cast<const HttpTile*>(batch + H->ttab_off);
  const uint8_t* tiles = batch + toff;
  // wave index made wave-uniform (SGPR): tile addresses then live in scalar
  // registers and each load needs only its lane offset in a VGPR
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                 nw = blockDim.x >> 6;
  // Chunks are dealt round-robin: a contiguous run per workgroup would pin
  // each workgroup to one program and the costliest program sets the tail.
  // Allowed/denied counts stay in registers while consecutive chunks share a
  // program and go to the global counters once per run (one atomic pair per
  // workgroup): concurrent workgroups work on the same program, so per-wave
  // atomics would all hit the same two addresses.
  uint32_t cur = kProgDeny;  // program of the current run (its block is in LDS if walked there)
  uint32_t n_allow = 0, n_deny = 0;
  // dealt in runs of kDealRun consecutive chunks (same program, mostly), so
  // the block is restaged once per run; dynamic: a run per ticket
  // the ticket lives in the dynamic LDS (s_cnt[2]): a static __shared__
  // variable would move the program block off LDS address 0
  uint32_t& s_ticket = s_cnt[2];
  uint32_t cr = blockIdx.x * kDealRun;
  if (kDynamicDeal && deal) {
    if (threadIdx.x == 0) s_ticket = atomicAdd(&deal[0], 1u);
    __syncthreads();
    cr = s_ticket * kDealRun;
  }
  for (; cr < nchunks;) {
  for (uint32_t c = cr; c < min(nchunks, cr + kDealRun); ++c) {
    const HttpChunk ch = chunks[c];
    if (ch.first_tile + ch.ntiles > ntiles || ch.ntiles > kChunkTiles) continue;  // malformed chunk
    const uint32_t prog = ch.prog;
    const bool real = prog < T.nprogs;
    HttpProg pg{};
    if (real) pg = T.progs[prog];
    const bool walkp = real && !(pg.flags & kProgAllowAll);
    const bool lds = walkp && (pg.flags & kProgRebased) && pg.cell_count <= T.lds_cells;
    if (kGlobal != (walkp && !lds)) continue;  // the other kernel's chunk
    if (prog != cur) {  // uniform across the workgroup: same chunk sequence
      flush_counts(T, cur, n_allow, n_deny, lane, s_cnt, s_hits);
      if (lds)
        for (uint32_t i = threadIdx.x; i < pg.cell_count; i += blockDim.x) lcells[i] = T.cells[pg.cell_begin + i];
      if (kRaw && lds && (pg.flags & kProgClass) && threadIdx.x < 64)
        lcells[T.lds_cells + threadIdx.x] = reinterpret_cast<const uint32_t*>(codes + (size_t)prog * 256)[threadIdx.x];
      __syncthreads();
      cur = prog;
    }
    const uint32_t tend = ch.first_tile + ch.ntiles;
    if (!walkp) {
      for (uint32_t t = ch.first_tile + wave; t < tend; t += nw) {
        // no policy for the port → allow; unknown policy → deny; a scope
        // without HTTP rules → allow (cilium_network_policy.h:129-138,187-191)
        const uint32_t flags = tile_ref(tiles, ttab[t]).meta[lane].y >> 24;
        const bool counted = !(flags & (CG_HTTP_F_PAD | CG_HTTP_F_MALFORMED));
        out.put((size_t)t * kWave + lane, counted && (prog == kProgAllow || real) ? 1u : 0u);
        n_allow += real && counted;
      }
    } else if (kGlobal) {
      const bool rebased = pg.flags & kProgRebased;
      for (uint32_t t = ch.first_tile + wave; t < tend; t += nw) {
        const uint32_t tile[1] = {t};
        const bool valid[1] = {true};
        http_tiles<1>(T, pg, prog, T.cells + pg.cell_begin, rebased, tiles, ttab, tile, valid, arena, arena_bytes, out, lane,
                      n_allow, n_deny, s_hits, kRaw ? codes : nullptr);
      }
    } else if (pg.part_count == 1) {
      const HttpPart pt = T.parts[pg.part_begin];
      if (pt.mode == kPartClass)
        one_part_tiles<true, kRaw>(T, pg, pt, prog, lcells, tiles, ttab, ch.first_tile + wave, tend, nw, arena,
                                   arena_bytes, out, lane, n_allow, n_deny, s_hits, T.lds_cells * 4);
      else
        one_part_tiles<false, kRaw>(T, pg, pt, prog, lcells, tiles, ttab, ch.first_tile + wave, tend, nw, arena,
                                    arena_bytes, out, lane, n_allow, n_deny, s_hits, 0u);
    } else {
      // each wave takes kTilesPerWave tiles at a time (wave, wave + nw, ...)
      for (uint32_t t0 = ch.first_tile + wave; t0 < tend; t0 += kTilesPerWave * nw) {
        uint32_t tile[kTilesPerWave];
        bool valid[kTilesPerWave];
#pragma unroll
        for (int j = 0; j < kTilesPerWave; ++j) {
          const uint32_t t = t0 + j * nw;
          valid[j] = t < tend;
          tile[j] = valid[j] ? t : t0;
        }
        http_tiles<kTilesPerWave>(T, pg, prog, lcells, true, tiles, ttab, tile, valid, arena, arena_bytes, out, lane,
                                  n_allow, n_deny, s_hits, kRaw ? codes : nullptr);
      }
    }
  }
    if (kDynamicDeal && deal) {
      __syncthreads();  // every wave has read s_ticket
      if (threadIdx.x == 0) s_ticket = atomicAdd(&deal[0], 1u);
      __syncthreads();
      cr = s_ticket * kDealRun;
    } else {
      cr += gridDim.x * kDealRun;
    }
  }
  flush_counts(T, cur, n_allow, n_deny, lane, s_cnt, s_hits);
}

template <bool kRaw>
__global__ __launch_bounds__(kHttpThreads) __attribute__((amdgpu_waves_per_eu(kHttpWaves, kHttpWaves))) void http_kernel(
    HttpDev T, const uint8_t* __restrict__ batch, size_t nslots, const uint8_t* __restrict__ arena,
    uint8_t* __restrict__ out, const uint32_t* __restrict__ order, uint32_t* __restrict__ deal,
    uint32_t* __restrict__ rule, uint32_t nout, const uint8_t* __restrict__ codes) {
  // dynamic LDS only, so the program block starts at LDS address 0 (a
  // class-mode step's address is then just state + code): [block:
  // T.lds_cells][code map: 64 words, kRaw][rule hits: kLdsRuleHits][allowed, denied, deal ticket]
  extern __shared__ __attribute__((aligned(16))) uint32_t lcells[];
  uint32_t* s_hits = lcells + T.lds_cells + (kRaw ? 64 : 0);
  uint32_t* s_cnt = s_hits + kLdsRuleHits;
  for (uint32_t i = threadIdx.x; i < kLdsRuleHits; i += blockDim.x) s_hits[i] = 0;
  if (threadIdx.x == 0) s_cnt[0] = s_cnt[1] = 0;
  __syncthreads();
  http_chunks<false, kRaw>(T, batch, nslots, arena, VOut{out, order, rule, nout}, lcells, s_cnt, s_hits, deal, codes);
}

template <bool kRaw>
__global__ __launch_bounds__(kHttpThreads) void http_kernel_global(HttpDev T, const uint8_t* __restrict__ batch,
                                                                   size_t nslots, const uint8_t* __restrict__ arena,
                                                                   uint8_t* __restrict__ out,
                                                                   const uint32_t* __restrict__ order,
                                                                   uint32_t* __restrict__ rule, uint32_t nout,
                                                                   const uint8_t* __restrict__ codes) {
  __shared__ uint32_t s_cnt[3];
  if (threadIdx.x == 0) s_cnt[0] = s_cnt[1] = 0;
  __syncthreads();
  http_chunks<true, kRaw>(T, batch, nslots, arena, VOut{out, order, rule, nout}, nullptr, s_cnt, nullptr, nullptr,
                          codes);
}

}  // namespace

int launch_http(const HttpDev& t, const void* batch, size_t nslots, const uint8_t* arena, uint8_t* out, void* stream,
                int cus, const uint32_t* order, uint32_t* rule, uint32_t nout, const uint8_t* codes) {
  if (nslots == 0) return 0;
  // hipFuncSetAttribute and the occupancy answer are per device: cached per
  // device ordinal, set once under a lock (handles on several GPUs may launch
  // from several threads)
  int dev = 0;
  (void)hipGetDevice(&dev);
  const bool raw = codes != nullptr;
  const size_t lds = ((size_t)t.lds_cells + (raw ? 64 : 0) + kLdsRuleHits + 3) * 4;
  const void* kern = raw ? (const void*)http_kernel<true> : (const void*)http_kernel<false>;
  int occ = 1;
  uint32_t* deal = nullptr;
  // The ticket reset and both launches are enqueued under one lock: two
  // host threads sharing a stream must not interleave as memset A, memset
  // B, kernel A, kernel B (B would start from A's spent ticket count and
  // write no verdicts).
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  {
    static std::map<std::pair<int, size_t>, int> occ_cache;
    static std::set<int> attr_set;
    // one ticket word per (device, stream), zeroed on the launch stream
    // right before the kernel: launches on one stream run in order, so each
    // starts from ticket 0 and no two launches in flight share a counter
    // (launches on different streams hold different words)
    static std::map<std::pair<int, void*>, uint32_t*> deal_words;
    if (kDynamicDeal) {
      auto& w = deal_words[{dev, stream}];
      if (!w) {
        void* p = nullptr;
        if (hipMalloc(&p, 64) != hipSuccess) return (int)hipErrorOutOfMemory;
        w = static_cast<uint32_t*>(p);
      }
      deal = w;
      const hipError_t rc = hipMemsetAsync(deal, 0, sizeof(uint32_t), (hipStream_t)stream);
      if (rc != hipSuccess) return (int)rc;
    }
    if (attr_set.insert(dev).second)
      for (const void* k : {(const void*)http_kernel<false>, (const void*)http_kernel<true>})
        (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    auto it = occ_cache.find({dev, lds});
    if (it == occ_cache.end()) {
      // one resident wave of workgroups: as many per CU as LDS and registers
      // allow (the largest staged program block sets the LDS share), then the
      // workgroups deal the chunks among themselves
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kHttpThreads, lds) !=
              hipSuccess ||
          nb < 1)
        nb = 1;
      it = occ_cache.emplace(std::make_pair(dev, lds), nb).first;
      if (getenv("CILIUM_GPU_DEBUG"))
        fprintf(stderr, "[cilium-gpu] http_kernel: device %d, %zu B dynamic LDS, %d workgroups per CU\n", dev, lds,
                nb);
    }
    occ = it->second;
  }
  const size_t tiles = nslots / kWave;
  size_t grid = std::min<size_t>(std::max<size_t>(tiles, 1), (size_t)cus * occ);
  if (raw)
    hipLaunchKernelGGL(http_kernel<true>, dim3((unsigned)grid), dim3(kHttpThreads), lds, (hipStream_t)stream, t,
                       (const uint8_t*)batch, nslots, arena, out, order, deal, rule, nout, codes);
  else
    hipLaunchKernelGGL(http_kernel<false>, dim3((unsigned)grid), dim3(kHttpThreads), lds, (hipStream_t)stream, t,
                       (const uint8_t*)batch, nslots, arena, out, order, deal, rule, nout, codes);
  if (t.n_global_progs) {
    grid = std::min<size_t>(std::max<size_t>(tiles, 1), (size_t)cus * 2);
    if (raw)
      hipLaunchKernelGGL(http_kernel_global<true>, dim3((unsigned)grid), dim3(kHttpThreads), 0, (hipStream_t)stream,
                         t, (const uint8_t*)batch, nslots, arena, out, order, rule, nout, codes);
    else
      hipLaunchKernelGGL(http_kernel_global<false>, dim3((unsigned)grid), dim3(kHttpThreads), 0, (hipStream_t)stream,
                         t, (const uint8_t*)batch, nslots, arena, out, order, rule, nout, codes);
  }
  return (int)hipGetLastError();
}

}  // namespace cg
