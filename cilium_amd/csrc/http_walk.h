// http_walk.h — the per-lane pieces of NetworkPolicyMap::Allowed
// (envoy/cilium_network_policy.h:223-237) that both the verdict kernel
// (kernels_http.hip) and the raw path's overflow walker (kernels_http_raw.hip)
// run: a comb-table DFA step (comb.h), the accept label of a state, the
// remote identity's PNPR mask row and the first rule two masks share.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dev_types.h"

namespace cg {
namespace walk {

// One comb transition (comb.h), branch-free: every lane reads the table and
// selects; the miss target max(S, dead) is one VALU (the walk is VALU-issue
// bound: each wave64 instruction holds the SIMD for 4 cycles).
// The walk is VALU-issue bound (PMC: ~60% of SIMD cycles issue VALU), so the
// select uses SDWA word selects: compare the check half and pick the next
// half in two instructions.  It goes through VCC, which serializes several
// chains per lane — one chain per lane (kTilesPerWave = 1) measured fastest.
__device__ __forceinline__ uint32_t comb_step(const uint32_t* __restrict__ cells, uint32_t dead, uint32_t st,
                                             uint32_t b) {
  const uint32_t e = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(cells) + ((st << 2) + (b << 2)));
  const uint32_t dflt = max(st, dead);
  // nx = e.lo == st ? e.hi : dflt
  uint32_t nx;
  asm("v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:WORD_0 src1_sel:DWORD\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_sdwa %0, %3, %1, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
      : "=v"(nx)
      : "v"(e), "v"(st), "v"(dflt)
      : "vcc");
  return nx;
}

// The class-mode step (comb.h): states are byte offsets and the string
// holds class codes 4*c, so the cell address is st + code — one SDWA add
// with the byte select, no shift.  The block sits at LDS address 0 in the
// fast path, so the add is the whole address.
__device__ __forceinline__ uint32_t comb_step_cls(const uint32_t* __restrict__ cells, uint32_t dead, uint32_t st,
                                                 uint32_t code) {
  const uint32_t e = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(cells) + (st + code));
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

template <bool kCls>
__device__ __forceinline__ uint32_t step(const uint32_t* __restrict__ cells, uint32_t dead, uint32_t st, uint32_t x) {
  return kCls ? comb_step_cls(cells, dead, st, x) : comb_step(cells, dead, st, x);
}

// Accept label of state st (its header cell).
template <bool kCls>
__device__ __forceinline__ uint32_t state_label(const uint32_t* __restrict__ cells, uint32_t st) {
  return (kCls ? *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(cells) + st - 4) : cells[st - 1]) >>
         16;
}

// Block offset of the PNPR mask of remote identity `remote`: the program's
// remote table (open addressing, {identity, mask offset} slots).
__device__ __forceinline__ uint32_t remote_row(const uint32_t* __restrict__ blk, const HttpProg& pg, uint32_t remote) {
  if (pg.flags & kProgRemoteDirect) {  // uniform: the direct array (dev_types.h)
    const uint32_t d = remote - pg.rdir_base;
    const bool in = d < pg.rdir_len;
    const uint32_t v = reinterpret_cast<const uint16_t*>(blk + pg.rdir_off)[in ? d : 0];
    return in ? v : pg.default_remote;
  }
  // both candidate buckets read together (dev_types.h rtab_b1/rtab_b2)
  const uint32_t h = rtab_hash(remote);
  const uint32_t* b1 = blk + pg.rtab_off + kRtabBucketCells * rtab_b1h(h, pg.rtab_nb);
  const uint32_t* b2 = blk + pg.rtab_off + kRtabBucketCells * rtab_b2h(h, pg.rtab_nb);
  const uint4 k1 = *reinterpret_cast<const uint4*>(b1), k2 = *reinterpret_cast<const uint4*>(b2);
  const uint4 r1 = *reinterpret_cast<const uint4*>(b1 + 4), r2 = *reinterpret_cast<const uint4*>(b2 + 4);
  // an empty slot holds an identity outside the table with the default row
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

// u64 word w of the block mask at block offset a (u32 units, 8-byte aligned).
__device__ __forceinline__ unsigned long long blk_word(const uint32_t* __restrict__ blk, uint32_t a, uint32_t w) {
  return *reinterpret_cast<const unsigned long long*>(blk + a + 2 * w);
}

// The first rule (lowest bit) the rule masks at block offsets a and row
// share, or kNoHit: the first rule that allows the request, in Envoy's
// evaluation order (http.cc build_prog).
constexpr uint32_t kNoHit = 0xFFFFFFFFu;
template <int W>
__device__ __forceinline__ uint32_t first_meet_w(const uint32_t* __restrict__ blk, uint32_t a, uint32_t row) {
  // every word read up front, no per-lane exits: the lowest word with a
  // shared bit wins
  unsigned long long x[W];
#pragma unroll
  for (int w = 0; w < W; ++w) x[w] = blk_word(blk, a, w) & blk_word(blk, row, w);
  unsigned long long sel = 0;
  uint32_t base = 0;
#pragma unroll
  for (int w = W - 1; w >= 0; --w) {
    const bool nz = x[w] != 0;
    sel = nz ? x[w] : sel;
    base = nz ? 64u * w : base;
  }
  return sel ? base + (uint32_t)__builtin_ctzll(sel) : kNoHit;
}

__device__ __forceinline__ uint32_t first_meet(const uint32_t* __restrict__ blk, uint32_t a, uint32_t row,
                                               uint32_t W) {
  switch (W) {  // uniform
    case 1: return first_meet_w<1>(blk, a, row);
    case 2: return first_meet_w<2>(blk, a, row);
    case 3: return first_meet_w<3>(blk, a, row);
    case 4: return first_meet_w<4>(blk, a, row);
    default:
      for (uint32_t w = 0; w < W; ++w) {
        const unsigned long long x = blk_word(blk, a, w) & blk_word(blk, row, w);
        if (x) return w * 64 + (uint32_t)__builtin_ctzll(x);
      }
      return kNoHit;
  }
}

}  // namespace walk
}  // namespace cg
