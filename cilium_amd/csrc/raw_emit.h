// raw_emit.h — the walked string's bytes into 16-byte tile units, coded
// through a program's code map (kernels_http_raw.hip raw_scan_dl_kernel /
// raw_defer_dl_kernel; http_pack.cc builds the same string on the host).
// Host and device: tests/native/tileout_test.cc runs it on the CPU.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dev_types.h"

namespace cg {

// Four string bytes through a code map.
CG_HD inline uint32_t code4(const uint8_t* lut, uint32_t q) {
  return (uint32_t)lut[q & 0xFFu] | (uint32_t)lut[(q >> 8) & 0xFFu] << 8 | (uint32_t)lut[(q >> 16) & 0xFFu] << 16 |
         (uint32_t)lut[q >> 24] << 24;
}

// Bytes gather in 16; each full unit is coded and stored to the slot's next
// string unit (64 uint4 = 1 KiB apart in the tile); in the last unit the
// bytes past the string stay zero (the walk's padding).
// kCode = false: the bytes go out uncoded (the device-layout scan: http_kernel
// codes them as it walks, launch_http `codes`).
template <bool kCode = true>
struct TileOut {
  uint32_t w0, w1, w2, w3, pos;
  uint4* dst;               // the slot's next string unit
  const uint8_t* lut;       // the program's code map
  CG_HD inline TileOut(uint4* d, const uint8_t* l) : w0(0), w1(0), w2(0), w3(0), pos(0), dst(d), lut(l) {}
  // nb (1..4) bytes, little-endian in v (its bytes past nb zero), at byte
  // pos: one 64-bit shift spreads them over dword pos / 4 and the next; the
  // part past the 16 bytes starts the next unit
  CG_HD inline void put4(uint32_t v, uint32_t nb) {
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
  CG_HD inline void put(uint32_t b) { put4(b, 1); }
  CG_HD inline void flush() {
    *dst = kCode ? make_uint4(code4(lut, w0), code4(lut, w1), code4(lut, w2), code4(lut, w3)) : make_uint4(w0, w1, w2, w3);
    dst += 64;
    w0 = w1 = w2 = w3 = 0;
    pos = 0;
  }
  // the last, partial unit: its coded bytes, zero past the string
  CG_HD inline void finish() {
    if (!pos) return;
    const uint32_t p = pos;
    auto keep = [&](uint32_t c, uint32_t at) {  // bytes of dword `at` below p
      return p >= at + 4 ? c : p <= at ? 0u : c & ((1u << (8 * (p - at))) - 1u);
    };
    auto c = [&](uint32_t w) { return kCode ? code4(lut, w) : w; };
    *dst = make_uint4(keep(c(w0), 0), keep(c(w1), 4), keep(c(w2), 8), keep(c(w3), 12));
  }
};

}  // namespace cg
