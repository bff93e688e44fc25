// comb.h — "default + exceptions" comb-packed DFA tables for the HTTP kernel.
//
// A minimized union DFA of a program has a few thousand states over ~50 byte
// classes, but almost every row is either a self-loop (states inside an
// unconstrained header field or a `.*`) or dead except for one or two bytes
// (literal path prefixes).  Each state therefore keeps a default target
// (dead, itself, or another state) and only its exception bytes are stored,
// packed first-fit into one array of 32-bit cells indexed by byte value
// (row displacement, Tarjan–Yao), so the kernel needs no byte-class lookup:
//
//   state encoding  S = base | kind << 14     (kind: 0 dead-default,
//                                              1 self-default, 2 other,
//                                              3 self on every byte but SEP)
//   cell[base + b]  = base | next(S, b) << 16  when b is an exception
//   cell[base - 1]  = 0xFFFF | default << 16   (header; 0xFFFF never a base)
//
//   next(S, b) = cell[base+b].lo == base ? cell[base+b].hi
//              : kind == 0 ? 0 : kind == 1 ? S : cell[base-1].hi
//
// The dead state is S = 0 (base 0 is never given to a state).  Bases are
// limited to 14 bits; a program whose table does not fit is split into more
// parts by the caller.
#pragma once

#include <cstdint>
#include <vector>

#include "clsdfa.h"

namespace cg {

constexpr uint32_t kCombMaxBase = 0x3FFF;
constexpr uint32_t kCombEmpty = 0xFFFFFFFFu;

struct CombTable {
  std::vector<uint32_t> cells;
  std::vector<uint32_t> state_enc;  // encoding of each DFA state (0 for dead)
  uint32_t start = 0;
  uint64_t exceptions = 0;
};

// Returns false if the table needs a base beyond kCombMaxBase.
bool build_comb(const ClsDfa& d, CombTable* out);

inline uint32_t comb_next(const uint32_t* cells, uint32_t s, uint32_t b) {
  const uint32_t base = s & kCombMaxBase;
  const uint32_t e = cells[base + b];
  if ((e & 0xFFFF) == base) return e >> 16;
  const uint32_t kind = s >> 14;
  return kind == 0 ? 0 : (kind == 1 || kind == 3) ? s : (cells[base - 1] >> 16);
}

}  // namespace cg
