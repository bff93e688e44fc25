// comb.h — "default + exceptions" comb-packed DFA tables for the HTTP kernel.
//
// A minimized union DFA of a program has a few thousand states over ~50 byte
// classes, but almost every row is either a self-loop (states inside an
// unconstrained header field or a `.*`) or dead except for one or two bytes
// (literal path prefixes).  Each state therefore keeps a default target —
// dead or itself — and only its exception bytes are stored, packed first-fit
// into one array of 32-bit cells indexed by byte value (row displacement,
// Tarjan–Yao), so the kernel needs no byte-class lookup:
//
//   state encoding  S = base | self << 14 | skip << 15
//       self: the default target is S itself (else dead)
//       skip: self on every byte but SEP (0x00): the kernel does not even
//             read the table inside such a field
//   cell[base + b]  = base | next(S, b) << 16    when b is an exception
//   cell[base - 1]  = 0xFFFF | label << 16       (header; 0xFFFF is never a
//                                                 base; label = accept-set
//                                                 index or 0xFFFF)
//
//   next(S, b) = cell[base+b].lo == base ? cell[base+b].hi : (self ? S : 0)
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
constexpr uint32_t kCombSelf = 1u << 14;
constexpr uint32_t kCombSkip = 1u << 15;
constexpr uint32_t kCombEmpty = 0xFFFFFFFFu;
constexpr uint32_t kCombNoLabel = 0xFFFF;

struct CombTable {
  std::vector<uint32_t> cells;
  std::vector<uint32_t> state_enc;  // encoding of each DFA state (0 for dead)
  uint32_t start = 0;
  uint64_t exceptions = 0;
};

// labels[s]: accept-set index of DFA state s (kCombNoLabel if none).
// Returns false if the table needs a base beyond kCombMaxBase.
bool build_comb(const ClsDfa& d, const std::vector<uint32_t>& labels, CombTable* out);

inline uint32_t comb_next(const uint32_t* cells, uint32_t s, uint32_t b) {
  const uint32_t base = s & kCombMaxBase;
  const uint32_t e = cells[base + b];
  if ((e & 0xFFFF) == base) return e >> 16;
  return (s & kCombSelf) ? s : 0;
}

inline uint32_t comb_label(const uint32_t* cells, uint32_t s) {
  return s ? cells[(s & kCombMaxBase) - 1] >> 16 : kCombNoLabel;
}

}  // namespace cg
