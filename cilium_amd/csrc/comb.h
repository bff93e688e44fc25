// comb.h — "default + exceptions" comb-packed DFA tables for the HTTP kernel.
//
// A minimized union DFA of a program has a few thousand states over ~50 byte
// classes, but almost every row is either a self-loop (states inside an
// unconstrained header field or a `.*`) or dead except for one or two bytes
// (literal path prefixes).  Each state therefore keeps a default target —
// dead or itself — and only its exception bytes are stored, packed first-fit
// into one array of 32-bit cells indexed by byte value (row displacement,
// Tarjan–Yao), so the kernel needs no byte-class lookup.  A state IS its base
// (a 16-bit cell index).  The dead state D is a row of its own with no
// exceptions, at the lowest base of the rows whose default is the state
// itself; every row defaulting to dead sits below it:
//
//   cell[S + b]  = S | next(S, b) << 16      when b is an exception of S
//   cell[S - 1]  = 0xFFFF | label << 16      (header; 0xFFFF is never a base;
//                                             label = accept-set index or 0xFFFF)
//
//   next(S, b) = cell[S+b].lo == S ? cell[S+b].hi : max(S, D)
//
// so the default costs one v_max_u32 per step (a dead-default row has S < D,
// a self row S > D, and D defaults to itself).  Base 0 is never given to a
// state, so no check half-word is ever 0.  Accepting states are made
// absorbing (self, no exceptions): the request strings these tables read end
// with the last field's separator, after which every accepting row is dead
// anyway, so the kernel may keep stepping through the zero padding of a
// record without checking the string length per byte.
//
// Bases are table-local; `rebase_comb` shifts them by the table's offset
// inside a program's cell block so that all parts of a program share one
// pointer (the LDS block) — possible while the block stays below 0xFFFF cells.
//
// Class mode (by_class): rows are indexed by byte class (cell[S + c], c <
// ncls) instead of byte, and `scale_comb` stores every state as its byte
// offset 4*S (the header of S is at byte offset 4*S - 4).  The packer then
// writes each string byte b as the code 4*clsmap[b] (one byte, so ncls <=
// 64), and a step's cell address is state + code: one add, no shift.
#pragma once

#include <cstdint>
#include <vector>

#include "clsdfa.h"

namespace cg {

constexpr uint32_t kCombMaxBase = 0xFEFF;  // base + 255 stays below 0xFFFF
constexpr uint32_t kCombEmpty = 0xFFFFFFFFu;
constexpr uint32_t kCombNoLabel = 0xFFFF;

struct CombTable {
  bool by_class = false;            // rows indexed by byte class (see above)
  bool scaled = false;              // states stored as byte offsets 4*S
  std::vector<uint32_t> cells;
  std::vector<uint32_t> state_enc;  // base of each DFA state (state 0 = dead: D)
  uint32_t start = 0;
  uint32_t dead = 0;                // the dead state; states >= dead default to themselves
  uint64_t exceptions = 0;
};

// labels[s]: accept-set index of DFA state s (kCombNoLabel if none).  An
// accepting state must have no live transition (throws Error otherwise).
// Returns false if the table needs a base beyond `max_base`.
bool build_comb(const ClsDfa& d, const std::vector<uint32_t>& labels, CombTable* out,
                uint32_t max_base = kCombMaxBase, bool by_class = false);

// Shift every base of `t` by `off` (its position inside a program block).
void rebase_comb(CombTable* t, uint32_t off);

// States → byte offsets 4*S (class mode); false if a state exceeds 16 bits.
bool scale_comb(CombTable* t);

// The DFA with its byte classes renumbered so that byte 0x00 (the record
// padding) is class 0: code 0 then walks as the padding byte.
ClsDfa zero_class_first(const ClsDfa& d);

// One step: s a state (raw: base, scaled: byte offset), x the byte (raw) or
// its code 4*class (scaled).
inline uint32_t comb_next(const uint32_t* cells, uint32_t dead, uint32_t s, uint32_t x, bool scaled = false) {
  const uint32_t e = scaled ? cells[(s + x) >> 2] : cells[s + x];
  if ((e & 0xFFFF) == s) return e >> 16;
  return s > dead ? s : dead;
}

inline uint32_t comb_label(const uint32_t* cells, uint32_t s, bool scaled = false) {
  return (scaled ? cells[(s >> 2) - 1] : cells[s - 1]) >> 16;
}

}  // namespace cg
