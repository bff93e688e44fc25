// clsdfa.h — byte-class-compressed DFA with per-state accept labels, and its
// Hopcroft minimization.  Used for the per-program union automata.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace cg {

struct ClsDfa {
  int ncls = 1;
  uint8_t clsmap[256] = {0};
  std::vector<int32_t> trans;   // size() * ncls; state 0 = dead, 1 = start
  std::vector<uint32_t> label;  // 0 = non-accepting, else an accept-set id
  int size() const { return (int)label.size(); }
  int next(int s, uint8_t b) const { return trans[(size_t)s * ncls + clsmap[b]]; }
};

// Hopcroft partition refinement (initial partition by label), quotient,
// canonical BFS renumbering from the start state (dead → 0, start → 1, then
// breadth-first in class order) and re-compression of byte classes.
ClsDfa minimize_cls(const ClsDfa& d);

}  // namespace cg
