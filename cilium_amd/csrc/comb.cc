// comb.cc — first-fit row-displacement packing of a DFA (see comb.h).
#include "comb.h"

#include <algorithm>
#include <numeric>

namespace cg {

bool build_comb(const ClsDfa& d, const std::vector<uint32_t>& labels, CombTable* out) {
  const int n = d.size();
  struct Row {
    bool self = false, skip = false;
    std::vector<uint8_t> exc;  // exception bytes
  };
  std::vector<Row> rows(n);
  for (int s = 1; s < n; ++s) {
    int self_n = 0, dead_n = 0;
    for (int b = 0; b < 256; ++b) {
      int t = d.trans[(size_t)s * d.ncls + d.clsmap[b]];
      self_n += t == s;
      dead_n += t == 0;
    }
    Row& r = rows[s];
    r.self = self_n > dead_n;
    const int dflt = r.self ? s : 0;
    for (int b = 0; b < 256; ++b)
      if (d.trans[(size_t)s * d.ncls + d.clsmap[b]] != dflt) r.exc.push_back((uint8_t)b);
    r.skip = r.self && r.exc.size() == 1 && r.exc[0] == 0;
  }
  // placement: most exceptions first, first fit; a state also owns the
  // header cell base-1, so bases are unique
  std::vector<int> order(n > 0 ? n - 1 : 0);
  std::iota(order.begin(), order.end(), 1);
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return rows[a].exc.size() > rows[b].exc.size(); });
  const uint32_t cap = kCombMaxBase + 257;
  std::vector<uint8_t> used(cap, 0);
  std::vector<uint32_t> base(n, 0);
  uint32_t lo_hint = 1;
  uint64_t excs = 0;
  for (int s : order) {
    const Row& r = rows[s];
    while (lo_hint < cap && used[lo_hint - 1]) ++lo_hint;
    uint32_t b0 = lo_hint;
    for (;; ++b0) {
      if (b0 > kCombMaxBase) return false;
      if (used[b0 - 1]) continue;
      bool ok = true;
      for (uint8_t x : r.exc)
        if (used[b0 + x]) {
          ok = false;
          break;
        }
      if (ok) break;
    }
    base[s] = b0;
    used[b0 - 1] = 1;
    for (uint8_t x : r.exc) used[b0 + x] = 1;
    excs += r.exc.size();
  }
  uint32_t ncells = 257;
  for (int s = 1; s < n; ++s) ncells = std::max(ncells, base[s] + 256);
  out->cells.assign(ncells, kCombEmpty);
  out->state_enc.assign(n, 0);
  for (int s = 1; s < n; ++s)
    out->state_enc[s] = base[s] | (rows[s].self ? kCombSelf : 0) | (rows[s].skip ? kCombSkip : 0);
  for (int s = 1; s < n; ++s) {
    const uint32_t b0 = base[s];
    out->cells[b0 - 1] = 0xFFFFu | ((labels[s] & 0xFFFFu) << 16);
    for (uint8_t x : rows[s].exc) {
      int t = d.trans[(size_t)s * d.ncls + d.clsmap[x]];
      out->cells[b0 + x] = b0 | (out->state_enc[t] << 16);
    }
  }
  out->start = n > 1 ? out->state_enc[1] : 0;
  out->exceptions = excs;
  return true;
}

}  // namespace cg
