// comb.cc — first-fit row-displacement packing of a DFA (see comb.h).
#include "comb.h"

#include <algorithm>
#include <numeric>

namespace cg {

bool build_comb(const ClsDfa& d, CombTable* out) {
  const int n = d.size();
  struct Row {
    int state;
    uint32_t kind;
    int dflt;
    std::vector<uint8_t> exc;  // exception bytes
  };
  std::vector<Row> rows(n);
  std::vector<int> cnt(n);
  for (int s = 1; s < n; ++s) {
    // per-class targets, then pick the default that minimizes exception bytes
    std::vector<int> cls_bytes(d.ncls, 0);
    for (int b = 0; b < 256; ++b) cls_bytes[d.clsmap[b]]++;
    int dead_n = 0, self_n = 0;
    std::vector<std::pair<int, int>> other;  // (target, bytes)
    for (int c = 0; c < d.ncls; ++c) {
      int t = d.trans[(size_t)s * d.ncls + c];
      if (t == 0) dead_n += cls_bytes[c];
      else if (t == s) self_n += cls_bytes[c];
      else {
        bool found = false;
        for (auto& o : other)
          if (o.first == t) {
            o.second += cls_bytes[c];
            found = true;
          }
        if (!found) other.push_back({t, cls_bytes[c]});
      }
    }
    Row r;
    r.state = s;
    int best_other = -1, best_other_n = -1;
    for (auto& o : other)
      if (o.second > best_other_n) best_other = o.first, best_other_n = o.second;
    if (self_n >= dead_n && self_n >= best_other_n) {
      r.kind = 1;
      r.dflt = s;
    } else if (dead_n >= best_other_n) {
      r.kind = 0;
      r.dflt = 0;
    } else {
      r.kind = 2;
      r.dflt = best_other;
    }
    for (int b = 0; b < 256; ++b)
      if (d.trans[(size_t)s * d.ncls + d.clsmap[b]] != r.dflt) r.exc.push_back((uint8_t)b);
    // a self-loop on every byte but the field separator: the kernel skips to
    // the next SEP without touching the table
    if (r.kind == 1 && r.exc.size() == 1 && r.exc[0] == 0) r.kind = 3;
    rows[s] = std::move(r);
  }
  // placement: most exceptions first
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
  uint32_t ncells = 0;
  for (int s = 1; s < n; ++s) ncells = std::max(ncells, base[s] + 256);
  out->cells.assign(std::max<uint32_t>(ncells, 257), kCombEmpty);
  out->state_enc.assign(n, 0);
  for (int s = 1; s < n; ++s) out->state_enc[s] = base[s] | (rows[s].kind << 14);
  for (int s = 1; s < n; ++s) {
    const Row& r = rows[s];
    uint32_t b0 = base[s];
    out->cells[b0 - 1] = 0xFFFFu | (out->state_enc[r.dflt] << 16);
    for (uint8_t x : r.exc) {
      int t = d.trans[(size_t)s * d.ncls + d.clsmap[x]];
      out->cells[b0 + x] = b0 | (out->state_enc[t] << 16);
    }
  }
  out->start = n > 1 ? out->state_enc[1] : 0;
  out->exceptions = excs;
  return true;
}

}  // namespace cg
