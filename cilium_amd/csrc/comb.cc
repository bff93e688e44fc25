// comb.cc — first-fit row-displacement packing of a DFA (see comb.h).
#include "comb.h"

#include <algorithm>
#include <numeric>

#include "common.h"

namespace cg {

bool build_comb(const ClsDfa& d, const std::vector<uint32_t>& labels, CombTable* out, uint32_t max_base,
                bool by_class) {
  const int n = d.size();
  // row width: 256 bytes, or the byte classes
  const int width = by_class ? d.ncls : 256;
  auto tr = [&](int s, int x) { return d.trans[(size_t)s * d.ncls + (by_class ? x : d.clsmap[x])]; };
  struct Row {
    bool self = false;
    std::vector<uint8_t> exc;  // exception bytes (classes)
  };
  std::vector<Row> rows(n);
  for (int s = 1; s < n; ++s) {
    Row& r = rows[s];
    if (labels[s] != kCombNoLabel) {
      for (int c = 0; c < d.ncls; ++c)
        if (d.trans[(size_t)s * d.ncls + c] != 0)
          fail(CG_UNKNOWN_ERROR, "internal: accepting DFA state with a live transition");
      r.self = true;  // absorbing: the kernel steps through record padding
      continue;
    }
    int self_n = 0, dead_n = 0;
    for (int b = 0; b < width; ++b) {
      int t = tr(s, b);
      self_n += t == s;
      dead_n += t == 0;
    }
    r.self = self_n > dead_n;
    const int dflt = r.self ? s : 0;
    for (int b = 0; b < width; ++b)
      if (tr(s, b) != dflt) r.exc.push_back((uint8_t)b);
  }
  // placement: rows defaulting to dead first, then self rows at bases above
  // all of them; within each group most exceptions first, first fit.  A
  // state also owns the header cell base-1, so bases are unique.
  const uint32_t cap = max_base + width + 1;
  std::vector<uint8_t> used(cap, 0);
  std::vector<uint32_t> base(n, 0);
  uint64_t excs = 0;
  uint32_t self_lo = 1;
  for (int group = 0; group < 2; ++group) {
    std::vector<int> order;
    for (int s = 1; s < n; ++s)
      if (rows[s].self == (group == 1)) order.push_back(s);
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return rows[a].exc.size() > rows[b].exc.size(); });
    uint32_t lo_hint = group == 0 ? 1 : self_lo;
    if (group == 1) {  // the dead state first: the lowest self-default base
      while (lo_hint <= max_base && used[lo_hint - 1]) ++lo_hint;
      if (lo_hint > max_base) return false;
      base[0] = lo_hint;
      used[lo_hint - 1] = 1;
    }
    for (int s : order) {
      const Row& r = rows[s];
      while (lo_hint < cap && used[lo_hint - 1]) ++lo_hint;
      uint32_t b0 = lo_hint;
      for (;; ++b0) {
        if (b0 > max_base) return false;
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
      if (group == 0) self_lo = std::max(self_lo, b0 + 1);
    }
  }
  uint32_t ncells = width + 1;
  for (int s = 0; s < n; ++s) ncells = std::max(ncells, base[s] + width);
  out->cells.assign(ncells, kCombEmpty);
  out->state_enc = base;
  out->cells[base[0] - 1] = 0xFFFFu | (kCombNoLabel << 16);  // D: no label, no exceptions
  for (int s = 1; s < n; ++s) {
    const uint32_t b0 = base[s];
    out->cells[b0 - 1] = 0xFFFFu | ((labels[s] & 0xFFFFu) << 16);
    for (uint8_t x : rows[s].exc) out->cells[b0 + x] = b0 | (base[tr(s, x)] << 16);
  }
  out->start = n > 1 ? base[1] : base[0];
  out->dead = base[0];
  out->exceptions = excs;
  out->by_class = by_class;
  out->scaled = false;
  return true;
}

bool scale_comb(CombTable* t) {
  uint32_t top = t->dead;
  for (uint32_t s : t->state_enc) top = std::max(top, s);
  if (4ull * top > 0xFFFC) return false;
  for (uint32_t& c : t->cells) {
    if (c == kCombEmpty) continue;
    if ((c & 0xFFFF) == 0xFFFF) continue;  // header: 0xFFFF is never a multiple of 4
    c = ((c & 0xFFFF) * 4) | (((c >> 16) * 4) << 16);
  }
  for (uint32_t& s : t->state_enc) s *= 4;
  t->start *= 4;
  t->dead *= 4;
  t->scaled = true;
  return true;
}

ClsDfa zero_class_first(const ClsDfa& d) {
  const int z = d.clsmap[0];
  if (z == 0) return d;
  ClsDfa o = d;
  for (int b = 0; b < 256; ++b) {
    const int c = d.clsmap[b];
    o.clsmap[b] = (uint8_t)(c == z ? 0 : c == 0 ? z : c);
  }
  for (int s = 0; s < d.size(); ++s)
    std::swap(o.trans[(size_t)s * d.ncls + 0], o.trans[(size_t)s * d.ncls + z]);
  return o;
}

void rebase_comb(CombTable* t, uint32_t off) {
  if (off == 0) return;
  if (t->scaled) fail(CG_UNKNOWN_ERROR, "internal: rebase of a scaled comb table");
  for (uint32_t& c : t->cells) {
    if (c == kCombEmpty || (c & 0xFFFF) == 0xFFFF) continue;  // empty / header
    const uint32_t next = c >> 16;
    c = ((c & 0xFFFF) + off) | ((next ? next + off : 0) << 16);
  }
  for (uint32_t& s : t->state_enc) s += off;
  t->start += off;
  t->dead += off;
}

}  // namespace cg
