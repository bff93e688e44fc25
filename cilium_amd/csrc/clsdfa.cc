// clsdfa.cc — Hopcroft minimization over byte classes.
#include "clsdfa.h"

#include <algorithm>
#include <deque>
#include <map>
#include <numeric>
#include <unordered_map>

#include "common.h"

namespace cg {

namespace {

// Refinable partition (Valmari-style): elements of a block are contiguous in
// `elems`; marking moves an element into the block's marked prefix.
struct Partition {
  std::vector<int> elems, loc, blk, first, end, mid;
  std::vector<int> touched;

  explicit Partition(int n) : elems(n), loc(n), blk(n, 0) {
    std::iota(elems.begin(), elems.end(), 0);
    std::iota(loc.begin(), loc.end(), 0);
  }
  int nblocks() const { return (int)first.size(); }
  void mark(int e) {
    int b = blk[e];
    int i = loc[e], j = mid[b];
    if (i < j) return;  // already marked
    std::swap(elems[i], elems[j]);
    loc[elems[i]] = i;
    loc[elems[j]] = j;
    if (mid[b]++ == first[b]) touched.push_back(b);
  }
};

}  // namespace

ClsDfa minimize_cls(const ClsDfa& d) {
  const int n = d.size();
  const int k = d.ncls;
  // initial partition by label (dead state shares block with other label-0 states)
  Partition P(n);
  {
    std::vector<std::pair<uint32_t, int>> v(n);
    for (int s = 0; s < n; ++s) v[s] = {d.label[s], s};
    std::stable_sort(v.begin(), v.end());
    for (int i = 0; i < n; ++i) {
      int s = v[i].second;
      P.elems[i] = s;
      P.loc[s] = i;
      if (i == 0 || v[i].first != v[i - 1].first) {
        P.first.push_back(i);
        if (i > 0) P.end.push_back(i);
      }
      P.blk[s] = (int)P.first.size() - 1;
    }
    P.end.push_back(n);
    P.mid = P.first;
  }
  // inverse transitions, CSR per (class, target)
  std::vector<int> inv_off((size_t)k * n + 1, 0);
  std::vector<int> inv((size_t)n * k);
  for (int s = 0; s < n; ++s)
    for (int c = 0; c < k; ++c) inv_off[(size_t)c * n + d.trans[(size_t)s * k + c] + 1]++;
  for (size_t i = 1; i < inv_off.size(); ++i) inv_off[i] += inv_off[i - 1];
  {
    std::vector<int> fill(inv_off.begin(), inv_off.end() - 1);
    for (int s = 0; s < n; ++s)
      for (int c = 0; c < k; ++c) inv[fill[(size_t)c * n + d.trans[(size_t)s * k + c]]++] = s;
  }
  std::vector<uint8_t> in_w(P.nblocks(), 1);
  std::vector<int> W;
  for (int b = 0; b < P.nblocks(); ++b) W.push_back(b);
  std::vector<int> splitter;
  while (!W.empty()) {
    int A = W.back();
    W.pop_back();
    in_w[A] = 0;
    splitter.assign(P.elems.begin() + P.first[A], P.elems.begin() + P.end[A]);
    for (int c = 0; c < k; ++c) {
      for (int t : splitter) {
        size_t o = (size_t)c * n + t;
        for (int i = inv_off[o]; i < inv_off[o + 1]; ++i) P.mark(inv[i]);
      }
      for (int b : P.touched) {
        if (P.mid[b] == P.end[b]) {  // every element marked: no split
          P.mid[b] = P.first[b];
          continue;
        }
        // split: marked [first, mid) becomes new block nb
        int nb = P.nblocks();
        P.first.push_back(P.first[b]);
        P.end.push_back(P.mid[b]);
        P.mid.push_back(P.first[b]);
        P.first[b] = P.mid[b];
        P.mid[b] = P.first[b];
        for (int i = P.first[nb]; i < P.end[nb]; ++i) P.blk[P.elems[i]] = nb;
        in_w.push_back(0);
        int sz_nb = P.end[nb] - P.first[nb], sz_b = P.end[b] - P.first[b];
        if (in_w[b]) {
          W.push_back(nb);
          in_w[nb] = 1;
        } else if (sz_nb <= sz_b) {
          W.push_back(nb);
          in_w[nb] = 1;
        } else {
          W.push_back(b);
          in_w[b] = 1;
        }
      }
      P.touched.clear();
    }
  }
  // quotient with canonical BFS order
  const int nb = P.nblocks();
  std::vector<int> rep(nb);
  for (int b = 0; b < nb; ++b) rep[b] = P.elems[P.first[b]];
  std::vector<int> newid(nb, -1);
  std::vector<int> order;
  int dead_b = P.blk[0];
  newid[dead_b] = 0;
  order.push_back(dead_b);
  ClsDfa out;
  int start_b = P.blk[1];
  if (start_b != dead_b) {
    newid[start_b] = 1;
    order.push_back(start_b);
    for (size_t qi = 1; qi < order.size(); ++qi) {
      int s = rep[order[qi]];
      for (int c = 0; c < k; ++c) {
        int t = P.blk[d.trans[(size_t)s * k + c]];
        if (newid[t] < 0) {
          newid[t] = (int)order.size();
          order.push_back(t);
        }
      }
    }
  } else {
    order.push_back(dead_b);  // language empty: start == a copy of dead
  }
  const int m = (int)order.size();
  // recompress classes: classes with identical columns merge
  std::vector<int> col_id(k);
  std::vector<int> col_rep;
  {
    std::map<std::vector<int>, int> cols;
    std::vector<int> col(m);
    for (int c = 0; c < k; ++c) {
      for (int i = 0; i < m; ++i) {
        int t = (i == 1 && start_b == dead_b) ? 0 : newid[P.blk[d.trans[(size_t)rep[order[i]] * k + c]]];
        col[i] = (i == 0) ? 0 : t;
      }
      auto it = cols.emplace(col, (int)cols.size());
      col_id[c] = it.first->second;
      if (it.second) col_rep.push_back(c);
    }
  }
  out.ncls = (int)col_rep.size();
  for (int b = 0; b < 256; ++b) out.clsmap[b] = (uint8_t)col_id[d.clsmap[b]];
  out.trans.assign((size_t)m * out.ncls, 0);
  out.label.assign(m, 0);
  for (int i = 1; i < m; ++i) {
    if (start_b == dead_b) break;
    int s = rep[order[i]];
    out.label[i] = d.label[s];
    for (int c = 0; c < out.ncls; ++c)
      out.trans[(size_t)i * out.ncls + c] = newid[P.blk[d.trans[(size_t)s * k + col_rep[c]]]];
  }
  return out;
}

}  // namespace cg
