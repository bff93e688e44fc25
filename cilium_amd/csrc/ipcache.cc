// ipcache.cc — device structures for the IP → identity longest-prefix map.
//
// With HAVE_LPM_MAP_TYPE the datapath asks the kernel LPM trie for the
// longest prefix covering the address (ipcache_lookup{4,6} with a full-length
// key, bpf/lib/eps.h:111-114); without it, it probes the configured prefix
// lengths from long to short (LPM_LOOKUP_FN, eps.h:86-108).  Both return the
// entry of the longest covering prefix.  The callers then take sec_label and
// tunnel_endpoint if the entry exists and sec_label != 0, else WORLD_ID
// (bpf_lxc.c:509-518, :202-211).  The tables below store that resolved pair.
#include "ipcache.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <tuple>

namespace cg {

namespace {

using U128 = std::pair<uint64_t, uint64_t>;  // (high word, low word)

U128 key128(const CidrKey& k) {
  uint64_t hi = 0, lo = 0;
  for (int i = 0; i < 8; ++i) hi = hi << 8 | k.net[i];
  for (int i = 8; i < 16; ++i) lo = lo << 8 | k.net[i];
  return {hi, lo};
}

U128 last128(U128 lo, int plen) {
  const int host = 128 - plen;
  if (host >= 64) {
    lo.second = ~0ULL;
    lo.first |= host == 128 ? ~0ULL : ((1ULL << (host - 64)) - 1);
  } else if (host > 0) {
    lo.second |= (1ULL << host) - 1;
  }
  return lo;
}

}  // namespace

void IpcacheState::build_tables() {
  // the resolved pair as a table entry: identity 0 (a pointer tag) never occurs
  auto resolved = [](const IpcVal& v) -> uint64_t {
    return v.identity == 0 ? kIpcMiss : ((uint64_t)v.tunnel << 32 | v.identity);
  };

  // ---- IPv4: paint prefixes in increasing length, so a range being painted
  // never holds a pointer below the prefix's own level.
  // Full-length prefixes (/32, /128: pod addresses, most of a cluster's
  // ipcache) go to the exact tables; the trie and the runs hold the rest.
  std::vector<std::tuple<int, uint32_t, uint64_t>> v4;  // plen, net (host order), entry
  std::vector<std::tuple<U128, int, uint64_t>> v6;      // start, plen, entry
  std::vector<std::pair<uint32_t, uint64_t>> x4;        // /32: address, entry
  std::vector<std::pair<U128, uint64_t>> x6;            // /128
  for (const auto& [k, v] : entries) {
    if (k.family == 4) {
      const uint32_t net = (uint32_t)k.net[0] << 24 | k.net[1] << 16 | k.net[2] << 8 | k.net[3];
      if (k.plen == 32) x4.emplace_back(net, resolved(v));
      else v4.emplace_back(k.plen, net, resolved(v));
    } else {
      if (k.plen == 128) x6.emplace_back(key128(k), resolved(v));
      else v6.emplace_back(key128(k), k.plen, resolved(v));
    }
  }
  // open addressing at load <= 1/4 (a lookup's first slot is nearly always
  // the answer or empty), linear probing; the longest probe sequence bounds
  // every lookup
  {
    uint32_t cap = 16;
    while (cap < 4 * x4.size()) cap <<= 1;
    ex4.assign(4 * (size_t)cap, 0);
    ex4_mask = cap - 1;
    ex4_probes = 0;
    for (const auto& [a, e] : x4) {
      uint32_t p = 0;
      while (ex4[4 * (size_t)((ipc_ex4_hash(a) + p) & ex4_mask) + 1]) ++p;
      uint32_t* sl = &ex4[4 * (size_t)((ipc_ex4_hash(a) + p) & ex4_mask)];
      sl[0] = a;
      sl[1] = 1;
      sl[2] = (uint32_t)e;
      sl[3] = (uint32_t)(e >> 32);
      ex4_probes = std::max(ex4_probes, p);
    }
    cap = 16;
    while (cap < 4 * x6.size()) cap <<= 1;
    ex6.assign(4 * (size_t)cap, 0);
    ex6_mask = cap - 1;
    ex6_probes = 0;
    for (const auto& [k, e] : x6) {
      const uint32_t h = ipc_ex6_hash(k.first, k.second);
      uint32_t p = 0;
      while (ex6[4 * (size_t)((h + p) & ex6_mask) + 3]) ++p;
      uint64_t* sl = &ex6[4 * (size_t)((h + p) & ex6_mask)];
      sl[0] = k.first;
      sl[1] = k.second;
      sl[2] = e;
      sl[3] = 1;
      ex6_probes = std::max(ex6_probes, p);
    }
  }
  std::sort(v4.begin(), v4.end());
  l16.assign(65536, kIpcMiss);
  chunks.clear();
  auto child = [&](uint64_t& e) -> uint32_t {
    if ((uint32_t)e != 0) {
      const uint64_t c = chunks.size() / 256;
      if (c > 0xFFFFFFFFull) fail(CG_MAP_FULL, "ipcache: too many trie chunks");
      chunks.insert(chunks.end(), 256, e);  // inherits the shorter prefix's value
      e = c << 32;
    }
    return (uint32_t)(e >> 32);
  };
  for (auto [plen, net, val] : v4) {
    if (plen <= 16) {
      const uint32_t q = net >> 16, n = 1u << (16 - plen);
      std::fill(l16.begin() + q, l16.begin() + q + n, val);
    } else if (plen <= 24) {
      const uint32_t c = child(l16[net >> 16]);
      const uint32_t k = (net >> 8) & 255, n = 1u << (24 - plen);
      std::fill(chunks.begin() + (size_t)c * 256 + k, chunks.begin() + (size_t)c * 256 + k + n, val);
    } else {
      const uint32_t c = child(l16[net >> 16]);
      uint64_t e = chunks[(size_t)c * 256 + ((net >> 8) & 255)];
      const uint32_t d = child(e);  // may grow chunks: write the entry back by index
      chunks[(size_t)c * 256 + ((net >> 8) & 255)] = e;
      const uint32_t k = net & 255, n = 1u << (32 - plen);
      std::fill(chunks.begin() + (size_t)d * 256 + k, chunks.begin() + (size_t)d * 256 + k + n, val);
    }
  }
  if (chunks.empty()) chunks.assign(256, kIpcMiss);

  // /16 summaries (on the dense chunks): background = the most frequent
  // value among the chunk's entries, [lo, hi] = the /24s holding anything
  // else, direct = that range is one /24 pointing to a /32 chunk
  std::vector<uint32_t> sum_chunk(65536, 0), sum_range(65536, 1);
  std::vector<uint64_t> sum_bg(65536);
  {
    std::vector<uint64_t> vals(256);
    for (uint32_t q = 0; q < 65536; ++q) {
      const uint64_t e = l16[q];
      uint64_t bg = e;
      uint32_t chunk = 0, lo = 1, hi = 0, direct = 0;
      if ((uint32_t)e == 0) {
        const uint32_t c = (uint32_t)(e >> 32);
        const uint64_t* ent = &chunks[(size_t)c * 256];
        vals.assign(ent, ent + 256);
        std::sort(vals.begin(), vals.end());
        bg = kIpcMiss;
        size_t best = 0;
        for (size_t i = 0; i < 256;) {
          size_t j = i;
          while (j < 256 && vals[j] == vals[i]) ++j;
          if ((uint32_t)vals[i] != 0 && j - i > best) best = j - i, bg = vals[i];
          i = j;
        }
        lo = 256;
        for (uint32_t k = 0; k < 256; ++k)
          if (ent[k] != bg) {
            lo = std::min(lo, k);
            hi = k;
          }
        if (lo == 256) lo = 1, hi = 0;
        chunk = c;
        if (lo == hi && (uint32_t)ent[lo] == 0) {
          direct = 1;
          chunk = (uint32_t)(ent[lo] >> 32);
        }
      }
      sum_bg[q] = bg;
      sum_chunk[q] = chunk;
      sum_range[q] = lo | hi << 8 | direct << 16;
    }
    for (const auto& xa : x4) sum_range[xa.first >> 16] |= kIpcExact;
  }

  // Encode the dense chunks (dev_types.h ipc_chunk_get): /32-level chunks
  // first, then the /24-level ones with their pointers rewritten to the
  // encoded references.
  const size_t ndense = chunks.size() / 256;
  std::vector<uint8_t> level(ndense, 0);  // 1: /24-level, 2: /32-level
  for (uint32_t q = 0; q < 65536; ++q)
    if ((uint32_t)l16[q] == 0) level[(uint32_t)(l16[q] >> 32)] = 1;
  for (size_t c = 0; c < ndense; ++c)
    if (level[c] == 1)
      for (uint32_t k = 0; k < 256; ++k)
        if ((uint32_t)chunks[c * 256 + k] == 0) level[(uint32_t)(chunks[c * 256 + k] >> 32)] = 2;
  std::vector<uint64_t> enc;
  std::vector<uint32_t> ref(ndense, 0);
  size_t n_runs = 0, n_sparse = 0, n_dense = 0;
  // Dense chunks unless CILIUM_GPU_IPC_ENCODE is set: the run lines and
  // sparse maps take ~20x less memory (7 MB, not 139 MB, at the bench's 512K
  // entries) but a third of the IPv4 lookups a second dependent load, and
  // measured slower (tools/ipcache_split.py: IPv4 59-66 vs 81 G lookups/s,
  // profiles/r06j_*, r06p_*); both forms go through the same kernel.
  const bool all_dense = getenv("CILIUM_GPU_IPC_ENCODE") == nullptr;
  auto encode = [&](const uint64_t* ent) -> uint32_t {
    const size_t at = enc.size();
    // the kernels address words with 32-bit offsets (dev_types.h ipc_chunk_first)
    if (at + 256 >= (1ull << 32)) fail(CG_MAP_FULL, "ipcache: encoded chunks past 32 GiB");
    uint32_t nr = all_dense ? 256 : 1;
    for (uint32_t k = 1; k < 256 && !all_dense; ++k) nr += ent[k] != ent[k - 1];
    if (nr <= 7) {
      uint64_t w0 = nr;
      uint32_t r = 0;
      enc.resize(at + 8, 0);
      enc[at + 1] = ent[0];
      for (uint32_t k = 1; k < 256; ++k)
        if (ent[k] != ent[k - 1]) {
          ++r;
          w0 |= (uint64_t)k << (8 * r);
          enc[at + 1 + r] = ent[k];
        }
      enc[at] = w0;
      ++n_runs;
      return kIpcRuns << 30 | (uint32_t)(at / 8);
    }
    std::vector<uint64_t> v(ent, ent + 256);
    std::sort(v.begin(), v.end());
    uint64_t base = v[0];
    size_t best = 0;
    for (size_t i = 0; i < 256;) {
      size_t j = i;
      while (j < 256 && v[j] == v[i]) ++j;
      if (j - i > best) best = j - i, base = v[i];
      i = j;
    }
    const size_t k_set = 256 - best;
    if (6 + k_set < 256 && !all_dense) {
      enc.resize(at + ((6 + k_set + 7) & ~(size_t)7), 0);
      size_t r = 0;
      for (uint32_t k = 0; k < 256; ++k) {
        if (k % 56 == 0) enc[at + k / 56] |= (uint64_t)r << 56;
        if (ent[k] != base) {
          enc[at + k / 56] |= 1ull << (k % 56);
          enc[at + 6 + r++] = ent[k];
        }
      }
      enc[at + 5] = base;
      ++n_sparse;
      return kIpcSparse << 30 | (uint32_t)(at / 8);
    }
    enc.insert(enc.end(), ent, ent + 256);
    ++n_dense;
    return kIpcDense << 30 | (uint32_t)(at / 8);
  };
  for (size_t c = 0; c < ndense; ++c)
    if (level[c] == 2) ref[c] = encode(&chunks[c * 256]);
  {
    std::vector<uint64_t> tmp(256);
    for (size_t c = 0; c < ndense; ++c) {
      if (level[c] != 1) continue;
      for (uint32_t k = 0; k < 256; ++k) {
        const uint64_t e = chunks[c * 256 + k];
        tmp[k] = (uint32_t)e == 0 ? (uint64_t)ref[(uint32_t)(e >> 32)] << 32 : e;
      }
      ref[c] = encode(tmp.data());
    }
  }
  if (enc.empty()) enc.assign(8, 0);
  l16x.assign(65536 * 4, 0);
  for (uint32_t q = 0; q < 65536; ++q) {
    uint32_t* x = &l16x[4 * (size_t)q];
    x[0] = (uint32_t)sum_bg[q];
    x[1] = (uint32_t)(sum_bg[q] >> 32);
    x[2] = (sum_range[q] & 255) <= ((sum_range[q] >> 8) & 255) ? ref[sum_chunk[q]] : 0u;
    x[3] = sum_range[q];
  }
  const size_t dense_bytes = chunks.size() * 8;
  chunks.swap(enc);

  // ---- IPv6: sweep the nested prefix intervals into runs of one value.
  std::sort(v6.begin(), v6.end(), [](const auto& a, const auto& b) {
    return std::get<0>(a) != std::get<0>(b) ? std::get<0>(a) < std::get<0>(b) : std::get<1>(a) < std::get<1>(b);
  });
  std::vector<std::pair<U128, uint64_t>> runs{{U128{0, 0}, kIpcMiss}};
  auto emit = [&](U128 pos, uint64_t v) {
    if (runs.back().first == pos) {
      runs.back().second = v;
      if (runs.size() > 1 && runs[runs.size() - 2].second == v) runs.pop_back();
      return;
    }
    if (runs.back().second != v) runs.push_back({pos, v});
  };
  const U128 kMax{~0ULL, ~0ULL};
  std::vector<std::pair<U128, uint64_t>> open;  // (last address, value)
  auto close_one = [&] {
    const U128 end = open.back().first;
    open.pop_back();
    if (end != kMax) {
      U128 nx = end;
      if (++nx.second == 0) ++nx.first;
      emit(nx, open.empty() ? kIpcMiss : open.back().second);
    }
  };
  for (const auto& [lo, plen, vi] : v6) {
    while (!open.empty() && open.back().first < lo) close_one();
    emit(lo, vi);
    open.push_back({last128(lo, plen), vi});
  }
  while (!open.empty()) close_one();
  runs6.clear();
  for (const auto& [pos, v] : runs) {
    runs6.push_back(pos.first);
    runs6.push_back(pos.second);
    runs6.push_back(v);
    runs6.push_back(0);
  }
  uint32_t bits = 16;
  while (bits < 22 && (1ull << bits) < 2 * runs.size()) ++bits;
  v6_bits = bits;
  const uint32_t nb = 1u << bits;
  std::vector<uint8_t> has_exact(nb, 0);  // buckets holding /128 entries (set, flagged)
  for (const auto& xk : x6) has_exact[(uint32_t)(xk.first.first >> (64 - bits))] = 1;
  code6.assign(nb / 32, 0);
  ent6.clear();
  crowd6.clear();
  size_t L = 0;  // last run starting at or before the bucket start
  uint64_t nset = 0;
  for (uint32_t t = 0; t < nb; ++t) {
    if ((t & 31) == 0) code6[t >> 5] = nset << 32;
    const U128 start{(uint64_t)t << (64 - bits), 0};
    const U128 end{t + 1 == nb ? ~0ULL : ((uint64_t)(t + 1) << (64 - bits)) - 1, ~0ULL};
    while (L + 1 < runs.size() && runs[L + 1].first <= start) ++L;
    size_t R = L;  // last run starting at or before the bucket end
    while (R + 1 < runs.size() && runs[R + 1].first <= end) ++R;
    if (R == L && runs[L].second == kIpcMiss && !has_exact[t]) continue;
    code6[t >> 5] |= 1ULL << (t & 31);
    ++nset;
    uint32_t crowd = kIpcNoCrowd;
    if (R - L >= 8 && R - L < 255) {
      // prefix of the starts of runs L+1..R (sorted: the first and last agree on it)
      const U128 a = runs[L + 1].first, b = runs[R].first;
      const uint64_t xh = a.first ^ b.first, xl = a.second ^ b.second;
      uint32_t sp = xh ? (uint32_t)__builtin_clzll(xh) : xl ? 64 + (uint32_t)__builtin_clzll(xl) : 128;
      sp = std::min<uint32_t>(sp, 122);
      const uint64_t mh = sp >= 64 ? ~0ULL : ~0ULL << (64 - sp), ml = sp > 64 ? ~0ULL << (128 - sp) : 0;
      const U128 P{a.first & mh, a.second & ml};
      crowd = (uint32_t)(crowd6.size() / 128);
      crowd6.resize(crowd6.size() + 128, 0);
      uint8_t* d = &crowd6[(size_t)crowd * 128];
      std::memcpy(d, &P.first, 8);
      std::memcpy(d + 8, &P.second, 8);
      std::memcpy(d + 16, &sp, 4);
      // sub[i] = last run (offset from L) starting at or before P + i * 2^(122 - sp)
      const uint32_t sh = 122 - sp;
      typedef unsigned __int128 u128;
      const u128 pv = (u128)P.first << 64 | P.second, step = (u128)1 << sh;
      size_t r = L;
      for (uint32_t i = 0; i <= 64; ++i) {
        const u128 qv = pv + step * i;  // wraps only for i = 64 at the top window
        const U128 q = (i && qv < pv) ? U128{~0ULL, ~0ULL} : U128{(uint64_t)(qv >> 64), (uint64_t)qv};
        while (r + 1 <= R && runs[r + 1].first <= q) ++r;
        d[24 + i] = (uint8_t)(r - L);
      }
    }
    ent6.insert(ent6.end(), {(uint32_t)L, (uint32_t)R, crowd, (uint32_t)has_exact[t]});
  }
  if (ent6.empty()) ent6.assign(4, 0);
  if (crowd6.empty()) crowd6.assign(128, 0);
  if (getenv("CILIUM_GPU_DEBUG")) {
    size_t c24 = 0, direct = 0;
    for (uint32_t q = 0; q < 65536; ++q)
      if ((uint32_t)l16[q] == 0) ++c24, direct += (l16x[4 * q + 3] >> 16) & 1;
    fprintf(stderr, "[cilium-gpu] ipcache: v4 chunks %zu (%zu /16s chunked, %zu direct): %zu runs, %zu sparse, "
            "%zu dense, %.1f MB (dense form %.1f MB); v6 runs %zu (%.1f MB), buckets 2^%u, set %zu (%.1f MB), "
            "crowd lines %zu; exact /32 %zu (%.1f MB, probes <= %u), /128 %zu (%.1f MB, probes <= %u)\n", ndense, c24,
            direct, n_runs, n_sparse, n_dense, chunks.size() * 8 / 1e6, dense_bytes / 1e6, runs6.size() / 4,
            runs6.size() * 8 / 1e6, v6_bits, ent6.size() / 4, ent6.size() * 4 / 1e6, crowd6.size() / 128, x4.size(),
            ex4.size() * 4 / 1e6, ex4_probes + 1, x6.size(), ex6.size() * 8 / 1e6, ex6_probes + 1);
  }
}

IpcacheDev IpcacheState::host_view() const {
  IpcacheDev v{};
  v.l16x = l16x.data();
  v.chunks = chunks.data();
  v.code6 = code6.data();
  v.ent6 = ent6.data();
  v.crowd6 = crowd6.data();
  v.runs6 = runs6.data();
  v.v6_bits = v6_bits;
  v.nruns6 = (uint32_t)(runs6.size() / 4);
  v.ex4 = ex4.data();
  v.ex6 = ex6.data();
  v.ex4_mask = ex4_mask;
  v.ex6_mask = ex6_mask;
  v.ex4_probes = ex4_probes;
  v.ex6_probes = ex6_probes;
  return v;
}

void IpcacheState::rebuild(Engine& e) {
  build_tables();
  if (e.has_gpu()) {
    e.set_device();
    auto t = std::make_shared<DevTables>();
    IpcacheDev d{};
    d.l16x = t->add(l16x);
    d.chunks = t->add(chunks);
    d.code6 = t->add(code6);
    d.ent6 = t->add(ent6);
    d.crowd6 = t->add(crowd6);
    d.runs6 = t->add(runs6);
    d.v6_bits = v6_bits;
    d.nruns6 = (uint32_t)(runs6.size() / 4);
    d.ex4 = t->add(ex4);
    d.ex6 = t->add(ex6);
    d.ex4_mask = ex4_mask;
    d.ex6_mask = ex6_mask;
    d.ex4_probes = ex4_probes;
    d.ex6_probes = ex6_probes;
    tab = std::move(t);  // publish (the caller holds the handle lock)
    dev = d;
  }
  dirty = false;
}

}  // namespace cg
