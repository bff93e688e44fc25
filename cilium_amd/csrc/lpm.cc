// lpm.cc — device structures for the XDP CIDR prefilter.
//
// check_v4/check_v6 (bpf/bpf_xdp.c:97-156) drop a packet whose source
// address is covered by any prefix of the dyn LPM map (only compiled in when
// both CIDR4_FILTER and CIDR4_LPM_PREFILTER are defined, i.e. fix4 && dyn4,
// prefilter.go:77-88) or equals a /32 (/128) of the fix hash map; otherwise
// the packet passes iff its destination is a local endpoint (cilium_lxc,
// bpf/lib/eps.h:26-46).  Both drop sources collapse into one "covered"
// interval set per family, which is what the device structures encode
// (dev_types.h LpmDev: two-level 2-bit /16 and /24 codes + ranked leaves for IPv4, a
// top-bits-indexed sorted interval array for IPv6).
#include "lpm.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <map>
#include <stdexcept>

namespace cg {

bool PrefilterState::enabled(int which) const {
  switch (which) {
    case 0: return config & CG_PF_DYN4;
    case 1: return config & CG_PF_FIX4;
    case 2: return config & CG_PF_DYN6;
    case 3: return config & CG_PF_FIX4;  // prefilter.go:237 gates v6 fix on fix4Enabled
  }
  return false;
}

namespace {

using U128 = std::pair<uint64_t, uint64_t>;  // (high word, low word)

U128 load128(const uint8_t* a) {
  uint64_t hi = 0, lo = 0;
  for (int i = 0; i < 8; ++i) hi = hi << 8 | a[i];
  for (int i = 8; i < 16; ++i) lo = lo << 8 | a[i];
  return {hi, lo};
}

U128 add1(U128 x) {
  if (++x.second == 0) ++x.first;
  return x;
}

}  // namespace

void PrefilterState::rebuild(Engine& e) {
  v4_filter = config & CG_PF_FIX4;
  v6_filter = config & CG_PF_FIX6;
  const bool lpm4 = v4_filter && (config & CG_PF_DYN4);
  const bool lpm6 = v6_filter && (config & CG_PF_DYN6);

  // ---------------- IPv4: 2-bit block codes + ranked leaves
  top.clear();
  top_rank.clear();
  mid.clear();
  leaf_base.clear();
  leaves.clear();
  if (v4_filter) {
    std::vector<std::pair<uint32_t, uint32_t>> iv;
    auto addv4 = [&](const CidrKey& k) {
      uint32_t net = (uint32_t)k.net[0] << 24 | k.net[1] << 16 | k.net[2] << 8 | k.net[3];
      uint32_t span = k.plen == 0 ? 0xFFFFFFFFu : ((1u << (32 - k.plen)) - 1);
      if (k.plen == 32) span = 0;
      iv.push_back({net, net + span});
    };
    if (lpm4)
      for (const auto& k : maps[0]) addv4(k);
    for (const auto& k : maps[1]) addv4(k);
    std::sort(iv.begin(), iv.end());
    std::vector<uint8_t> state(1u << 24, 0);
    std::map<uint32_t, std::array<uint64_t, 4>> part;  // block → leaf bits
    for (auto [a, b] : iv) {
      uint32_t ba = a >> 8, bb = b >> 8;
      for (uint64_t blk = ba; blk <= bb; ++blk) {
        uint32_t lo = (blk == ba) ? (a & 0xFF) : 0;
        uint32_t hi = (blk == bb) ? (b & 0xFF) : 0xFF;
        if (state[blk] == 1) continue;
        if (lo == 0 && hi == 0xFF) {
          state[blk] = 1;
          part.erase((uint32_t)blk);
          continue;
        }
        state[blk] = kLpmPartial;
        auto& l = part[(uint32_t)blk];
        for (uint32_t x = lo; x <= hi; ++x) l[x >> 6] |= 1ULL << (x & 63);
      }
    }
    top.assign(4096, 0);
    top_rank.assign(4096, 0);
    mid.clear();
    leaf_base.clear();
    uint32_t nmixed = 0, nleaf = 0;
    for (uint32_t q = 0; q < 65536; ++q) {
      if ((q & 15) == 0) top_rank[q >> 4] = nmixed;
      bool all1 = true, all0 = true;
      for (uint32_t k = 0; k < 256; ++k) {
        const uint8_t st = state[(q << 8) | k];
        all1 &= st == 1;
        all0 &= st == 0;
      }
      const uint32_t code = all1 ? 1 : all0 ? 0 : kLpmPartial;
      top[q >> 4] |= code << (2 * (q & 15));
      if (code != kLpmPartial) continue;
      ++nmixed;
      leaf_base.push_back(nleaf);
      for (uint32_t w = 0; w < 16; ++w) {
        uint32_t word = 0;
        for (uint32_t k = 0; k < 16; ++k) word |= (uint32_t)state[(q << 8) | (w << 4) | k] << (2 * k);
        mid.push_back(word);
        nleaf += __builtin_popcount(lpm_partials(word));
      }
    }
    if (mid.empty()) {
      mid.assign(16, 0);
      leaf_base.assign(1, 0);
    }
    leaves.reserve(part.size() * 4);
    for (const auto& [blk, l] : part) leaves.insert(leaves.end(), l.begin(), l.end());
    if (leaves.empty()) leaves.assign(4, 0);
  }

  // ---------------- IPv6 intervals + top-bits index
  v6_code.clear();
  v6_mix.clear();
  v6_iv.clear();
  if (v6_filter) {
    std::vector<std::pair<U128, U128>> iv;
    auto addv6 = [&](const CidrKey& k) {
      U128 lo = load128(k.net.data());
      U128 hi = lo;
      int host = 128 - k.plen;
      if (host >= 64) {
        hi.second = ~0ULL;
        hi.first |= (host == 128) ? ~0ULL : ((1ULL << (host - 64)) - 1);
      } else if (host > 0) {
        hi.second |= (1ULL << host) - 1;
      }
      iv.push_back({lo, hi});
    };
    if (lpm6)
      for (const auto& k : maps[2]) addv6(k);
    for (const auto& k : maps[3]) addv6(k);
    std::sort(iv.begin(), iv.end());
    std::vector<std::pair<U128, U128>> mg;
    for (auto& x : iv) {
      if (!mg.empty()) {
        U128 end = mg.back().second;
        bool adjacent = end != U128{~0ULL, ~0ULL} && add1(end) == x.first;
        if (x.first <= end || adjacent) {
          if (x.second > mg.back().second) mg.back().second = x.second;
          continue;
        }
      }
      mg.push_back(x);
    }
    for (auto& x : mg) {
      v6_iv.push_back(x.first.first);
      v6_iv.push_back(x.first.second);
      v6_iv.push_back(x.second.first);
      v6_iv.push_back(x.second.second);
    }
    // bucket bits: about two buckets per interval, 16..22 bits
    uint32_t bits = 16;
    while (bits < 22 && (1ull << bits) < 2 * mg.size()) ++bits;
    v6_bits = bits;
    if (mg.size() >= (1u << 28)) throw std::runtime_error("prefilter: too many IPv6 intervals");
    const uint32_t nb = 1u << bits;
    v6_code.assign(nb / 16, 0);
    size_t i = 0;  // first interval with hi >= the bucket start
    uint32_t nmixed = 0;
    for (uint32_t t = 0; t < nb; ++t) {
      if ((t & 15) == 0) v6_code[t >> 4] = (uint64_t)nmixed << 32;
      const U128 bs{(uint64_t)t << (64 - bits), 0};
      const U128 be{t + 1 == nb ? ~0ULL : ((uint64_t)(t + 1) << (64 - bits)) - 1, ~0ULL};
      while (i < mg.size() && mg[i].second < bs) ++i;
      size_t r = i;  // one past the last interval with lo <= the bucket end
      while (r < mg.size() && mg[r].first <= be) ++r;
      uint64_t code = 0;
      if (r > i) code = (r == i + 1 && mg[i].first <= bs && mg[i].second >= be) ? 1 : kLpmPartial;
      v6_code[t >> 4] |= code << (2 * (t & 15));
      if (code != kLpmPartial) continue;
      ++nmixed;
      const uint32_t R = (uint32_t)(r - 1), span = (uint32_t)std::min<size_t>(r - 1 - i, 15);
      v6_mix.push_back(R << 4 | span);
    }
  }
  // the kernel reads entry 0 / record 0 unconditionally
  if (v6_mix.empty()) v6_mix.assign(1, 0);
  if (v6_iv.empty()) v6_iv.assign(4, 0);

  // ---------------- endpoint tables (0 = empty slot)
  {
    uint32_t cap = next_pow2(std::max<size_t>(ep4.size() * 2, 16));
    ep4_keys.assign(cap, 0);
    ep4_zero = false;
    for (uint32_t a : ep4) {
      if (a == 0) {
        ep4_zero = true;
        continue;
      }
      uint32_t h = ep_hash32(a) & (cap - 1);
      while (ep4_keys[h] != 0 && ep4_keys[h] != a) h = (h + 1) & (cap - 1);
      ep4_keys[h] = a;
    }
  }
  {
    uint32_t cap = next_pow2(std::max<size_t>(ep6.size() * 2, 16));
    ep6_keys.assign((size_t)cap * 2, 0);
    ep6_zero = false;
    for (const auto& a : ep6) {
      U128 k = load128(a.data());
      if (k.first == 0 && k.second == 0) {
        ep6_zero = true;
        continue;
      }
      uint32_t h = ep_hash128(k.first, k.second) & (cap - 1);
      while ((ep6_keys[2 * h] | ep6_keys[2 * h + 1]) != 0 &&
             !(ep6_keys[2 * h] == k.first && ep6_keys[2 * h + 1] == k.second))
        h = (h + 1) & (cap - 1);
      ep6_keys[2 * h] = k.first;
      ep6_keys[2 * h + 1] = k.second;
    }
  }

  if (e.has_gpu()) {
    e.set_device();
    if (!d_counters) {
      d_counters = std::make_shared<DevMem>();
      d_counters->alloc(2 * sizeof(uint64_t));
      d_counters->zero();
    }
    auto t = std::make_shared<DevTables>();
    LpmDev d{};
    if (v4_filter) {
      d.top = t->add(top);
      d.top_rank = t->add(top_rank);
      d.mid = t->add(mid);
      d.leaf_base = t->add(leaf_base);
      d.leaves = t->add(leaves);
    }
    if (v6_filter) {
      d.v6_code = t->add(v6_code);
      d.v6_bits = v6_bits;
    }
    d.v6_mix = t->add(v6_mix);
    d.v6_iv = t->add(v6_iv);
    d.ep4_keys = t->add(ep4_keys);
    d.ep4_mask = (uint32_t)ep4_keys.size() - 1;
    d.ep4_zero = ep4_zero;
    d.ep6_keys = t->add(ep6_keys);
    d.ep6_mask = (uint32_t)(ep6_keys.size() / 2) - 1;
    d.ep6_zero = ep6_zero;
    t->counters = d_counters;
    d.counters = d_counters->as<unsigned long long>();
    tab = std::move(t);  // publish (the caller holds the handle lock)
    dev = d;
  }
  dirty = false;
}

}  // namespace cg
