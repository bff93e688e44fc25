// lpm.cc — device structures for the XDP CIDR prefilter.
//
// check_v4/check_v6 (bpf/bpf_xdp.c:97-156) drop a packet whose source
// address is covered by any prefix of the dyn LPM map (only compiled in when
// both CIDR4_FILTER and CIDR4_LPM_PREFILTER are defined, i.e. fix4 && dyn4,
// prefilter.go:77-88) or equals a /32 (/128) of the fix hash map; otherwise
// the packet passes iff its destination is a local endpoint (cilium_lxc,
// bpf/lib/eps.h:26-46).  Both drop sources collapse into one "covered"
// interval set per family, which is what the device structures encode.
#include "lpm.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <map>

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

  // ---------------- IPv4 DIR-24-8
  dir24.clear();
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
    dir24.assign(1u << 24, 0);
    std::map<uint32_t, uint32_t> leaf_of;
    auto leaf = [&](uint32_t blk) -> uint64_t* {
      auto it = leaf_of.find(blk);
      if (it == leaf_of.end()) {
        it = leaf_of.emplace(blk, (uint32_t)(leaves.size() / 4)).first;
        leaves.resize(leaves.size() + 4, 0);
      }
      return &leaves[(size_t)it->second * 4];
    };
    for (auto [a, b] : iv) {
      uint32_t ba = a >> 8, bb = b >> 8;
      for (uint64_t blk = ba; blk <= bb; ++blk) {
        uint32_t lo = (blk == ba) ? (a & 0xFF) : 0;
        uint32_t hi = (blk == bb) ? (b & 0xFF) : 0xFF;
        if (dir24[blk] == 1) continue;
        if (lo == 0 && hi == 0xFF) {
          dir24[blk] = 1;
          continue;
        }
        uint64_t* l = leaf((uint32_t)blk);
        for (uint32_t x = lo; x <= hi; ++x) l[x >> 6] |= 1ULL << (x & 63);
      }
    }
    for (auto [blk, li] : leaf_of)
      if (dir24[blk] != 1) dir24[blk] = li + 2;
    if (leaves.empty()) leaves.assign(4, 0);
  }

  // ---------------- IPv6 intervals + top-16 index
  v6_idx.clear();
  v6_lo.clear();
  v6_hi.clear();
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
      v6_lo.push_back(x.first.first);
      v6_lo.push_back(x.first.second);
      v6_hi.push_back(x.second.first);
      v6_hi.push_back(x.second.second);
    }
    v6_idx.assign(65537, 0);
    size_t i = 0;
    for (uint32_t t = 0; t < 65536; ++t) {
      uint64_t block_start = (uint64_t)t << 48;
      while (i < mg.size() && mg[i].second.first < block_start) ++i;
      v6_idx[t] = (uint32_t)i;
    }
    v6_idx[65536] = (uint32_t)mg.size();
    if (v6_lo.empty()) {
      v6_lo.assign(2, 0);
      v6_hi.assign(2, 0);
    }
  }

  // ---------------- endpoint tables
  {
    uint32_t cap = next_pow2(std::max<size_t>(ep4.size() * 2, 16));
    ep4_keys.assign(cap, 0);
    ep4_occ.assign(cap, 0);
    for (uint32_t a : ep4) {
      uint32_t h = ep_hash32(a) & (cap - 1);
      while (ep4_occ[h] && ep4_keys[h] != a) h = (h + 1) & (cap - 1);
      ep4_keys[h] = a;
      ep4_occ[h] = 1;
    }
  }
  {
    uint32_t cap = next_pow2(std::max<size_t>(ep6.size() * 2, 16));
    ep6_keys.assign((size_t)cap * 2, 0);
    ep6_occ.assign(cap, 0);
    for (const auto& a : ep6) {
      U128 k = load128(a.data());
      uint32_t h = ep_hash128(k.first, k.second) & (cap - 1);
      while (ep6_occ[h] && !(ep6_keys[2 * h] == k.first && ep6_keys[2 * h + 1] == k.second))
        h = (h + 1) & (cap - 1);
      ep6_keys[2 * h] = k.first;
      ep6_keys[2 * h + 1] = k.second;
      ep6_occ[h] = 1;
    }
  }

  if (e.has_gpu()) {
    e.set_device();
    dev = LpmDev{};
    if (v4_filter) {
      d_dir24.upload_vec(dir24);
      d_leaves.upload_vec(leaves);
      dev.dir24 = d_dir24.as<uint32_t>();
      dev.leaves = d_leaves.as<uint64_t>();
    }
    if (v6_filter) {
      d_v6_idx.upload_vec(v6_idx);
      d_v6_lo.upload_vec(v6_lo);
      d_v6_hi.upload_vec(v6_hi);
      dev.v6_idx = d_v6_idx.as<uint32_t>();
      dev.v6_lo = d_v6_lo.as<uint64_t>();
      dev.v6_hi = d_v6_hi.as<uint64_t>();
    }
    d_ep4k.upload_vec(ep4_keys);
    d_ep4o.upload_vec(ep4_occ);
    d_ep6k.upload_vec(ep6_keys);
    d_ep6o.upload_vec(ep6_occ);
    dev.ep4_keys = d_ep4k.as<uint32_t>();
    dev.ep4_occ = d_ep4o.as<uint8_t>();
    dev.ep4_mask = (uint32_t)ep4_occ.size() - 1;
    dev.ep6_keys = d_ep6k.as<uint64_t>();
    dev.ep6_occ = d_ep6o.as<uint8_t>();
    dev.ep6_mask = (uint32_t)ep6_occ.size() - 1;
    if (d_counters.size() == 0) {
      d_counters.alloc(2 * sizeof(uint64_t));
      d_counters.zero();
    }
    dev.counters = d_counters.as<unsigned long long>();
  }
  dirty = false;
}

}  // namespace cg
