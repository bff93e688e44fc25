// l4.cc — cuckoo table build for policy maps.
//
// The reference keeps one BPF_MAP_TYPE_HASH per endpoint keyed by the 8-byte
// struct policy_key (bpf/lib/common.h:180-186, pkg/maps/policymap).  The
// device copy is a 2-choice (partial-key) cuckoo hash of 64-byte buckets (4
// slots of {key, entry id | proxy_port_be << 16, fingerprint}) plus one u32 of
// 8-bit fingerprints per bucket: the kernel screens a key against its two
// buckets' fingerprints in LDS and reads a slot only on a fingerprint match.  Counters live in a separate per-entry-id array so a rebuild never
// moves them.
#include "l4.h"

#include <hip/hip_runtime_api.h>

#include <random>

namespace cg {

namespace {

bool try_build(const std::unordered_map<uint64_t, PolicyMapState::Entry>& entries, uint32_t nbuckets,
               std::vector<L4Slot>& slots) {
  slots.assign((size_t)nbuckets * 4, L4Slot{kL4EmptyKey, 0, 0});
  const uint32_t mask = nbuckets - 1;
  std::mt19937_64 rng(0xC111A);
  for (const auto& [key, ent] : entries) {
    L4Slot cur{key, (uint32_t)ent.id | ((uint32_t)ent.proxy_port_be << 16), 0};
    uint32_t b1, b2, fp;
    l4_place(cur.key, mask, &b1, &b2, &fp);
    cur.pad = fp;
    uint32_t b = b1;
    bool placed = false;
    for (int kick = 0; kick < 500 && !placed; ++kick) {
      const uint32_t alt = b ^ (l4_alt(cur.pad) & mask);
      for (uint32_t bb : {b, alt}) {
        for (int s = 0; s < 4 && !placed; ++s)
          if (slots[(size_t)bb * 4 + s].key == kL4EmptyKey) {
            slots[(size_t)bb * 4 + s] = cur;
            placed = true;
          }
        if (placed) break;
      }
      if (placed) break;
      // evict a random slot of the alternate bucket; the victim moves on to
      // its own alternate (partial-key cuckoo: bucket XOR alt(fingerprint))
      b = alt;
      std::swap(cur, slots[(size_t)b * 4 + (rng() & 3)]);
    }
    if (!placed) return false;
  }
  return true;
}

}  // namespace

void PolicyMapState::rebuild(Engine& e) {
  // load factor (0.25, 0.5]: 16,384 entries fit 8,192 buckets, whose 32 KiB
  // fingerprint array sits in LDS next to the 128 KiB of counters
  uint32_t nb = next_pow2(std::max<size_t>((entries.size() + 1) / 2, 4));
  while (!try_build(entries, nb, slots)) nb *= 2;
  bucket_mask = nb - 1;
  fp.assign(nb, 0);
  for (uint32_t bk = 0; bk < nb; ++bk)
    for (int s = 0; s < 4; ++s)
      if (slots[(size_t)bk * 4 + s].key != kL4EmptyKey) fp[bk] |= slots[(size_t)bk * 4 + s].pad << (8 * s);
  if (e.has_gpu()) {
    e.set_device();
    if (!d_counters) {
      d_counters = std::make_shared<DevMem>();
      d_counters->alloc((size_t)max_entries * 2 * sizeof(uint64_t));
      d_counters->zero();
    }
    auto t = std::make_shared<DevTables>();
    L4Dev d{};
    d.slots = t->add(slots);
    d.fp = t->add(fp);
    t->counters = d_counters;
    d.bucket_mask = bucket_mask;
    d.max_entries = max_entries;
    d.counters = d_counters->as<unsigned long long>();
    tab = std::move(t);  // publish (the caller holds the handle lock)
    dev = d;
  }
  dirty = false;
}

void PolicyMapState::read_counters(Engine& e, uint32_t id, uint64_t* pk, uint64_t* by) {
  *pk = *by = 0;
  if (!e.has_gpu() || !d_counters) return;
  e.set_device();
  uint64_t v[2];
  hip_check(hipMemcpy(v, d_counters->as<uint64_t>() + (size_t)id * 2, 16, hipMemcpyDeviceToHost),
            "read counters");
  *pk = v[0];
  *by = v[1];
}

void PolicyMapState::zero_counter(Engine& e, uint32_t id) {
  if (!e.has_gpu() || !d_counters) return;
  e.set_device();
  hip_check(hipMemset(d_counters->as<uint64_t>() + (size_t)id * 2, 0, 16), "zero counter");
}

}  // namespace cg
