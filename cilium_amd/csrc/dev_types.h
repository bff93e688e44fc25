// dev_types.h — table layouts shared by the host builders (.cc) and the HIP
// kernels (kernels.hip).  Plain structs passed to kernels by value.
#pragma once

#include <cstddef>
#include <cstdint>

#include "../../include/cilium_gpu.h"

#if defined(__HIP__) || defined(__HIPCC__)
#define CG_HD __host__ __device__
#else
#define CG_HD
#endif

namespace cg {

// ------------------------------------------------------------------ L4 ----
// Cuckoo hash of policy keys (2 choices × 64-B buckets of 4 slots).
// slot = {u64 key, u32 val, u32 pad}; key = sec_label | dport<<32 | proto<<48 |
// egress_byte<<56 (the 8-byte struct policy_key read little-endian);
// val = entry id (bits 0..15) | proxy_port_be (bits 16..31).
// Empty slot: key == kL4EmptyKey (an all-ones key, rejected on insert).
constexpr uint64_t kL4EmptyKey = ~0ULL;
struct L4Slot {
  uint64_t key;
  uint32_t val;
  uint32_t pad;
};
struct L4Dev {
  const L4Slot* slots;   // nbuckets * 4
  const uint32_t* fp;    // nbuckets: the 4 slots' 8-bit fingerprints (0 = empty)
  uint32_t bucket_mask;  // nbuckets - 1
  uint32_t max_entries;  // counter ids < max_entries
  unsigned long long* counters;  // [id*2] packets, [id*2+1] bytes
};

CG_HD inline uint64_t l4_hash1(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
// Policy-key hash for the device table, 32-bit arithmetic only (three
// quarter-rate multiplies per key and the first two shared between the three
// keys of one tuple): key = identity | (dport | proto << 16 | egress << 24) << 32.
CG_HD inline uint32_t l4_fin(uint32_t x) {
  x ^= x >> 15;
  x *= 0x2C1B3C6Du;
  x ^= x >> 13;
  return x;
}
constexpr uint32_t kL4MulLo = 0x9E3779B1u, kL4MulHi = 0x85EBCA77u;
CG_HD inline uint32_t l4_h(uint64_t key) {
  return l4_fin((uint32_t)key * kL4MulLo + (uint32_t)(key >> 32) * kL4MulHi);
}
// Second-bucket offset from the fingerprint (8-bit x 24-bit: a full-rate mul24).
CG_HD inline uint32_t l4_alt(uint32_t fp) { return (fp * 0x9E3779u) | 1u; }

CG_HD inline uint64_t l4_hash2(uint64_t k) {
  k += 0x9e3779b97f4a7c15ULL;
  k ^= k >> 30;
  k *= 0xbf58476d1ce4e5b9ULL;
  k ^= k >> 27;
  k *= 0x94d049bb133111ebULL;
  k ^= k >> 31;
  return k;
}

// Partial-key cuckoo placement: the hash gives the first bucket (low bits) and
// an 8-bit fingerprint (top byte, 1..255); the second bucket is the first XOR
// a function of the fingerprint, so either bucket and the fingerprint recover
// the other.
CG_HD inline void l4_place_h(uint32_t h, uint32_t mask, uint32_t* b1, uint32_t* b2, uint32_t* fp) {
  uint32_t f = h >> 24;
  f = f ? f : 1u;
  *fp = f;
  *b1 = h & mask;
  *b2 = *b1 ^ (l4_alt(f) & mask);
}
CG_HD inline void l4_place(uint64_t key, uint32_t mask, uint32_t* b1, uint32_t* b2, uint32_t* fp) {
  l4_place_h(l4_h(key), mask, b1, b2, fp);
}

// ----------------------------------------------------------------- LPM ----
// IPv4: two levels of 2-bit codes (0 not covered, 1 covered, 2 mixed/partial),
// 16 per u32 word.  Level 1: one code per /16 (16 KiB, cache resident).
// Level 2, only for mixed /16s (ranked by popcount over level 1 plus
// top_rank per word): the 256 /24 codes of the /16 in one 64-B chunk.  A
// partial /24's 256-bit leaf (4 x u64 over the last octet) is leaf_base of its
// /16 plus the partial /24s before it in the chunk.
// IPv6: disjoint covered intervals sorted by lo, 32-B records {lo hi-word,
// lo lo-word, hi hi-word, hi lo-word}, bucketed by the top v6_bits address
// bits (~2 buckets per interval).  Level 1 is the v4 scheme again: one 2-bit
// code per bucket (0 no interval touches it, 1 one interval covers it, 2
// mixed), 16 per u64 word whose high half counts the mixed buckets before the
// word — 512 KiB at 2^20 buckets, L2 resident, and it settles every address
// outside the mixed buckets.  A mixed bucket's u32 in v6_mix is R << 4 |
// min(R - L, 15): its candidate intervals are [L, R] (L = first interval with
// hi >= the bucket start, R = the last one with lo <= the bucket end; 15
// means "search from 0", correct because earlier intervals end before the
// bucket), so a mixed lookup reads one 4-B entry and the interval records.
// Local endpoints (cilium_lxc): open addressing, linear probing, 0 = empty
// slot (the all-zero address is a flag of its own).
constexpr uint32_t kLpmPartial = 2;
struct LpmDev {
  const uint32_t* top;       // 4096 words: /16 codes (nullptr: no v4 filter)
  const uint32_t* top_rank;  // 4096: mixed /16s before each word
  const uint32_t* mid;       // 16 words per mixed /16: its /24 codes
  const uint32_t* leaf_base; // per mixed /16: partial /24s before it
  const uint64_t* leaves;    // 4 u64 per partial /24, in address order
  const uint64_t* v6_code;   // (1 << v6_bits) / 16 words (nullptr: no v6 filter)
  const uint32_t* v6_mix;    // per mixed bucket (at least one entry)
  const uint64_t* v6_iv;     // 4 u64 per interval (at least one record)
  uint32_t v6_bits;
  const uint32_t* ep4_keys;  // v4 endpoint table (network-order addresses)
  uint32_t ep4_mask;
  uint32_t ep4_zero;         // 0.0.0.0 is an endpoint
  const uint64_t* ep6_keys;  // 2 u64 per slot (hi, lo)
  uint32_t ep6_mask;
  uint32_t ep6_zero;
  unsigned long long* counters;  // [0] drop, [1] pass
};

CG_HD inline uint32_t ep_hash32(uint32_t a) { return l4_fin(a * kL4MulLo); }
CG_HD inline uint32_t ep_hash128(uint64_t hi, uint64_t lo) {
  return l4_fin((uint32_t)hi * kL4MulLo + (uint32_t)(hi >> 32) * kL4MulHi + (uint32_t)lo * 0xC2B2AE3Du +
                (uint32_t)(lo >> 32) * 0x27D4EB2Fu);
}
// Partial-block count among the 16 2-bit codes of a word (code 2 = binary 10).
CG_HD inline uint32_t lpm_partials(uint32_t w) { return w & ~(w << 1) & 0xAAAAAAAAu; }
// IPv6 bucket tb: its code (0/1/2) and, for a mixed one, its v6_mix index.
CG_HD inline uint32_t v6_code_of(uint64_t cw, uint32_t tb, uint32_t* m) {
  const uint32_t w = (uint32_t)cw, sh = 2 * (tb & 15);
  *m = (uint32_t)(cw >> 32) + (uint32_t)__builtin_popcount(lpm_partials(w) & ((1u << sh) - 1));
  return (w >> sh) & 3;
}

// ---------------------------------------------------------------- HTTP ----
// Program = one (policy, direction, port) evaluation: Envoy's exact-port
// PortNetworkPolicyRules merged with the port-0 ones (cilium_network_policy.h:169-192).
constexpr uint32_t kProgAllowAll = 1;  // some scope has no HTTP rules / no rules
constexpr uint32_t kProgHasAlways = 2;  // some PNPR has an empty HTTP rule list
constexpr uint32_t kNoAcc = 0xFFFFFFFFu;
struct HttpProg {
  uint32_t part_begin;
  uint32_t part_count;
  uint32_t flags;
  uint32_t mask_words;      // W
  uint32_t always_off;      // block offset (u32 units) of the "no HTTP rules" PNPR mask
  uint32_t default_remote;  // block offset of the PNPR mask of identities not in the table
  uint32_t cell_begin;      // the program's block in cells[], staged into LDS
  uint32_t cell_count;      // as one piece: parts' comb cells, label tables, masks,
  uint32_t rtab_off;        // remote-identity table: 2-choice buckets (rtab_buckets())
  uint32_t rtab_nb;         // buckets (any count)
  uint32_t rule_base;       // this program's first per-rule hit counter
  uint32_t nrules;          // mask bits = rules (HttpSnapshot::rule_info)
  // kProgRemoteDirect: identities rdir_base .. rdir_base + rdir_len - 1 map
  // to their mask row through a u16 array at block offset rdir_off (others:
  // default_remote) — one LDS read instead of the bucket search
  uint32_t rdir_base, rdir_len, rdir_off, pad;
};
constexpr uint32_t kProgRemoteDirect = 16;
constexpr uint32_t kRdirMaxSpan = 8192;
// Per-rule hit counters a workgroup keeps in LDS for its current program
// (programs with more rules count straight into global memory).
constexpr uint32_t kLdsRuleHits = 512;
// 160 KiB less the rest of http_kernel's LDS (allowed/denied pair and deal
// ticket, per-rule hit counters, and the 64-word code map the raw-byte
// instantiation stages after the block): the largest program table a
// workgroup stages (http.cc, http_pack.cc)
constexpr uint32_t kMaxLdsCells = (160 * 1024 - 64 - 4 * kLdsRuleHits - 4 * 64) / 4;
constexpr uint32_t kNoRow = 0xFFFFFFFFu;  // empty remote-table slot
// One DFA of a program as a comb-packed table (comb.h).  A state is its base
// cell index relative to `walk_off`; `dead` is the dead state, states above it
// default to themselves and states below it to `dead` (comb.h).
// An accepting state's header cell holds its accept label; the label's PNPR
// mask (u64 words stored as u32 pairs, 8-byte aligned) is at block offset
// acc_off + label * 2 * mask_words, block = cells + cell_begin.  When a program's DFA
// cells stay below 0xFFFF its parts are rebased onto the block (walk_off =
// cell_begin for every part), so the kernel walks all parts through one
// pointer — the LDS copy.
constexpr uint32_t kProgRebased = 4;
// One part in class mode (kPartClass): the packer writes the program's
// strings as class codes (HttpSnapshot::prog_code).
constexpr uint32_t kProgClass = 8;
struct HttpPart {
  uint32_t cell_off;  // first cell of this part in cells[]
  uint32_t ncells;
  uint32_t acc_off;   // block offset of accept label 0's PNPR mask (label l: + l * 2 * mask_words)
  uint32_t start;     // start state
  uint32_t nstates;
  uint32_t dead;
  uint32_t walk_off;  // cells[] offset the states are relative to
  uint32_t mode;      // 0: byte-indexed rows; kPartClass: class rows, states as byte offsets (comb.h)
};
constexpr uint32_t kPartClass = 1;
// Special program ids in the program lookup.
constexpr uint32_t kProgAllow = 0xFFFFFFFEu;  // no policy for the port → allow
constexpr uint32_t kProgDeny = 0xFFFFFFFFu;   // unknown policy → deny

// Packed HTTP batch (cg_http_pack): a 64-byte header, the chunk table, the
// tile table, then the tiles (1 KiB aligned).  A tile is 64 request records
// stored unit-major: the meta block (8 bytes per lane), then `units` 16-byte
// string units, each one contiguous 1 KiB (string unit u ≥ 1 of lane l at
// tile + 512 + (u-1)*1024 + l*16).  A tile whose lanes hold at most 8 bytes
// in its last unit may store that unit as a half unit (kTileHalfLast: 8 bytes
// per lane, 512 B, lane l at its start + l*8): cg_http_pack does, the
// device-built batches do not.  The
// packer groups requests by program so every chunk (≤ kChunkTiles tiles)
// belongs to one program and a workgroup can stage that program's table in
// LDS.  Slot order is returned to the caller (order[]).
constexpr uint32_t kBatchMagic = 0x34484743u;  // "CGH4"
constexpr uint32_t kChunkTiles = 64;
struct HttpBatchHeader {
  uint32_t magic;
  uint32_t epoch;      // snapshot the batch was packed against
  uint32_t nchunks;
  uint32_t ntiles;
  uint64_t tiles_off;  // byte offset of the tile data (multiple of 1024)
  uint64_t nslots;
  uint64_t ttab_off;   // byte offset of the tile table (ntiles HttpTile)
  uint64_t total_bytes;
  uint64_t arena_bytes;  // overflow arena bytes the batch refers to (0: none)
  uint32_t pad[2];
};
struct HttpTile {
  uint32_t at;     // tile data at tiles_off + at * 512: the 512-byte meta block
  uint32_t units;  // (8 bytes per lane), then `units` 1 KiB string units (0..8) in bits 0..14;
                   // bit 15 (kTileHalfLast): the last of them is a 512-B half unit;
                   // bits 16..31: string bytes its lanes hold in the last unit (1..16), the
                   // rest of that unit being padding the walk may skip (0: walk all 16)
};
constexpr uint32_t kTileHalfLast = 0x8000u;
CG_HD inline uint32_t tile_units(const HttpTile& t) { return t.units & 0x7FFFu; }
CG_HD inline uint32_t tile_tail(const HttpTile& t) { return t.units >> 16; }
CG_HD inline bool tile_half(const HttpTile& t) { return (t.units & kTileHalfLast) != 0; }
// 512-byte granules of a tile's data: the meta block, two per full unit, one
// for a half unit
CG_HD inline uint32_t tile_granules(const HttpTile& t) { return 1 + 2 * tile_units(t) - (tile_half(t) ? 1u : 0u); }
struct HttpChunk {
  uint32_t prog;
  uint32_t first_tile;
  uint32_t ntiles;
  uint32_t pad;
};
struct HttpDev {
  const HttpProg* progs;
  const HttpPart* parts;
  const uint32_t* cells;
  const uint32_t* dflt;        // [policy*2 + ingress] → program id or kProg*
  uint32_t npolicies;
  uint32_t nprogs;
  uint32_t nparts;
  uint32_t epoch;
  uint32_t lds_cells;            // max cells a workgroup stages in LDS
  uint32_t n_global_progs;       // walked programs too large for LDS
  unsigned long long* counters;  // [prog*2] allowed, [prog*2+1] denied, [2*nprogs] stale batches
  unsigned long long* rule_hits; // counters + 2*nprogs + 1: first-match hits per rule
};

// ---- HTTP/1 raw heads → batch on the device (kernels_http_raw.hip) ----
// The packer's inputs derived on the GPU from raw request heads: the field
// values (http_parse.cc semantics), the program (HttpSnapshot::lookup_prog),
// the string and its class codes (http_pack.cc).  Fields beyond
// kRawMaxFields are not supported on this path (CG_UNSUPPORTED); heads longer
// than kRawMaxHead are rejected as Envoy's default 60 KiB header limit
// (max_request_headers_kb) rejects them.
constexpr uint32_t kRawMaxFields = 32;
constexpr uint32_t kRawMaxHead = 61440;
constexpr uint32_t kRawKeys = 10;  // bucket key: walked units 0..8, 9 = overflow arena
// The same machinery takes cg_http_pack's "name\0value\0" header lists
// (cg_http_verdicts_fields_*): value spans are 16-bit offsets into a
// request's list, so one list holds at most kFieldsMaxList bytes (Envoy's
// headers past its 60 KiB default limit never reach the filter).
constexpr uint32_t kFieldsMaxList = 65535;
struct HttpRawDev {
  const uint32_t* phash_keys;  // (policy << 17 | ingress << 16 | port) → program
  const uint32_t* phash_vals;
  uint32_t phash_mask;
  uint32_t npolicies;
  const uint32_t* dflt;        // [policy*2 + ingress]
  const HttpProg* progs;
  uint32_t nprogs;
  uint32_t nfields;
  int32_t f_method, f_path, f_authority;  // field index of each pseudo header, or -1
  uint32_t fmask;              // field-name table: fmask + 1 slots
  const uint32_t* fslots;      // per slot {FNV-1a of the lowercase name, name length (0 = empty), field, name offset}
  const uint8_t* fnames;       // lowercase names
  const uint8_t* codes;        // nprogs × 256: string byte → code (identity for byte-mode programs)
  // field names by their lowercase key (raw_name_key): per slot 8 u32 {length
  // (0 = empty), first 8 bytes (2 u32), last 8 bytes (2 u32; 0 when length
  // <= 8), field, name offset, 0}; nkmask + 1 slots
  const uint32_t* nkeys;
  uint32_t nkmask;
  uint32_t fnames_bytes;  // size of fnames
  const uint32_t* walk_bits;  // bit p: program p is walked (not allow-all)
  uint32_t raw_values;  // proxylib snapshot: header lists carry escaped values (http_pack.cc)
  int32_t f_empty;      // field index of the empty name, or -1 (header lists only)
};
// The key of a lowercase header name b[0, nl): its length, its first 8 bytes
// and (nl > 8) its last 8 bytes, little-endian, zero past the name.
CG_HD inline uint32_t raw_name_hash(uint32_t nl, uint32_t lo0, uint32_t lo1, uint32_t hi0, uint32_t hi1) {
  // rotate-xor fold, one 24-bit multiply (full rate on the GPU, unlike a
  // 32-bit one): the table has a few dozen slots, probed after
  uint32_t x = lo0 ^ (lo1 << 7 | lo1 >> 25) ^ (hi0 << 13 | hi0 >> 19) ^ (hi1 << 21 | hi1 >> 11) ^ nl;
  x ^= x >> 16;
  return ((x & 0xFFFFFFu) * 0x9E3779u) ^ (x >> 11);
}
// FNV-1a, 32 bit, over lowercase bytes
CG_HD inline uint32_t raw_fnv(uint32_t h, uint8_t c) { return (h ^ c) * 16777619u; }
constexpr uint32_t kRawFnvInit = 2166136261u;
// ---- the persistent verdict ring (cg_http_ring_*, ring.cc): Envoy-sized
// calls of header lists decided by a resident kernel that polls request
// slots — no launch, no copies, no stream synchronization per call.  A
// request slot holds one call: a 64-byte header {seq (the host's doorbell),
// served (the last seq the device answered), n, bytes}, the per-request
// inputs, list offsets relative to the slot's blob and the blob.  The request
// slots live in fine-grained DEVICE memory the host writes through its
// mapping (the kernel polls and reads them locally; the host's writes are
// posted), the reply slots {done word 1, phase stamps, verdicts at kRingOut}
// in pinned host memory the host polls; CILIUM_GPU_RING_SLOTS=host keeps both
// in one pinned host slot (reply == request).
constexpr uint32_t kRingReqs = 256;          // requests per slot (larger calls take the staged path)
constexpr uint32_t kRingBlob = 32 * 1024;    // list bytes per slot
// A slot: [header: 64 B][verdicts: kRingReqs B][data], the data packed for
// the call's n so a small call is a few hundred contiguous bytes (one round
// of 16-byte loads over the bus): policy[n] u32, remote[n] u32, port[n] u16,
// ingress[n] u8 (each padded to 4 bytes), list offsets[n + 1] u32 relative
// to the blob, the blob from the next 16-byte boundary.
constexpr size_t kRingOut = 64, kRingData = kRingOut + kRingReqs;
struct RingLayout {
  uint32_t rem, port, ing, off, blob;  // byte offsets in the data
};
CG_HD inline RingLayout ring_layout(uint32_t n) {
  RingLayout L;
  L.rem = 4 * n;
  L.port = 8 * n;
  L.ing = L.port + ((2 * n + 3) & ~3u);
  L.off = L.ing + ((n + 3) & ~3u);
  L.blob = (L.off + 4 * (n + 1) + 15) & ~15u;
  return L;
}
constexpr size_t kRingDataMax = ((15 * kRingReqs + 4 + 16) & ~(size_t)15) + kRingBlob;
constexpr size_t kRingSlotBytes = (kRingData + kRingDataMax + 255) & ~(size_t)255;
static_assert(kRingData % 16 == 0, "the data is copied in 16-byte units");
// ring control words (host memory, before the slots): the host's stop word
// (the device only reads host memory with loads and writes it with plain
// stores: no read-modify-write over the bus)
constexpr uint32_t kRingStop = 0, kRingCtlBytes = 256;
constexpr size_t kRingReplyBytes = 512;       // [header: 64 B (done: word 1, stamps)][verdicts]
static_assert(kRingOut + kRingReqs <= kRingReplyBytes, "reply slot");
struct HttpRingDev {
  uint8_t* slots;         // request slots (device memory, or the device view of host slots), kRingSlotBytes apart
  uint8_t* reply;         // reply slots (device view of pinned host memory), reply_stride apart
  uint32_t reply_stride;  // kRingReplyBytes, or kRingSlotBytes when reply == slots
  uint32_t* ctl;          // device view of the control words
  uint32_t nslots, nwg;   // slot s is served by workgroup s % nwg
  uint64_t idle_ticks;    // wall-clock ticks without a call before the kernel exits
  uint64_t life_ticks;    // hard bound on one launch's life
  uint32_t lds_cells;     // largest program block the kernel stages in LDS (0: none)
  uint32_t trace;         // write phase stamps into slot words 8..14 (CILIUM_GPU_RING_TRACE)
  uint32_t echo;          // transport experiments (CILIUM_GPU_RING_ECHO): 1 done at once, 2 after the data; 0 serve
  uint32_t lds_tabs;      // the list parser's lookup tables staged in LDS (ring_lds_bytes)
};
// phase stamps of a served call (low 32 bits of wall_clock64): polled,
// data and list masks in LDS, program looked up / staged, request 0 parsed,
// its string emitted, verdicts written, released
constexpr uint32_t kRingStampAt = 8, kRingStamps = 7;

// A run of tiles of a raw batch with the same string units and program:
// tiles [t0, next run's t0), tile t at granule base + (t - t0) * (1 + 2 * units).
struct HttpRawRun {
  uint32_t t0, units, base, prog;
  uint32_t send;  // one past the last real slot of the run's group (later slots are padding)
};

// bucket key of a request on the device-layout path: its group (program,
// then allow and deny) x its walked string's 16-byte units (0..8); longer
// strings are walked by raw_walk_kernel, not slotted
constexpr uint32_t kRawUnits = 9;
// The raw path's device-built batch (kernels_http_raw.hip, http_raw.cc): the
// scan takes slot s of bucket key k from a per-key counter; slots come in
// chunks of 64 * ext (ext tiles, a power of two <= kChunkTiles), the first
// slot of a chunk takes a chunk id from ctl[kRawCtlChunks] and publishes it
// in dir[k * dpk + c] as seq << 32 | id (seq: the sub-batch's tag, so the
// directory is never cleared).  Tile t = id * ext + (s / 64) % ext keeps its
// data at granule t * kRawTileGran (room for 8 units), slot s % 64.
constexpr uint32_t kRawTileGran = 1 + 2 * 8;
// threads per workgroup of the raw scan kernels (the device layout's
// directory bound counts grid-stride iterations of this many requests)
constexpr uint32_t kRawScanThreads = 256;
constexpr uint32_t kRawCntStride = 64;  // u32 between two keys' counters (own 256-B line)
enum : uint32_t {
  kRawCtlChunks = 0,  // chunk ids taken
  kRawCtlWalk = 1,    // requests on the walk list (raw_walk_kernel)
  kRawCtlDefer = 2,   // requests on the deferred list (heads outside their wave's stage)
  kRawCtlError = 3,   // bit 0: a chunk past the layout's bounds (its requests walked instead)
                      // bit 1: a slot whose chunk id was not seen in time (late list)
  kRawCtlLate = 4,    // slots on the late list
  kRawCtlWords = 16
};
struct RawLayoutDev {
  uint32_t* kcnt;            // [key * kRawCntStride] slots taken
  unsigned long long* dir;   // [key * dpk + c]
  HttpChunk* chunks;         // in id order: {prog, first tile, ntiles, key} (raw_seal_kernel sorts them)
  HttpTile* ttab;            // units | tail << 16 by atomicMax (zeroed per sub-batch), at by the slot-0 lane
  uint8_t* tiles;            // tile data
  uint32_t* order;           // slot → request index
  uint32_t* ctl;             // kRawCtl*
  uint32_t* walk;            // request indices for raw_walk_kernel
  uint32_t* dlist;           // request indices for raw_defer_kernel
  // slots taken whose lane gave up waiting for the chunk id (key << 32 | s):
  // the request is walked, and raw_seal_kernel pads the slot once every id
  // is published, so http_kernel never reads an unfilled slot
  unsigned long long* late;
  uint32_t dpk, ext, cshift; // directory entries per key, tiles per chunk, log2(64 * ext)
  uint32_t seq, maxchunks, nkeys;
  uint32_t spin;             // polls of a chunk id before giving up (CILIUM_GPU_RAW_SPIN, tests)
  // slot counters per bucket key and stripe: a workgroup takes its slots from
  // stripe blockIdx % stripes of its key (vkey = key * stripes + stripe), so
  // each hot key's returning atomics spread over `stripes` addresses
  uint32_t stripes;
};
// the stripe-expanded bucket key of a request of key k in workgroup b
CG_HD inline uint32_t raw_vkey(const RawLayoutDev& L, uint32_t k, uint32_t b) { return k * L.stripes + (b & (L.stripes - 1u)); }

CG_HD inline uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
// Remote-identity table of a program (staged into LDS with it): buckets of
// 8 u32 cells — 4 identities, then their 4 mask-row block offsets — and
// every identity in one of its two buckets, so a lookup reads at most two
// buckets (2-choice cuckoo, load up to ~90%: no power-of-two padding and no
// probe chains).  An empty slot holds the program's `rtab_empty` identity
// (one not in its table) with the default row, so matching it changes
// nothing and the kernel needs no emptiness test.  The bucket hashes use
// 24-bit multiplies only (full-rate v_mul_u32_u24 / v_mul_hi_u32_u24; the
// 32-bit ones issue at a quarter rate) and scale to [0, nb), nb < 65536.
constexpr uint32_t kRtabBucketCells = 8;
CG_HD inline uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul24(a, b);
#else
  return (a & 0xFFFFFFu) * (b & 0xFFFFFFu);
#endif
}
CG_HD inline uint32_t mulhi24(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)(a & 0xFFFFFFu) * (b & 0xFFFFFFu)) >> 32);
}
CG_HD inline uint32_t rtab_hash(uint32_t id) {
  const uint32_t a = id ^ (id >> 15);
  return mul24(a, 0x9E3779u) ^ (a >> 17);
}
CG_HD inline uint32_t rtab_b1h(uint32_t h, uint32_t nb) { return mulhi24(h, nb << 8); }
CG_HD inline uint32_t rtab_b2h(uint32_t h, uint32_t nb) {
  return mulhi24(mul24(h ^ (h >> 11), 0x85EBCBu) >> 8, nb << 8);  // product bits 8..31
}
CG_HD inline uint32_t rtab_b1(uint32_t id, uint32_t nb) { return rtab_b1h(rtab_hash(id), nb); }
CG_HD inline uint32_t rtab_b2(uint32_t id, uint32_t nb) { return rtab_b2h(rtab_hash(id), nb); }

CG_HD inline uint32_t hash64to32(uint64_t k) {
  k = l4_hash1(k);
  return (uint32_t)k;
}

// --------------------------------------------------------------- Kafka ----
// Per (redirect, identity group) the rule set is compiled into decision
// summaries, one per (context, apiKey bucket): context 0 = the request has
// topics (only topic-less rules apply unconditionally), 1 = it has none (every
// rule applies); bucket = apiKey for 0..63, 64 for any other key (only
// apiKey-wildcard rules reach it).  A summary answers ruleMatches for all its
// rules at once per request class (typed / consumer-metadata / nil): `any`
// bit c = some rule matches every version, vm[c] bit v = some rule matches
// version v.  Rules the bits cannot express (a clientID that must be compared,
// a version outside 0..63) are kept as exception rules, evaluated one by one.
// Topic rules are reached per (group, topic) through a hash table.
struct KafkaRuleDev {
  unsigned long long keys;  // bit k: apiKey k allowed (k < 64)
  uint32_t flags;           // kKf* bits
  int32_t version;
  uint32_t client_id;
  uint32_t pad;
};
constexpr uint32_t kKfKeyWild = 1, kKfVerWild = 2, kKfHasClient = 4, kKfHasTopic = 8;
// Kafka table hash over a (hi, lo) u32 key pair: 32-bit multiplies only.
CG_HD inline uint32_t kf_hash(uint64_t k) {
  return l4_fin((uint32_t)k * kL4MulLo + (uint32_t)(k >> 32) * kL4MulHi);
}
constexpr uint32_t kKfBuckets = 65;                // apiKey 0..63 + "other"
constexpr uint32_t kKfSumsPerGroup = 2 * kKfBuckets;
struct KafkaSumDev {
  unsigned long long vm[3];  // class 0 typed, 1 consumer-metadata, 2 nil: versions 0..63
  uint32_t any;              // bit c: class c matches any version; bit 3: has clientID entries
  uint32_t x_off, x_cnt;     // exception rules (KafkaRuleDev index range)
  uint32_t pad;
};
constexpr uint32_t kKfSumHasClients = 8;
// Typed requests against clientID rules: per (summary, clientID) the versions
// those rules accept, so the comparison is one hash probe.
struct KafkaClientDev {
  unsigned long long key;    // summary index<<32 | client id; ~0 = empty
  unsigned long long vm;     // versions 0..63
  uint32_t any, pad[3];      // any: some rule accepts every version
};
struct KafkaGroupSlot {
  unsigned long long key;    // redirect<<32 | identity; ~0 = empty
  uint32_t group, pad;
};
struct KafkaTopicDev {
  unsigned long long key;    // group<<32 | topic id; ~0 = empty
  uint32_t off, cnt;         // KafkaRuleDev index range (rules with this Topic)
};
struct KafkaDev {
  const KafkaSumDev* sums;        // [group * kKfSumsPerGroup + ctx * kKfBuckets + bucket]
  const KafkaRuleDev* rules;
  const KafkaTopicDev* thash;
  uint32_t thash_mask;
  const KafkaClientDev* chash;
  uint32_t chash_mask;
  const KafkaGroupSlot* ghash;    // (redirect, identity) → group
  uint32_t ghash_mask;
  const uint32_t* dflt_group;     // per redirect: group for unlisted identities
  uint32_t nredirects;
  unsigned long long* counters;   // [redirect*2] allowed, [+1] denied
};

// Rule strings (topics, clientIDs) for interning on the device: open
// addressing over FNV-1a, 32-byte slots {hash, len (~0 empty), id, blob
// offset of the bytes past the first 16, the first 16 bytes zero-padded}.
constexpr uint32_t kKfDictSlotWords = 8;
struct KafkaDictDev {
  const uint32_t* slots;  // kKfDictSlotWords u32 per slot
  const uint8_t* blob;
  uint32_t mask, pad;
};
constexpr uint32_t kKfDictEmpty = 0xFFFFFFFFu;
CG_HD inline uint32_t kf_fnv1a(const uint8_t* p, uint32_t n) {
  uint32_t h = 2166136261u;
  for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 16777619u;
  return h;
}

// ------------------------------------------------------------- ipcache ----
// cilium_ipcache (bpf/lib/maps.h:135-159), looked up by
// lookup_ip{4,6}_remote_endpoint (bpf/lib/eps.h:48-115) and resolved as the
// callers do (bpf_lxc.c:509-518): hit with sec_label != 0 → {sec_label,
// tunnel_endpoint}, else {WORLD_ID, 0}.
//
// Table entries hold that resolved pair inline as a u64 (identity in the low
// word, tunnel in the high word), so a lookup ends at its last table level.
// A resolved identity is never 0, so identity 0 marks a pointer: the high
// word is then the index of the next level's 256-entry chunk.
//  IPv4: 16-8-8 stride trie of 2-KiB chunks under a 16-B summary per /16
//        (1 MiB, mostly L2 resident): {background value (identity, tunnel),
//        chunk, lo | hi << 8 | direct << 16}.  /24 indices outside [lo, hi]
//        resolve to the background without touching a chunk (most /16 chunks
//        hold one short range: a node's /24, a /17../28 prefix); inside it
//        the chunk's entry is read, and a pointer there leads to the /32
//        chunk.  direct: the range is one /24 whose entry is a pointer, and
//        chunk names its /32 chunk, skipping a level.
//  IPv6: the prefixes partition the address space into runs with one
//        longest-prefix value each; runs are 32-B records {start hi, start lo,
//        value, 0} sorted by start.  The top v6_bits address bits pick a
//        bucket; a bit per bucket (32 per u64 word, the high half counting
//        the set bits before the word: 256 KiB at 2^20 buckets, L2
//        resident) is clear when one WORLD run spans the whole bucket, which
//        settles the lookup.  A set bucket's 16-B ent6 entry is {L, R, crowd,
//        0}: runs L..R meet the bucket.  A node's /64 of pods crowds ~50
//        runs into one bucket; such a bucket (8..255 runs) names a 128-B
//        crowd6 line {prefix P of the starts of runs L+1..R (top s bits),
//        s, 65 u8 offsets from L}: the 6 address bits after P pick one of 64
//        sub-ranges, cutting a ~6-step binary search to about one record.
constexpr uint32_t kWorldId = 2;  // bpf/node_config.h:35
constexpr uint64_t kIpcMiss = kWorldId;  // {WORLD_ID, 0}
struct alignas(8) IpcVal {
  uint32_t identity;
  uint32_t tunnel;  // tunnel_endpoint as stored (network-order bytes)
};
struct IpcacheDev {
  const uint32_t* l16x;    // 4 words per /16 (16-B aligned)
  const uint64_t* chunks;  // encoded 256-entry chunks (ipc_chunk_get), 64-byte units
  const uint64_t* code6;   // (1 << v6_bits) / 32 words
  const uint32_t* ent6;    // {L, R, crowd, 0} per set bucket (at least one entry)
  const uint8_t* crowd6;   // 128 B per crowded bucket (kIpcNoCrowd: none)
  const uint64_t* runs6;   // 4 u64 per run
  uint32_t v6_bits;
  uint32_t nruns6;
  // the /32 and /128 entries, by exact match (a full-length prefix is the
  // longest one covering its address): open addressing, linear probing at
  // load <= 1/2; a v4 slot {address, used, entry lo, entry hi}, a v6 slot
  // {address hi, address lo, entry, used} (u64 words); ex*_probes bounds
  // every search (the longest probe sequence the build made)
  const uint32_t* ex4;
  const uint64_t* ex6;
  uint32_t ex4_mask, ex6_mask, ex4_probes, ex6_probes;
};
// summary flag (l16x word 3): the /16 holds exact /32 entries
constexpr uint32_t kIpcExact = 1u << 17;
CG_HD inline uint32_t ipc_ex4_hash(uint32_t a) {
  a ^= a >> 16;
  a *= 0x7FEB352Du;
  a ^= a >> 15;
  a *= 0x846CA68Bu;
  return a ^ (a >> 16);
}
CG_HD inline uint32_t ipc_ex6_hash(uint64_t hi, uint64_t lo) {
  uint64_t x = hi * 0x9E3779B97F4A7C15ull ^ lo;
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  return (uint32_t)(x >> 32);
}
// The exact /32 entry of a (host order): 1 found (*e), 0 not there.
CG_HD inline int ipc_ex4_find(const IpcacheDev& t, uint32_t a, uint32_t h, uint64_t* e) {
  for (uint32_t p = 0; p <= t.ex4_probes; ++p) {
    const uint32_t* s = t.ex4 + 4 * (size_t)((h + p) & t.ex4_mask);
    if (!s[1]) return 0;
    if (s[0] == a) {
      *e = (uint64_t)s[3] << 32 | s[2];
      return 1;
    }
  }
  return 0;
}
CG_HD inline int ipc_ex6_find(const IpcacheDev& t, uint64_t hi, uint64_t lo, uint32_t h, uint64_t* e) {
  for (uint32_t p = 0; p <= t.ex6_probes; ++p) {
    const uint64_t* s = t.ex6 + 4 * (size_t)((h + p) & t.ex6_mask);
    if (!s[3]) return 0;
    if (s[0] == hi && s[1] == lo) {
      *e = s[2];
      return 1;
    }
  }
  return 0;
}

// ---- IPv4: 256-entry chunks in one of three encodings (ipcache.cc) ------
// An entry is a resolved {identity, tunnel} (identity != 0) or a pointer to
// a /32-level chunk (low word 0, high word = a chunk reference).  A chunk
// reference is kind << 30 | offset, the offset in 64-byte units of
// IpcacheDev.chunks:
//   DENSE   256 u64 entries (2 KiB)
//   RUNS    one 64-byte line: word 0 = {run count n <= 7, the starts of runs
//           1..n-1 as bytes 1..6}, words 1..7 the runs' entries — a chunk of
//           a few prefixes (most /16s hold one or two CIDR prefixes)
//   SPARSE  words 0-4: bits 0-55 of word w a map of keys 56w..56w+55 whose
//           entry is not the base, bits 56-63 the keys set in words < w;
//           word 5 the base entry, words 6.. the set keys' entries in key
//           order — a node's /24 of pod /32s (~60 of 256 set: 530 B, not 2 KiB)
// so the hot part of the table (summaries, run lines, pod maps) is a few MB:
// an XCD's L2, where the dense form was 139 MB at the bench's 512K entries.
constexpr uint32_t kIpcDense = 0, kIpcRuns = 1, kIpcSparse = 2;
CG_HD inline uint32_t ipc_runs_index(uint64_t w0, uint32_t key) {
  const uint32_t n = (uint32_t)(w0 & 0xFF);
  uint32_t idx = 0;
  for (uint32_t i = 1; i < 7; ++i) idx += (uint32_t)(i < n) & (uint32_t)(((w0 >> (8 * i)) & 0xFF) <= key);
  return idx;
}
// A chunk entry in two rounds of loads (the kernels issue each round for all
// of a lane's addresses before the next): round 1 reads the aligned 16-byte
// word pair at ipc_chunk_first (the entry's pair; run word 0 and the first
// run's entry; the map word holding the key); ipc_chunk_mid settles the
// entry from it or names the word round 2 reads (~0u: settled).  Word
// offsets are 32-bit: the builder keeps the encoded table under 2^32 words.
struct alignas(16) IpcPair {
  uint64_t lo, hi;
};
CG_HD inline uint32_t ipc_chunk_first(uint32_t ref, uint32_t key) {
  const uint32_t b = (ref & 0x3FFFFFFFu) * 8;
  const uint32_t kind = ref >> 30;
  return b + (kind == kIpcDense ? (key & ~1u) : kind == kIpcRuns ? 0u : ((key / 56) & ~1u));
}
CG_HD inline uint64_t ipc_chunk_mid(uint32_t ref, uint32_t key, IpcPair A, uint32_t* vword) {
  const uint32_t b = (ref & 0x3FFFFFFFu) * 8;
  const uint32_t kind = ref >> 30;
  *vword = ~0u;
  if (kind == kIpcDense) return (key & 1) ? A.hi : A.lo;
  if (kind == kIpcRuns) {
    const uint32_t idx = ipc_runs_index(A.lo, key);
    if (idx) *vword = b + 1 + idx;
    return A.hi;
  }
  const uint32_t wi = key / 56, bit = key - 56 * wi;
  const uint64_t w = (wi & 1) ? A.hi : A.lo;
  *vword = ((w >> bit) & 1) ? b + 6 + (uint32_t)(w >> 56) + (uint32_t)__builtin_popcountll(w & ((1ull << bit) - 1))
                            : b + 5;
  return 0;
}
CG_HD inline uint64_t ipc_chunk_get(const uint64_t* ch, uint32_t ref, uint32_t key) {
  uint32_t v;
  const uint64_t r = ipc_chunk_mid(ref, key, *reinterpret_cast<const IpcPair*>(ch + ipc_chunk_first(ref, key)), &v);
  return v == ~0u ? r : ch[v];
}
// The /16 summary {background, chunk reference, lo | hi << 8 | direct << 16}:
// an address whose /24 lies outside [lo, hi] has the background value; else
// its entry is key (a >> 8) & 255 of the chunk, or — direct: the /16's only
// non-background /24 points to a /32 chunk, named by the summary — key a & 255.
CG_HD inline bool ipc_v4_in(uint32_t r, uint32_t a) {
  const uint32_t k = (a >> 8) & 255;
  return k >= (r & 255) && k <= ((r >> 8) & 255);
}
CG_HD inline uint32_t ipc_v4_key(uint32_t r, uint32_t a) { return ((r >> 16) & 1) ? (a & 255) : ((a >> 8) & 255); }
// K chunk reads at once, each round's loads issued for all K before the
// next round (the kernels' form of ipc_chunk_get); a lane reads the round-2
// word only when its entry needs it.
template <uint32_t K>
CG_HD inline void ipc_chunk_rounds(const uint64_t* __restrict__ ch, const uint32_t (&ref)[K],
                                   const uint32_t (&key)[K], uint64_t (&out)[K]) {
  uint32_t vw[K];
  IpcPair A[K];
#pragma unroll
  for (uint32_t u = 0; u < K; ++u) A[u] = *reinterpret_cast<const IpcPair*>(ch + ipc_chunk_first(ref[u], key[u]));
#pragma unroll
  for (uint32_t u = 0; u < K; ++u) out[u] = ipc_chunk_mid(ref[u], key[u], A[u], &vw[u]);
#pragma unroll
  for (uint32_t u = 0; u < K; ++u)
    if (vw[u] != ~0u) out[u] = ch[vw[u]];
}
// K IPv4 addresses (host order) → their resolved entries: the summaries, the
// /24-level chunk (or the direct /32 chunk), then the /32-level chunk for
// the addresses whose entry is a pointer.
template <uint32_t K>
CG_HD inline void ipc_v4_resolve(const IpcacheDev& t, const uint32_t (&a)[K], uint64_t (&e)[K]) {
  uint32_t ref[K], key[K];
  bool in[K], ex[K];
  IpcPair x[K];
#pragma unroll
  for (uint32_t u = 0; u < K; ++u) x[u] = *reinterpret_cast<const IpcPair*>(t.l16x + 4 * (size_t)(a[u] >> 16));
#pragma unroll
  for (uint32_t u = 0; u < K; ++u) {
    const uint32_t r = (uint32_t)(x[u].hi >> 32);
    in[u] = ipc_v4_in(r, a[u]);
    ex[u] = (r & kIpcExact) != 0;
    e[u] = x[u].lo;
    ref[u] = in[u] ? (uint32_t)x[u].hi : 0u;
    key[u] = ipc_v4_key(r, a[u]);
  }
  // a /16 holding /32 entries: the exact table's first slot, loaded in the
  // chunk round (a hit is the answer; a used slot of another address
  // continues the probe sequence)
  uint32_t hx[K];
  IpcPair sx[K];
#pragma unroll
  for (uint32_t u = 0; u < K; ++u) {
    hx[u] = ipc_ex4_hash(a[u]) & t.ex4_mask;
    sx[u] = IpcPair{0, 0};
    if (ex[u]) sx[u] = *reinterpret_cast<const IpcPair*>(t.ex4 + 4 * (size_t)hx[u]);
  }
  uint64_t r[K];
  ipc_chunk_rounds<K>(t.chunks, ref, key, r);
#pragma unroll
  for (uint32_t u = 0; u < K; ++u) {
    if (!ex[u] || (uint32_t)(sx[u].lo >> 32) == 0) continue;  // no exact entry here
    uint64_t v;
    if ((uint32_t)sx[u].lo == a[u] ? (v = sx[u].hi, true) : ipc_ex4_find(t, a[u], hx[u] + 1, &v)) {
      e[u] = v;
      in[u] = false;  // settled: the longest prefix
    }
  }
  bool ptr[K], any = false;
#pragma unroll
  for (uint32_t u = 0; u < K; ++u) {
    ptr[u] = in[u] && (uint32_t)r[u] == 0;
    any |= ptr[u];
    ref[u] = ptr[u] ? (uint32_t)(r[u] >> 32) : 0u;
    key[u] = a[u] & 255;
    if (in[u]) e[u] = r[u];
  }
  if (any) {
    ipc_chunk_rounds<K>(t.chunks, ref, key, r);
#pragma unroll
    for (uint32_t u = 0; u < K; ++u)
      if (ptr[u]) e[u] = r[u];
  }
}
CG_HD inline uint64_t ipc_v4_value(const IpcacheDev& t, uint32_t a) {  // a in host order
  const uint32_t* x = t.l16x + 4 * (size_t)(a >> 16);
  uint64_t ev;
  if ((x[3] & kIpcExact) && ipc_ex4_find(t, a, ipc_ex4_hash(a) & t.ex4_mask, &ev)) return ev;
  if (!ipc_v4_in(x[3], a)) return (uint64_t)x[1] << 32 | x[0];
  uint64_t e = ipc_chunk_get(t.chunks, x[2], ipc_v4_key(x[3], a));
  if ((uint32_t)e == 0) e = ipc_chunk_get(t.chunks, (uint32_t)(e >> 32), a & 255);
  return e;
}

CG_HD inline bool ipc_le128(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
  return ah < bh || (ah == bh && al <= bl);
}

// IPv6 bucket tb of code word cw: false when one WORLD run spans it; else
// *idx = its ent6 index.
CG_HD inline bool ipc_v6_bucket(uint64_t cw, uint32_t tb, uint32_t* idx) {
  const uint32_t w = (uint32_t)cw, b = tb & 31;
  *idx = (uint32_t)(cw >> 32) + (uint32_t)__builtin_popcount(w & ((1u << b) - 1));
  return (w >> b) & 1;
}

constexpr uint32_t kIpcNoCrowd = 0xFFFFFFFFu;
// Where (hi, lo) falls against a crowd line's window (prefix P, top s bits):
// 0 before it (the answer is run L), 1 after it (run R), 2 inside it, with
// *i the sub-range of the 6 bits below P.
CG_HD inline uint32_t ipc_v6_window(uint64_t ph, uint64_t pl, uint32_t s, uint64_t hi, uint64_t lo, uint32_t* i) {
  const uint64_t mh = s >= 64 ? ~0ULL : ~0ULL << (64 - s), ml = s > 64 ? ~0ULL << (128 - s) : 0;
  const uint64_t ah = hi & mh, al = lo & ml;
  if (ah < ph || (ah == ph && al < pl)) return 0;
  if (ah > ph || (ah == ph && al > pl)) return 1;
  const uint32_t sh = 122 - s;  // s in 1..122
  *i = (uint32_t)((sh >= 64 ? hi >> (sh - 64) : sh == 0 ? lo : (lo >> sh) | (hi << (64 - sh))) & 63);
  return 2;
}
// Narrow a crowded bucket's run range [*L, *R] for address (hi, lo) with its
// crowd6 line d (runs L+1..R start inside the window of prefix P).
CG_HD inline void ipc_v6_narrow(const uint8_t* d, uint64_t hi, uint64_t lo, uint32_t* L, uint32_t* R) {
  uint32_t i = 0;
  const uint32_t w = ipc_v6_window(reinterpret_cast<const uint64_t*>(d)[0], reinterpret_cast<const uint64_t*>(d)[1],
                                   reinterpret_cast<const uint32_t*>(d)[4], hi, lo, &i);
  if (w == 0) {
    *R = *L;
  } else if (w == 1) {
    *L = *R;
  } else {
    const uint32_t base = *L;
    *L = base + d[24 + i];
    *R = base + d[25 + i];
  }
}

// Last run whose start is <= (hi, lo), searched in [L, R] (run L qualifies).
CG_HD inline uint32_t ipc_v6_run(const IpcacheDev& t, uint64_t hi, uint64_t lo, uint32_t L, uint32_t R) {
  while (L < R) {
    const uint32_t m = (L + R + 1) >> 1;
    if (ipc_le128(t.runs6[4 * (size_t)m], t.runs6[4 * (size_t)m + 1], hi, lo)) L = m;
    else R = m - 1;
  }
  return L;
}

// A set bucket's value when its last run R starts after the address: the
// search over [L, R - 1], narrowed first in a crowded bucket.
CG_HD inline uint64_t ipc_v6_search_value(const IpcacheDev& t, uint64_t hi, uint64_t lo, uint32_t L, uint32_t R,
                                          uint32_t crowd) {
  uint32_t l = L, r = R - 1;
  if (crowd != kIpcNoCrowd) {
    uint32_t rr = R;
    ipc_v6_narrow(t.crowd6 + 128 * (size_t)crowd, hi, lo, &l, &rr);
    r = rr < R - 1 ? rr : R - 1;
    l = l < r ? l : r;
  }
  return t.runs6[4 * (size_t)ipc_v6_run(t, hi, lo, l, r) + 2];
}

}  // namespace cg
