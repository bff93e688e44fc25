// http_pack.cc — program-grouped request batches and the host table walker.
//
// The packer resolves each request's program on the host (the lookup the
// reference does per request in PortNetworkPolicy::Matches,
// envoy/cilium_network_policy.h:169-192), groups requests by program and
// pads every group to whole 64-request tiles, so each chunk of tiles has one
// program whose comb table a workgroup stages in LDS.  A tile holds the meta
// unit and only as many 16-byte string units as its longest string needs
// (the tile table gives each tile's offset and unit count), so the batch is
// as large as its strings, not as the 128-byte slot.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>
#include <exception>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <atomic>
#include <cstddef>
#include <array>
#include <cstring>
#include <map>
#include <string>

#include "comb.h"
#include "http.h"

namespace cg {

namespace {

constexpr uint8_t kSep = 0x00;
constexpr uint8_t kAbsent = 0x01;
constexpr uint8_t kRestAbsent = 0x02;  // every remaining field absent (http.cc)

// A header value byte Envoy's HTTP/1 codec rejects (http_parser's
// IS_HEADER_CHAR: control bytes other than HTAB, and DEL); the request never
// reaches the L7 filter.
inline bool codec_rejects(uint8_t c) { return (c < 0x20 && c != 0x09) || c == 0x7F; }
constexpr size_t kUnitBytes = (size_t)CG_HTTP_TILE * 16;  // one string unit of a tile: 1 KiB
constexpr size_t kMetaBytes = (size_t)CG_HTTP_TILE * CG_HTTP_META_BYTES;  // the tile's meta block: 512 B
constexpr size_t kGranule = 512;  // tile offsets count 512-byte granules
constexpr size_t kMaxTileBytes = kMetaBytes + (size_t)(CG_HTTP_UNITS - 1) * kUnitBytes;

// byte offset of unit u (0 = meta block) of tile t, lane l (its last unit
// a half unit of 8 bytes per lane when tile_half)
inline size_t tile_unit_at(const HttpTile& t, uint32_t u, size_t lane) {
  const bool half = u && u == tile_units(t) && tile_half(t);
  return (size_t)t.at * kGranule +
         (u ? kMetaBytes + (size_t)(u - 1) * kUnitBytes + lane * (half ? 8 : 16) : lane * CG_HTTP_META_BYTES);
}

bool name_eq_ci(const uint8_t* a, size_t an, const std::string& lower_b) {
  if (an != lower_b.size()) return false;
  for (size_t i = 0; i < an; ++i) {
    uint8_t c = a[i];
    if (c >= 'A' && c <= 'Z') c = c - 'A' + 'a';
    if (c != (uint8_t)lower_b[i]) return false;
  }
  return true;
}

size_t max_groups(const HttpSnapshot& s, size_t n) { return std::min(n, s.progs.size() + 2); }

// chunk table, then the tile table, then (1 KiB aligned) the tile data
size_t ttab_off(size_t max_tiles) { return sizeof(HttpBatchHeader) + sizeof(HttpChunk) * max_tiles; }
size_t header_bytes(size_t max_tiles) {
  size_t b = ttab_off(max_tiles) + sizeof(HttpTile) * max_tiles;
  return (b + 1023) & ~(size_t)1023;
}

}  // namespace

size_t http_batch_slots(const HttpSnapshot& s, size_t n) {
  return ((n + CG_HTTP_TILE - 1) / CG_HTTP_TILE + max_groups(s, n)) * CG_HTTP_TILE;
}

size_t http_batch_bytes(const HttpSnapshot& s, size_t n) {
  size_t tiles = http_batch_slots(s, n) / CG_HTTP_TILE;
  return header_bytes(tiles) + tiles * kMaxTileBytes;
}

namespace {

// Worker threads for the packer: CILIUM_GPU_PACK_THREADS, else the hardware
// threads (at most 16); small batches stay on the calling thread.
unsigned pack_threads(size_t n) {
  if (n < 16384) return 1;
  static const unsigned t = [] {
    if (const char* e = getenv("CILIUM_GPU_PACK_THREADS")) {
      const long v = strtol(e, nullptr, 10);
      if (v >= 1 && v <= 256) return (unsigned)v;
    }
    return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  }();
  return t;
}

// fn(begin, end, worker) over [0, n) in `nt` contiguous ranges.
template <class F>
void parallel_ranges(size_t n, unsigned nt, F&& fn) {
  if (nt <= 1 || n == 0) {
    fn((size_t)0, n, 0u);
    return;
  }
  std::vector<std::thread> th;
  std::exception_ptr err;
  std::mutex mu;
  for (unsigned t = 0; t < nt; ++t) {
    const size_t a = n * t / nt, b = n * (t + 1) / nt;
    th.emplace_back([&, a, b, t] {
      try {
        fn(a, b, t);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu);
        if (!err) err = std::current_exception();
      }
    });
  }
  for (auto& x : th) x.join();
  if (err) std::rethrow_exception(err);
}

// fn(item) for items [0, n) taken dynamically by `nt` workers.
template <class F>
void parallel_items(size_t n, unsigned nt, F&& fn) {
  std::atomic<size_t> next{0};
  parallel_ranges(nt, nt, [&](size_t, size_t, unsigned) {
    for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
  });
}

}  // namespace

void http_pack(const HttpSnapshot& s, size_t n, const uint32_t* policy, const uint8_t* ingress,
               const uint16_t* port, const uint32_t* remote, const uint8_t* hdr_blob,
               const uint64_t* hdr_off, void* batch, size_t batch_cap, uint32_t* order, size_t* nslots_out,
               uint8_t* arena, size_t arena_cap, size_t* arena_used) {
  const unsigned nt = pack_threads(n);
  const bool build = batch || arena_used;
  const bool dbg = getenv("CILIUM_GPU_PACK_DEBUG") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!dbg) return;
    auto t1 = std::chrono::steady_clock::now();
    fprintf(stderr, "[pack] %-10s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
    t0 = t1;
  };
  // program groups are laid out in ascending program id, the two special
  // ids (allow, deny) last: group index gi
  const size_t np = s.progs.size();
  auto group_of = [&](uint32_t p) -> size_t { return p < np ? p : np + (p == kProgAllow ? 0 : 1); };
  auto prog_of_group = [&](size_t g) -> uint32_t { return g < np ? (uint32_t)g : g == np ? kProgAllow : kProgDeny; };
  // ---- per request (parallel): program, walked string (field values in
  // field order, SEP-terminated, class-coded for class-mode programs),
  // codec verdict.  Each worker appends its strings to its own buffer.
  const size_t F = s.fields.size();
  std::vector<std::vector<uint8_t>> sbuf(nt);
  std::vector<uint32_t> prog(n), soff(n), slen(n);
  std::vector<uint8_t> malformed(n, 0);
  std::vector<std::vector<size_t>> gcount(nt, std::vector<size_t>(np + 2, 0));
  // fields by name length: a header name is compared with same-length fields only
  std::vector<std::vector<uint32_t>> by_len;
  for (size_t f = 0; f < F; ++f) {
    const size_t L = s.fields[f].size();
    if (by_len.size() <= L) by_len.resize(L + 1);
    by_len[L].push_back((uint32_t)f);
  }
  auto worker_of = [&](size_t i) -> unsigned {
    // parallel_ranges splits [0, n) at n*t/nt
    unsigned t = (unsigned)((i * nt) / n);
    while (t + 1 < nt && i >= n * (t + 1) / nt) ++t;
    while (t > 0 && i < n * t / nt) --t;
    return t;
  };
  parallel_ranges(n, nt, [&](size_t a, size_t b, unsigned t) {
    std::vector<uint8_t>& strs = sbuf[t];
    if (build) strs.reserve((b - a) * 64);
    std::vector<const uint8_t*> vp(F);
    std::vector<size_t> vl(F);
    for (size_t i = a; i < b; ++i) {
      prog[i] = policy[i] >= s.npolicies ? kProgDeny : s.lookup_prog(policy[i], ingress[i] != 0, port[i]);
      gcount[t][group_of(prog[i])]++;
      if (!build) continue;
      std::fill(vp.begin(), vp.end(), nullptr);
      const uint8_t* p = hdr_blob + hdr_off[i];
      const uint8_t* e = hdr_blob + hdr_off[i + 1];
      while (p < e) {
        const uint8_t* nm = p;
        while (p < e && *p) ++p;
        size_t nl = p - nm;
        if (p < e) ++p;
        const uint8_t* v = p;
        while (p < e && *p) ++p;
        size_t vlen = p - v;
        if (p < e) ++p;
        if (s.raw_values) {
          // escaped proxylib value: no raw byte <= 0x02, and 0x03 only as
          // the first byte of an escape pair
          for (size_t k = 0; k < vlen; ++k) {
            if (v[k] <= 0x02) malformed[i] = 1;
            if (v[k] == 0x03) {
              // an escape pair, or the list-item separator pair {0x03, 0x14}
              if (k + 1 >= vlen || v[k + 1] < 0x10 || v[k + 1] > 0x14) malformed[i] = 1;
              ++k;
            }
          }
        } else {
          for (size_t k = 0; k < vlen; ++k)
            if (codec_rejects(v[k])) malformed[i] = 1;
        }
        if (nl < by_len.size())
          for (uint32_t f : by_len[nl])
            if (!vp[f] && name_eq_ci(nm, nl, s.fields[f])) {  // first value wins (HeaderMap::get)
              vp[f] = v;
              vl[f] = vlen;
            }
      }
      const size_t o = strs.size();
      size_t last = 0;  // fields [last, F) are all absent
      for (size_t f = 0; f < F; ++f)
        if (vp[f]) last = f + 1;
      for (size_t f = 0; f < last; ++f) {
        if (!vp[f]) strs.push_back(kAbsent);
        else strs.insert(strs.end(), vp[f], vp[f] + vl[f]);
        strs.push_back(kSep);
      }
      if (last < F) strs.push_back(kRestAbsent);
      if (strs.size() - o > 0xFFFFFFFFull) fail(CG_INVALID_ARGUMENT, "request string beyond 4 GiB");
      soff[i] = (uint32_t)o;  // offsets within one worker's buffer stay below 4 GiB per worker
      slen[i] = (uint32_t)(strs.size() - o);
      if (strs.size() > 0xFFFFFFFFull) fail(CG_INVALID_ARGUMENT, "packer buffer beyond 4 GiB per worker");
      if (prog[i] < np && (s.progs[prog[i]].flags & kProgClass)) {
        const auto& code = s.prog_code[prog[i]];
        for (size_t k = o; k < strs.size(); ++k) strs[k] = code[strs[k]];
      }
    }
  });
  // string pointers (the workers' buffers no longer grow)
  std::vector<const uint8_t*> sp(build ? n : 0);
  if (build)
    parallel_ranges(n, nt, [&](size_t a, size_t b, unsigned t) {
      for (size_t i = a; i < b; ++i) sp[i] = sbuf[t].data() + soff[i];
    });
  lap("strings");
  auto str_ptr = [&](size_t i) -> const uint8_t* { return sp[i]; };
  auto str_len = [&](size_t i) -> size_t { return build ? slen[i] : 0; };
  // string units a request needs in its tile: 0 when the kernel does not
  // walk the slot string (malformed, or spilled to the overflow arena)
  auto walked_units = [&](size_t i) -> uint32_t {
    const size_t len = str_len(i);
    if (malformed[i] || len > CG_HTTP_SLOT_BYTES) return 0;
    return (uint32_t)((len + 15) / 16);
  };
  // ---- groups, their first slots and chunks
  std::vector<size_t> count(np + 2, 0);
  for (unsigned t = 0; t < nt; ++t)
    for (size_t g = 0; g < np + 2; ++g) count[g] += gcount[t][g];
  std::vector<size_t> first_slot(np + 2, 0);
  std::vector<HttpChunk> chunks;
  size_t tiles = 0;
  for (size_t g = 0; g < np + 2; ++g) {
    if (!count[g]) continue;
    first_slot[g] = tiles * CG_HTTP_TILE;
    size_t t = (count[g] + CG_HTTP_TILE - 1) / CG_HTTP_TILE;
    for (size_t k = 0; k < t; k += kChunkTiles)
      chunks.push_back({prog_of_group(g), (uint32_t)(tiles + k), (uint32_t)std::min<size_t>(kChunkTiles, t - k), 0});
    tiles += t;
  }
  const size_t nslots = tiles * CG_HTTP_TILE;
  if (nslots_out) *nslots_out = nslots;
  // ---- slot assignment: within a program group, requests ordered by the
  // number of 16-byte units their string spans, so the lanes of a tile end
  // their walks together, then by the string itself, so neighbouring lanes
  // share DFA states for as long as their strings share a prefix (their LDS
  // reads then broadcast instead of conflicting).  A counting sort into
  // (group, units) buckets, then each bucket sorted by content in parallel.
  constexpr size_t kKeys = CG_HTTP_UNITS + 2;
  auto key_of = [&](size_t i) -> size_t {
    const size_t len = str_len(i);
    return len > CG_HTTP_SLOT_BYTES ? CG_HTTP_UNITS + 1 : (len + 15) / 16;
  };
  std::vector<size_t> bstart((np + 2) * kKeys + 1, 0);
  for (size_t i = 0; i < n; ++i) bstart[group_of(prog[i]) * kKeys + key_of(i) + 1]++;
  for (size_t k = 1; k < bstart.size(); ++k) bstart[k] += bstart[k - 1];
  lap("buckets");
  std::vector<uint32_t> idx(n);
  {
    std::vector<size_t> fill(bstart.begin(), bstart.end() - 1);
    for (size_t i = 0; i < n; ++i) idx[fill[group_of(prog[i]) * kKeys + key_of(i)]++] = (uint32_t)i;
  }
  lap("idx");
  if (build) {
    // each bucket (one program, one unit count) ordered by string length,
    // so a tile's lanes end together (the last-unit tail is tight), then by
    // the first 32 bytes and a hash of the rest: lanes with a common prefix
    // sit together and walk the same DFA states (their LDS reads broadcast)
    // for that long, identical strings all the way.  Keys are local
    // records: no string compares in the sort.
    struct Rec {
      uint32_t len, i;
      uint64_t pre[4];  // bytes 0..31, big-endian, zero-padded
      uint64_t rest;    // FNV-1a of bytes 32..
    };
    std::vector<size_t> buckets;
    for (size_t k = 0; k + 1 < bstart.size(); ++k)
      if (bstart[k + 1] - bstart[k] > 1) buckets.push_back(k);
    // largest buckets first
    std::sort(buckets.begin(), buckets.end(),
              [&](size_t a, size_t b) { return bstart[a + 1] - bstart[a] > bstart[b + 1] - bstart[b]; });
    parallel_items(buckets.size(), nt, [&](size_t bi) {
      const size_t k = buckets[bi];
      std::vector<Rec> r(bstart[k + 1] - bstart[k]);
      for (size_t j = 0; j < r.size(); ++j) {
        const uint32_t i = idx[bstart[k] + j];
        const uint8_t* q = sp[i];
        const size_t L = slen[i];
        Rec& e = r[j];
        for (int w = 0; w < 4; ++w) {
          uint64_t x = 0;
          for (size_t c = 8 * w; c < 8 * w + 8; ++c) x = x << 8 | (c < L ? q[c] : 0);
          e.pre[w] = x;
        }
        uint64_t h = 1469598103934665603ull;
        for (size_t c = 32; c < L; ++c) h = (h ^ q[c]) * 1099511628211ull;
        e.rest = h;
        e.i = i;
        e.len = (uint32_t)L;
      }
      std::sort(r.begin(), r.end(), [](const Rec& a, const Rec& b) {
        if (a.len != b.len) return a.len < b.len;
        for (int w = 0; w < 4; ++w)
          if (a.pre[w] != b.pre[w]) return a.pre[w] < b.pre[w];
        if (a.rest != b.rest) return a.rest < b.rest;
        return a.i < b.i;
      });
      for (size_t j = 0; j < r.size(); ++j) idx[bstart[k] + j] = r[j].i;
    });
  }
  lap("sort");
  std::vector<uint32_t> slot_of(n);
  std::vector<uint32_t> req_of_slot(nslots, 0xFFFFFFFFu);
  for (size_t g = 0; g < np + 2; ++g) {
    size_t pos = first_slot[g];
    for (size_t r = bstart[g * kKeys]; r < bstart[(g + 1) * kKeys]; ++r) {
      slot_of[idx[r]] = (uint32_t)pos;
      req_of_slot[pos] = idx[r];
      ++pos;
    }
  }
  // ---- tile table: each tile's string units = its longest walked string,
  // and the bytes its lanes hold in that last unit (padding past the longest
  // one need not be walked: comb.h, padding never changes a label)
  std::vector<HttpTile> ttab(tiles);
  // half last units only in tiles of programs http_kernel walks one part at
  // a time from LDS (one_part_tiles; its other walkers read whole units)
  std::vector<uint8_t> half_ok(tiles, 0);
  for (const HttpChunk& c : chunks) {
    const bool ok = c.prog < np && !(s.progs[c.prog].flags & kProgAllowAll) && s.progs[c.prog].part_count == 1 &&
                    (s.progs[c.prog].flags & kProgRebased) && s.progs[c.prog].cell_count <= kMaxLdsCells;
    std::fill(half_ok.begin() + c.first_tile, half_ok.begin() + c.first_tile + c.ntiles, (uint8_t)ok);
  }
  parallel_ranges(tiles, nt, [&](size_t a, size_t b, unsigned) {
    for (size_t k = a; k < b; ++k) {
      uint32_t units = 0, tail = 0;
      for (size_t l = 0; l < CG_HTTP_TILE; ++l) {
        const uint32_t i = req_of_slot[k * CG_HTTP_TILE + l];
        if (i != 0xFFFFFFFFu) units = std::max(units, walked_units(i));
      }
      for (size_t l = 0; l < CG_HTTP_TILE && units; ++l) {
        const uint32_t i = req_of_slot[k * CG_HTTP_TILE + l];
        if (i != 0xFFFFFFFFu && walked_units(i) == units)
          tail = std::max<uint32_t>(tail, (uint32_t)(str_len(i) - 16 * (units - 1)));
      }
      if (units && !tail) tail = 16;
      // a last unit holding at most 8 bytes of any lane is stored as a half
      // unit: 512 B less per tile (config 5: 6.7% of the batch)
      ttab[k].units = units | (units && tail <= 8 && half_ok[k] ? kTileHalfLast : 0u) | tail << 16;
    }
  });
  lap("ttab");
  uint64_t gran = 0;
  for (auto& t : ttab) {
    if (gran > 0xFFFFFFFFull) fail(CG_INVALID_ARGUMENT, "batch beyond 2 TiB");
    t.at = (uint32_t)gran;
    gran += tile_granules(t);
  }
  const size_t max_tiles = http_batch_slots(s, n) / CG_HTTP_TILE;
  const size_t hdr = header_bytes(max_tiles);
  const size_t need = hdr + gran * kGranule;
  if (batch && need > batch_cap) fail(CG_INVALID_ARGUMENT, "batch buffer too small");
  uint8_t* data = batch ? (uint8_t*)batch + hdr : nullptr;
  auto unit_ptr = [&](size_t slot, uint32_t u) {
    return data + tile_unit_at(ttab[slot / CG_HTTP_TILE], u, slot % CG_HTTP_TILE);
  };
  // overflow arena entries in request order: u32 length then the string,
  // 16-byte aligned
  std::vector<uint64_t> aoff(n, ~0ull);
  size_t used = 0;
  for (size_t i = 0; i < n && build; ++i) {
    const size_t len = str_len(i);
    if (len <= CG_HTTP_SLOT_BYTES) continue;
    if (used / 16 >= (1u << 24)) fail(CG_INVALID_ARGUMENT, "overflow arena beyond 256 MiB");
    aoff[i] = used;
    used += (4 + len + 15) & ~(size_t)15;
  }
  if (batch) {
    HttpBatchHeader h{};
    h.magic = kBatchMagic;
    h.epoch = s.epoch;
    h.nchunks = (uint32_t)chunks.size();
    h.ntiles = (uint32_t)tiles;
    h.tiles_off = hdr;
    h.nslots = nslots;
    h.ttab_off = ttab_off(max_tiles);
    h.total_bytes = need;
    h.arena_bytes = used;
    memcpy(batch, &h, sizeof(h));
    memcpy((uint8_t*)batch + sizeof(h), chunks.data(), chunks.size() * sizeof(HttpChunk));
    memcpy((uint8_t*)batch + h.ttab_off, ttab.data(), ttab.size() * sizeof(HttpTile));
  }
  if (order)
    for (size_t sl = 0; sl < nslots; ++sl) order[sl] = req_of_slot[sl];
  // ---- tiles (parallel): meta block, string units, padding slots
  if (batch || (arena && build)) {
    parallel_ranges(tiles, nt, [&](size_t a, size_t b, unsigned) {
      for (size_t k = a; k < b; ++k) {
        if (batch) memset(data + (size_t)ttab[k].at * kGranule, 0, (size_t)tile_granules(ttab[k]) * kGranule);
        for (size_t l = 0; l < CG_HTTP_TILE; ++l) {
          const size_t sl = k * CG_HTTP_TILE + l;
          const uint32_t i = req_of_slot[sl];
          if (i == 0xFFFFFFFFu) {
            if (batch) unit_ptr(sl, 0)[7] = CG_HTTP_F_PAD;
            continue;
          }
          const uint8_t* str = str_ptr(i);
          const uint32_t len = (uint32_t)str_len(i);
          // meta (CG_HTTP_META_BYTES = 8): [0..3] remote identity, [4..6]
          // overflow arena offset / 16, [7] flags
          uint8_t meta[CG_HTTP_META_BYTES] = {0};
          memcpy(meta, &remote[i], 4);
          uint8_t flags = ingress[i] ? CG_HTTP_F_INGRESS : 0;
          if (malformed[i]) flags |= CG_HTTP_F_MALFORMED;
          if (len > CG_HTTP_SLOT_BYTES) {
            flags |= CG_HTTP_F_OVERFLOW;
            const uint64_t o = aoff[i];
            if (arena && o + 4 + len <= arena_cap) {
              memcpy(arena + o, &len, 4);
              memcpy(arena + o + 4, str, len);
            }
            const uint32_t off16 = (uint32_t)(o / 16);
            meta[4] = off16 & 0xFF;
            meta[5] = (off16 >> 8) & 0xFF;
            meta[6] = (off16 >> 16) & 0xFF;
          }
          meta[7] = flags;
          if (batch) {
            memcpy(unit_ptr(sl, 0), meta, CG_HTTP_META_BYTES);
            const uint32_t wu = walked_units(i);
            const HttpTile& tt = ttab[k];
            for (uint32_t u = 0; u < wu; ++u) {
              // (a half unit holds the tile's last ≤ 8 bytes of every lane)
              const size_t cap = u + 1 == tile_units(tt) && tile_half(tt) ? 8 : 16;
              memcpy(unit_ptr(sl, u + 1), str + u * 16, std::min<size_t>(cap, len - u * 16));
            }
          }
        }
      }
    });
  }
  lap("write");
  if (arena_used) *arena_used = used;
  if (arena && used > arena_cap) fail(CG_INVALID_ARGUMENT, "overflow arena too small");
}

void http_eval_host(const HttpSnapshot& s, const uint8_t* batch, const uint8_t* arena, size_t arena_len,
                    uint8_t* out, uint32_t* rule) {
  HttpBatchHeader h;
  memcpy(&h, batch, sizeof(h));
  if (h.magic != kBatchMagic || h.epoch != s.epoch) fail(CG_INVALID_ARGUMENT, "batch packed for another snapshot");
  const HttpChunk* chunks = (const HttpChunk*)(batch + sizeof(h));
  const HttpTile* ttab = (const HttpTile*)(batch + h.ttab_off);
  const uint8_t* data = batch + h.tiles_off;
  auto unit_ptr = [&](size_t slot, uint32_t u) {
    return data + tile_unit_at(ttab[slot / CG_HTTP_TILE], u, slot % CG_HTTP_TILE);
  };
  for (uint32_t c = 0; c < h.nchunks; ++c) {
    const uint32_t prog = chunks[c].prog;
    for (size_t sl = (size_t)chunks[c].first_tile * CG_HTTP_TILE;
         sl < (size_t)(chunks[c].first_tile + chunks[c].ntiles) * CG_HTTP_TILE; ++sl) {
      uint8_t meta[CG_HTTP_META_BYTES];
      memcpy(meta, unit_ptr(sl, 0), CG_HTTP_META_BYTES);
      uint32_t remote;
      memcpy(&remote, meta, 4);
      const uint32_t off = ((uint32_t)meta[4] | ((uint32_t)meta[5] << 8) | ((uint32_t)meta[6] << 16)) * 16u;
      const uint8_t flags = meta[7];
      uint8_t v = 0;
      out[sl] = 0;
      if (rule) rule[sl] = 0xFFFFFFFFu;
      if (flags & (CG_HTTP_F_PAD | CG_HTTP_F_MALFORMED)) continue;
      if (prog == kProgDeny) continue;
      if (prog == kProgAllow) {
        out[sl] = 1;
        continue;
      }
      const HttpProg& pg = s.progs[prog];
      if (pg.flags & kProgAllowAll) {
        out[sl] = 1;
        continue;
      }
      // the bytes the kernel walks: the arena string, or the tile's units
      // (the string and its zero padding, which cannot change the verdict)
      std::string str;
      if (flags & CG_HTTP_F_OVERFLOW) {
        uint32_t len = 0;
        if ((size_t)off + 4 > arena_len) continue;
        memcpy(&len, arena + off, 4);
        if ((size_t)off + 4 + len > arena_len) continue;
        str.assign((const char*)arena + off + 4, len);
      } else {
        const HttpTile& tt = ttab[sl / CG_HTTP_TILE];
        for (uint32_t u = 0; u < tile_units(tt); ++u) {
          const bool half = u + 1 == tile_units(tt) && tile_half(tt);
          str.append((const char*)unit_ptr(sl, u + 1), half ? 8 : 16);
          if (half) str.append(8, '\0');
        }
      }
      const uint32_t* blk = s.cells.data() + pg.cell_begin;
      auto bmask = [&](uint32_t o, uint32_t w) { return (uint64_t)blk[o + 2 * w] | (uint64_t)blk[o + 2 * w + 1] << 32; };
      uint32_t roff = pg.default_remote;
      if (pg.flags & kProgRemoteDirect) {
        if (remote - pg.rdir_base < pg.rdir_len)
          roff = ((const uint16_t*)(s.cells.data() + pg.cell_begin + pg.rdir_off))[remote - pg.rdir_base];
      } else
      for (uint32_t bk : {rtab_b1(remote, pg.rtab_nb), rtab_b2(remote, pg.rtab_nb)})
        for (uint32_t sl = 0; sl < 4; ++sl) {
          const uint32_t* b = blk + pg.rtab_off + kRtabBucketCells * bk;
          if (b[sl] == remote) roff = b[4 + sl];
        }
      // first rule (lowest bit) the mask at block offset a shares with the row
      uint32_t hit = 0xFFFFFFFFu;
      auto first = [&](uint32_t a) {
        for (uint32_t w = 0; w < pg.mask_words; ++w)
          if (const uint64_t x = bmask(a, w) & bmask(roff, w)) return w * 64 + (uint32_t)__builtin_ctzll(x);
        return 0xFFFFFFFFu;
      };
      hit = std::min(hit, first(pg.always_off));
      for (uint32_t pi = 0; pi < pg.part_count; ++pi) {
        const HttpPart& pt = s.parts[pg.part_begin + pi];
        const uint32_t* cells = s.cells.data() + pt.walk_off;
        const bool scaled = pt.mode == kPartClass;
        uint32_t st = pt.start;
        for (unsigned char ch : str) {
          st = comb_next(cells, pt.dead, st, ch, scaled);
          if (st == pt.dead) break;
        }
        const uint32_t lab = comb_label(cells, st, scaled);
        if (lab == kCombNoLabel) continue;
        hit = std::min(hit, first(pt.acc_off + lab * 2 * pg.mask_words));
      }
      v = hit != 0xFFFFFFFFu;
      out[sl] = v;
      if (rule && v) rule[sl] = pg.rule_base + hit;
    }
  }
}

}  // namespace cg

// The packer's worker count for a large batch (what cg_http_pack uses).
extern "C" uint32_t cg_http_pack_threads(void) { return cg::pack_threads((size_t)1 << 20); }
