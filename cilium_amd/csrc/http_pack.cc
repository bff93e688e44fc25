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

// byte offset of unit u (0 = meta block) of a tile at granule g, lane l
inline size_t tile_unit_at(uint32_t g, uint32_t u, size_t lane) {
  return (size_t)g * kGranule + (u ? kMetaBytes + (size_t)(u - 1) * kUnitBytes + lane * 16 : lane * CG_HTTP_META_BYTES);
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

void http_pack(const HttpSnapshot& s, size_t n, const uint32_t* policy, const uint8_t* ingress,
               const uint16_t* port, const uint32_t* remote, const uint8_t* hdr_blob,
               const uint64_t* hdr_off, void* batch, size_t batch_cap, uint32_t* order, size_t* nslots_out,
               uint8_t* arena, size_t arena_cap, size_t* arena_used) {
  // ---- program of every request, groups in ascending program id
  std::vector<uint32_t> prog(n);
  std::map<uint32_t, size_t> count;
  for (size_t i = 0; i < n; ++i) {
    prog[i] = policy[i] >= s.npolicies ? kProgDeny : s.lookup_prog(policy[i], ingress[i] != 0, port[i]);
    count[prog[i]]++;
  }
  std::map<uint32_t, size_t> first_slot;
  std::vector<HttpChunk> chunks;
  size_t tiles = 0;
  for (auto& [p, c] : count) {
    first_slot[p] = tiles * CG_HTTP_TILE;
    size_t t = (c + CG_HTTP_TILE - 1) / CG_HTTP_TILE;
    for (size_t k = 0; k < t; k += kChunkTiles)
      chunks.push_back({p, (uint32_t)(tiles + k), (uint32_t)std::min<size_t>(kChunkTiles, t - k), 0});
    tiles += t;
  }
  const size_t nslots = tiles * CG_HTTP_TILE;
  if (nslots_out) *nslots_out = nslots;
  // ---- request strings (field values in field order, SEP-terminated)
  const size_t F = s.fields.size();
  std::vector<uint8_t> strs;
  std::vector<uint64_t> soff(n + 1, 0);
  std::vector<uint8_t> malformed(n, 0);
  const bool build = batch || arena_used;
  if (build) {
    strs.reserve(n * 64);
    std::vector<const uint8_t*> vp(F);
    std::vector<size_t> vl(F);
    for (size_t i = 0; i < n; ++i) {
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
              if (k + 1 >= vlen || v[k + 1] < 0x10 || v[k + 1] > 0x13) malformed[i] = 1;
              ++k;
            }
          }
        } else {
          for (size_t k = 0; k < vlen; ++k)
            if (codec_rejects(v[k])) malformed[i] = 1;
        }
        for (size_t f = 0; f < F; ++f)
          if (!vp[f] && name_eq_ci(nm, nl, s.fields[f])) {  // first value wins (HeaderMap::get)
            vp[f] = v;
            vl[f] = vlen;
          }
      }
      size_t last = 0;  // fields [last, F) are all absent
      for (size_t f = 0; f < F; ++f)
        if (vp[f]) last = f + 1;
      for (size_t f = 0; f < last; ++f) {
        if (!vp[f]) strs.push_back(kAbsent);
        else strs.insert(strs.end(), vp[f], vp[f] + vl[f]);
        strs.push_back(kSep);
      }
      if (last < F) strs.push_back(kRestAbsent);
      soff[i + 1] = strs.size();
      if (prog[i] < s.progs.size() && (s.progs[prog[i]].flags & kProgClass)) {
        const auto& code = s.prog_code[prog[i]];
        for (size_t k = soff[i]; k < soff[i + 1]; ++k) strs[k] = code[strs[k]];
      }
    }
  }
  auto str_len = [&](size_t i) -> size_t { return build ? soff[i + 1] - soff[i] : 0; };
  // string units a request needs in its tile: 0 when the kernel does not
  // walk the slot string (malformed, or spilled to the overflow arena)
  auto walked_units = [&](size_t i) -> uint32_t {
    const size_t len = str_len(i);
    if (malformed[i] || len > CG_HTTP_SLOT_BYTES) return 0;
    return (uint32_t)((len + 15) / 16);
  };
  // ---- slot assignment: within a program group, requests ordered by the
  // number of 16-byte units their string spans, so the lanes of a tile end
  // their walks together, then by the string itself, so neighbouring lanes
  // share DFA states for as long as their strings share a prefix (their LDS
  // reads then broadcast instead of conflicting)
  std::vector<uint32_t> slot_of(n);
  {
    std::vector<uint8_t> key(n, 0);
    for (size_t i = 0; i < n; ++i) {
      const size_t len = str_len(i);
      key[i] = len > CG_HTTP_SLOT_BYTES ? CG_HTTP_UNITS + 1 : (uint8_t)((len + 15) / 16);
    }
    std::vector<uint32_t> idx(n);
    for (size_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
    std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
      if (prog[a] != prog[b]) return prog[a] < prog[b];
      if (key[a] != key[b]) return key[a] < key[b];
      if (build) {
        const size_t la = soff[a + 1] - soff[a], lb = soff[b + 1] - soff[b];
        const int c = memcmp(strs.data() + soff[a], strs.data() + soff[b], std::min(la, lb));
        if (c != 0) return c < 0;
        if (la != lb) return la < lb;
      }
      return a < b;
    });
    size_t pos = 0;
    for (size_t r = 0; r < n; ++r) {
      const uint32_t i = idx[r];
      if (r == 0 || prog[i] != prog[idx[r - 1]]) pos = first_slot[prog[i]];
      slot_of[i] = (uint32_t)pos++;
    }
  }
  // ---- tile table: each tile's string units = its longest walked string
  std::vector<HttpTile> ttab(tiles);
  for (size_t i = 0; i < n; ++i) {
    HttpTile& t = ttab[slot_of[i] / CG_HTTP_TILE];
    t.units = std::max(t.units, walked_units(i));
  }
  // the bytes the lanes of a tile hold in its last unit (padding past the
  // longest one need not be walked: comb.h, padding never changes a label)
  {
    std::vector<uint32_t> tail(ttab.size(), 0);
    for (size_t i = 0; i < n; ++i) {
      const uint32_t wu = walked_units(i);
      HttpTile& t = ttab[slot_of[i] / CG_HTTP_TILE];
      if (wu && wu == t.units) {
        uint32_t& tl = tail[slot_of[i] / CG_HTTP_TILE];
        tl = std::max<uint32_t>(tl, (uint32_t)(str_len(i) - 16 * (wu - 1)));
      }
    }
    for (size_t k = 0; k < ttab.size(); ++k)
      if (ttab[k].units) ttab[k].units |= (tail[k] ? tail[k] : 16u) << 16;
  }
  uint64_t gran = 0;
  for (auto& t : ttab) {
    if (gran > 0xFFFFFFFFull) fail(CG_INVALID_ARGUMENT, "batch beyond 2 TiB");
    t.at = (uint32_t)gran;
    gran += 1 + 2 * tile_units(t);
  }
  const size_t max_tiles = http_batch_slots(s, n) / CG_HTTP_TILE;
  const size_t hdr = header_bytes(max_tiles);
  const size_t need = hdr + gran * kGranule;
  if (batch && need > batch_cap) fail(CG_INVALID_ARGUMENT, "batch buffer too small");
  uint8_t* data = batch ? (uint8_t*)batch + hdr : nullptr;
  auto unit_ptr = [&](size_t slot, uint32_t u) {
    return data + tile_unit_at(ttab[slot / CG_HTTP_TILE].at, u, slot % CG_HTTP_TILE);
  };
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
    memcpy(batch, &h, sizeof(h));
    memcpy((uint8_t*)batch + sizeof(h), chunks.data(), chunks.size() * sizeof(HttpChunk));
    memcpy((uint8_t*)batch + h.ttab_off, ttab.data(), ttab.size() * sizeof(HttpTile));
    memset(data, 0, gran * kGranule);
    // padding slots of every group
    for (auto& [p, c] : count) {
      size_t s0 = first_slot[p];
      size_t end = s0 + ((c + CG_HTTP_TILE - 1) / CG_HTTP_TILE) * CG_HTTP_TILE;
      for (size_t sl = s0 + c; sl < end; ++sl) {
        unit_ptr(sl, 0)[7] = CG_HTTP_F_PAD;
        if (order) order[sl] = 0xFFFFFFFFu;
      }
    }
  }
  size_t used = 0;
  for (size_t i = 0; i < n; ++i) {
    const size_t sl = slot_of[i];
    if (order) order[sl] = (uint32_t)i;
    if (!build) continue;
    const uint8_t* str = strs.data() + soff[i];
    const uint32_t len = (uint32_t)(soff[i + 1] - soff[i]);
    // meta (CG_HTTP_META_BYTES = 8): [0..3] remote identity, [4..6] overflow
    // arena offset / 16, [7] flags; an overflow arena entry is its u32 length
    // then the string, 16-byte aligned
    uint8_t meta[CG_HTTP_META_BYTES] = {0};
    memcpy(meta, &remote[i], 4);
    uint8_t flags = ingress[i] ? CG_HTTP_F_INGRESS : 0;
    if (malformed[i]) flags |= CG_HTTP_F_MALFORMED;
    if (len > CG_HTTP_SLOT_BYTES) {
      flags |= CG_HTTP_F_OVERFLOW;
      if (used / 16 >= (1u << 24)) fail(CG_INVALID_ARGUMENT, "overflow arena beyond 256 MiB");
      uint32_t off16 = (uint32_t)(used / 16);
      if (arena && used + 4 + len <= arena_cap) {
        memcpy(arena + used, &len, 4);
        memcpy(arena + used + 4, str, len);
      }
      used += (4 + len + 15) & ~(size_t)15;
      meta[4] = off16 & 0xFF;
      meta[5] = (off16 >> 8) & 0xFF;
      meta[6] = (off16 >> 16) & 0xFF;
    }
    meta[7] = flags;
    if (batch) {
      memcpy(unit_ptr(sl, 0), meta, CG_HTTP_META_BYTES);
      const uint32_t wu = walked_units(i);
      for (uint32_t u = 0; u < wu; ++u)
        memcpy(unit_ptr(sl, u + 1), str + u * 16, std::min<size_t>(16, len - u * 16));
    }
  }
  if (arena_used) *arena_used = used;
  if (arena && used > arena_cap) fail(CG_INVALID_ARGUMENT, "overflow arena too small");
  if (batch) {
    uint64_t ab = used;
    memcpy((uint8_t*)batch + offsetof(HttpBatchHeader, arena_bytes), &ab, sizeof(ab));
  }
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
    return data + tile_unit_at(ttab[slot / CG_HTTP_TILE].at, u, slot % CG_HTTP_TILE);
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
        for (uint32_t u = 0; u < tile_units(ttab[sl / CG_HTTP_TILE]); ++u)
          str.append((const char*)unit_ptr(sl, u + 1), 16);
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
