// http_raw.cc — host side of the raw HTTP/1 path (kernels_http_raw.hip):
// the snapshot's device tables for it, and the launch sequence
//   scan → (bucket counts to the host) → layout → rank → build → http_kernel
// on one stream.  The host step is the layout of a few thousand bucket
// counts (chunks, runs of equal-units tiles, bucket cursors); request bytes
// never leave the device.  CILIUM_GPU_RAW_LAYOUT=device selects the
// device-layout sequence instead (raw_device_layout):
//   clear → scan (+ deferred) → seal → http_kernel → walk
// per sub-batch, all on the caller's stream, with no copy back and no host
// synchronization (the layout is raw_seal_kernel's).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "http.h"
#include "kernels.h"

namespace cg {

namespace {

uint32_t next_pow2(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

void http_raw_upload(HttpSnapshot& S) {
  S.raw_ok = S.lists_ok = false;
  S.raw = HttpRawDev{};
  const uint32_t F = (uint32_t)S.fields.size();
  if (F > kRawMaxFields) return;
  HttpRawDev& R = S.raw;
  R.f_method = R.f_path = R.f_authority = R.f_empty = -1;
  R.raw_values = S.raw_values ? 1u : 0u;
  const uint32_t cap = next_pow2(std::max<uint32_t>(2 * F, 4));
  std::vector<uint32_t> slots(4 * (size_t)cap, 0);
  std::vector<uint8_t> names;
  for (uint32_t f = 0; f < F; ++f) {
    const std::string& nm = S.fields[f];
    if (nm == ":method") R.f_method = (int32_t)f;
    else if (nm == ":path") R.f_path = (int32_t)f;
    else if (nm == ":authority") R.f_authority = (int32_t)f;
    else if (nm.empty()) R.f_empty = (int32_t)f;
    // pseudo headers are in the tables for header lists; a head's header line
    // never names one (':' is not a token byte)
    if (nm.empty()) continue;
    uint32_t h = kRawFnvInit;
    for (unsigned char c : nm) h = raw_fnv(h, (uint8_t)((c >= 'A' && c <= 'Z') ? c + 32 : c));
    uint32_t sl = h & (cap - 1);
    while (slots[4 * (size_t)sl + 1]) sl = (sl + 1) & (cap - 1);
    slots[4 * (size_t)sl] = h;
    slots[4 * (size_t)sl + 1] = (uint32_t)nm.size();
    slots[4 * (size_t)sl + 2] = f;
    slots[4 * (size_t)sl + 3] = (uint32_t)names.size();
    for (unsigned char c : nm) names.push_back((uint8_t)((c >= 'A' && c <= 'Z') ? c + 32 : c));
  }
  if (names.empty()) names.push_back(0);
  // the same names by (length, first 8, last 8) key (kernels_http_raw.hip
  // field_of_key); name offsets index `names`
  std::vector<uint32_t> nk(8 * (size_t)cap, 0);
  for (uint32_t f = 0; f < F; ++f) {
    const std::string& nm = S.fields[f];
    if (nm.empty()) continue;
    const uint32_t nl = (uint32_t)nm.size();
    auto byte = [&](uint32_t j) -> uint32_t {
      const unsigned char c = (unsigned char)nm[j];
      return (c >= 'A' && c <= 'Z') ? c + 32u : c;
    };
    auto word = [&](uint32_t at, uint32_t lim) {  // bytes at..at+3 below lim
      uint32_t w = 0;
      for (uint32_t j = 0; j < 4; ++j)
        if (at + j < lim) w |= byte(at + j) << (8 * j);
      return w;
    };
    const uint32_t lo0 = word(0, nl), lo1 = word(4, nl);
    const uint32_t hi0 = nl > 8 ? word(nl - 8, nl) : 0u, hi1 = nl > 8 ? word(nl - 4, nl) : 0u;
    uint32_t sl = raw_name_hash(nl, lo0, lo1, hi0, hi1) & (cap - 1);
    while (nk[8 * (size_t)sl]) sl = (sl + 1) & (cap - 1);
    uint32_t off = 0;  // the name's offset in `names` (from the FNV table)
    for (uint32_t k = 0; k < cap; ++k)
      if (slots[4 * (size_t)k + 1] && slots[4 * (size_t)k + 2] == f) off = slots[4 * (size_t)k + 3];
    const uint32_t e[8] = {nl, lo0, lo1, hi0, hi1, f, off, 0};
    memcpy(&nk[8 * (size_t)sl], e, sizeof e);
  }
  std::vector<uint8_t> codes(std::max<size_t>(S.progs.size(), 1) * 256);
  for (size_t p = 0; p < S.progs.size(); ++p)
    for (int b = 0; b < 256; ++b)
      codes[p * 256 + b] = (S.progs[p].flags & kProgClass) ? S.prog_code[p][b] : (uint8_t)b;
  S.d_phk.upload_vec(S.phash_keys);
  S.d_phv.upload_vec(S.phash_vals);
  S.d_fslots.upload_vec(slots);
  S.d_fnames.upload_vec(names);
  S.d_codes.upload_vec(codes);
  std::vector<uint32_t> walk((S.progs.size() + 31) / 32 + 1, 0);
  for (size_t p = 0; p < S.progs.size(); ++p)
    if (!(S.progs[p].flags & kProgAllowAll)) walk[p / 32] |= 1u << (p % 32);
  S.d_walk.upload_vec(walk);
  S.d_nkeys.upload_vec(nk);
  R.phash_keys = S.d_phk.as<uint32_t>();
  R.phash_vals = S.d_phv.as<uint32_t>();
  R.phash_mask = S.phash_mask;
  R.npolicies = S.npolicies;
  R.dflt = S.d_dflt.as<uint32_t>();
  R.progs = S.d_progs.as<HttpProg>();
  R.nprogs = (uint32_t)S.progs.size();
  R.nfields = F;
  R.fmask = cap - 1;
  R.fslots = S.d_fslots.as<uint32_t>();
  R.fnames = S.d_fnames.as<uint8_t>();
  R.fnames_bytes = (uint32_t)names.size();
  R.codes = S.d_codes.as<uint8_t>();
  R.nkeys = S.d_nkeys.as<uint32_t>();
  R.walk_bits = S.d_walk.as<uint32_t>();
  R.nkmask = cap - 1;
  S.lists_ok = true;
  S.raw_ok = !S.raw_values;  // proxylib snapshots take escaped values, not heads
}

namespace {

// One raw call between its phases (raw_scan_phase → raw_rest_phase).  Tried:
// two halves on two streams, the second half's scan under the first half's
// rank and build — the streams shared one hardware queue, so nothing
// overlapped (21.7 against 21.3 ms), not kept.
struct RawCall {
  const HttpSnapshot* s;
  StagingSlot* sl;
  int cus;
  RawInput in;
  const uint8_t* d_raw;
  const uint64_t* d_off;
  size_t n;
  const uint32_t *d_policy, *d_remote;
  const uint8_t* d_ingress;
  const uint16_t* d_port;
  uint8_t* d_out;
  hipStream_t st;
  // set by raw_scan_phase
  size_t hist_bytes = 0;
  uint8_t *small = nullptr, *hh = nullptr;
  uint32_t* hist = nullptr;
  unsigned long long* ovf = nullptr;
  uint8_t* sbuf = nullptr;
  void* rinfo = nullptr;
  uint32_t *bbase = nullptr, nblk = 0;
  RawCall half(size_t a, size_t m) const {
    RawCall c = *this;
    c.d_off = d_off + a;
    c.n = m;
    c.d_policy = d_policy + a;
    c.d_ingress = d_ingress + a;
    c.d_port = d_port + a;
    c.d_remote = d_remote + a;
    c.d_out = d_out + a;
    return c;
  }
};

// Workspace, the offsets' range, scan (+ deferred requests) and prefix
// launched, their counts copied back (async).  false: the string buffer
// would pass 2^32 16-B units — the caller splits the call.
bool raw_scan_phase(RawCall& c) {
  const HttpSnapshot& s = *c.s;
  const uint32_t np = (uint32_t)s.progs.size(), G = np + 2, K = kRawKeys;
  // workspace: [histogram G*K u32][overflow bytes u64][arena cursor u64][head
  // bytes u64][deferred-request count u32, pad]
  c.hist_bytes = ((size_t)G * K * 4 + 7) & ~(size_t)7;
  const size_t hist_bytes = c.hist_bytes;
  c.small = (uint8_t*)c.sl->dev_buf(8, hist_bytes + 32);
  uint8_t* small = c.small;
  c.hist = (uint32_t*)small;
  c.ovf = (unsigned long long*)(small + hist_bytes);
  hip_check(hipMemsetAsync(small, 0, hist_bytes + 16, c.st), "hipMemsetAsync");
  // the head bytes [off[0], off[n]) size the string buffer
  hip_check(hipMemcpyAsync(small + hist_bytes + 16, c.d_off + c.n, 8, hipMemcpyDeviceToDevice, c.st), "D2D");
  hip_check(hipMemcpyAsync(small + hist_bytes + 8, c.d_off, 8, hipMemcpyDeviceToDevice, c.st), "D2D");
  c.hh = (uint8_t*)c.sl->host_buf(8, hist_bytes + 24);
  hip_check(hipMemcpyAsync(c.hh, small, hist_bytes + 24, hipMemcpyDeviceToHost, c.st), "D2H");
  hip_check(hipStreamSynchronize(c.st), "hipStreamSynchronize");
  uint64_t o0, o1;
  memcpy(&o0, c.hh + hist_bytes + 8, 8);
  memcpy(&o1, c.hh + hist_bytes + 16, 8);
  if (o1 < o0) fail(CG_INVALID_ARGUMENT, "raw_off must be non-decreasing");
  // the arena cursor, the head-bytes slot, the deferred-request count
  hip_check(hipMemsetAsync(small + hist_bytes + 8, 0, 24, c.st), "hipMemsetAsync");
  auto* dcount = (uint32_t*)(small + hist_bytes + 24);
  // string buffer: request i's record (16-byte header + uncoded string) in
  // its region at align16(off[i] - off[0]) + cst * i (kernels_http_raw.hip
  // rec_off); the build pass addresses records in 16-byte units through u32
  // order words
  // (+128: room to move a record to a line start, kernels_http_raw.hip rec_off)
  const uint32_t cst = (uint32_t)((2 * std::max<size_t>(s.raw.nfields, 1) + 48 + 15) & ~(size_t)15) + 128;
  // (+256: the build kernel reads whole 16-B chunks up to 8 units past a record's start)
  const size_t sbytes = ((o1 - o0 + 15) & ~(uint64_t)15) + (size_t)cst * c.n + 256;
  if (sbytes / 16 >= (1ull << 32)) {
    if (c.n < 2) fail(CG_INVALID_ARGUMENT, "raw head too large");
    return false;
  }
  c.sbuf = (uint8_t*)c.sl->dev_buf(15, sbytes);
  c.rinfo = c.sl->dev_buf(9, c.n * 8);
  // per-block bucket counts → per-block slot offsets (when the bucket
  // counters fit the kernels' LDS), else one global histogram
  const bool lds_keys = http_raw_lds_keys(s.raw);
  const bool lists = c.in == RawInput::Lists;
  c.nblk = (uint32_t)http_raw_grid(s.raw, lists, c.n, c.cus);
  uint32_t* bcount = lds_keys ? (uint32_t*)c.sl->dev_buf(16, (size_t)G * K * c.nblk * 4) : c.hist;
  c.bbase = lds_keys ? (uint32_t*)c.sl->dev_buf(17, (size_t)G * K * c.nblk * 4) : nullptr;
  auto* dlist = (uint32_t*)c.sl->dev_buf(18, c.n * 4);
  hip_check(launch_http_raw_scan(s.raw, lists, c.d_raw, c.d_off, c.n, c.d_policy, c.d_ingress, c.d_port, bcount,
                                 c.rinfo, c.d_remote, c.sbuf, cst, c.ovf, dlist, dcount, c.st, c.cus),
            "raw scan kernel launch");
  if (lds_keys)
    hip_check(launch_http_raw_prefix(bcount, G * K, c.nblk, c.bbase, c.hist, c.st), "raw prefix kernel launch");
  hip_check(hipMemcpyAsync(c.hh, small, hist_bytes + 8, hipMemcpyDeviceToHost, c.st), "D2H");
  return true;
}

// Waits for the scan's counts, lays the batch out, launches rank, build and
// http_kernel (no final sync).  false: the long strings need more than the
// 256 MiB overflow arena — the caller splits the call.
bool raw_rest_phase(RawCall& c) {
  const HttpSnapshot& s = *c.s;
  const uint32_t np = (uint32_t)s.progs.size(), G = np + 2, K = kRawKeys;
  const size_t hist_bytes = c.hist_bytes;
  hip_check(hipStreamSynchronize(c.st), "hipStreamSynchronize");
  const uint32_t* hc = (const uint32_t*)c.hh;
  unsigned long long ovf_bytes;
  memcpy(&ovf_bytes, c.hh + hist_bytes, 8);
  if (ovf_bytes & kRawListTooLong)
    fail(CG_INVALID_ARGUMENT, "a header list beyond " + std::to_string(kFieldsMaxList) +
                                  " bytes (evaluate it with cg_http_pack)");
  // the meta word holds arena offsets / 16 in 24 bits: a batch whose long
  // strings need more than 256 MiB of arena runs as two halves (one head is
  // at most kRawMaxHead bytes, so halving always ends)
  if (ovf_bytes / 16 >= (1ull << 24)) {
    if (c.n < 2) fail(CG_INVALID_ARGUMENT, "overflow arena beyond 256 MiB");
    return false;
  }
  // ---- layout: groups in program order (then allow, deny), 64-slot tiles,
  // chunks of <= kChunkTiles tiles, runs of tiles with equal string units
  // (a tile's units: the bucket key of its last walked slot; keys ascend
  // within a group, overflow-arena slots last), a cursor per (group, key)
  std::vector<HttpChunk> chunks;
  std::vector<HttpRawRun> runs;
  std::vector<uint32_t> cursors((size_t)G * K, 0);
  uint32_t tiles = 0, gran = 0;
  auto add_run = [&](uint32_t t0, uint32_t t1, uint32_t units, uint32_t prog, uint32_t send) {
    if (t1 <= t0) return;
    runs.push_back({t0, units, gran, prog, send});
    gran += (t1 - t0) * (1 + 2 * units);
  };
  for (uint32_t g = 0; g < G; ++g) {
    uint32_t bstart[kRawKeys + 1], cnt = 0;
    for (uint32_t k = 0; k < K; ++k) {
      bstart[k] = cnt;
      cnt += hc[(size_t)g * K + k];
    }
    bstart[K] = cnt;
    if (!cnt) continue;
    const uint32_t prog = g < np ? g : g == np ? kProgAllow : kProgDeny;
    for (uint32_t k = 0; k < K; ++k) cursors[(size_t)g * K + k] = tiles * CG_HTTP_TILE + bstart[k];
    const uint32_t T = (cnt + CG_HTTP_TILE - 1) / CG_HTTP_TILE;
    for (uint32_t k = 0; k < T; k += kChunkTiles) chunks.push_back({prog, tiles + k, std::min(kChunkTiles, T - k), 0});
    // tiles j with a walked slot: units = key of slot min(64j + 63, e - 1)
    const uint32_t e = bstart[K - 1];
    uint32_t j = 0;
    while ((uint64_t)64 * j < e) {
      const uint32_t last = std::min(64 * j + 63, e - 1);
      uint32_t u = 0;
      for (uint32_t k = 0; k + 1 < K; ++k)
        if (bstart[k] <= last && last < bstart[k + 1]) u = k;
      const uint32_t next = bstart[u + 1];  // first slot of a larger key (or e)
      const uint32_t jend = next >= e ? (e + 63) / 64 : next / 64;
      add_run(tiles + j, tiles + jend, u, prog, tiles * CG_HTTP_TILE + cnt);
      j = jend;
    }
    add_run(tiles + j, tiles + T, 0, prog, tiles * CG_HTTP_TILE + cnt);  // only overflow-arena slots
    tiles += T;
  }
  const size_t nslots = (size_t)tiles * CG_HTTP_TILE;
  HttpBatchHeader hdr{};
  hdr.magic = kBatchMagic;
  hdr.epoch = s.epoch;
  hdr.nchunks = (uint32_t)chunks.size();
  hdr.ntiles = tiles;
  hdr.nslots = nslots;
  hdr.ttab_off = sizeof(HttpBatchHeader) + sizeof(HttpChunk) * chunks.size();
  hdr.tiles_off = (hdr.ttab_off + sizeof(HttpTile) * tiles + 1023) & ~(uint64_t)1023;
  hdr.total_bytes = hdr.tiles_off + (uint64_t)gran * 512;
  hdr.arena_bytes = ovf_bytes;
  uint8_t* batch = (uint8_t*)c.sl->dev_buf(10, hdr.total_bytes);
  const size_t head = hdr.ttab_off;
  uint8_t* hb = (uint8_t*)c.sl->host_buf(9, head + runs.size() * sizeof(HttpRawRun) + cursors.size() * 4);
  memcpy(hb, &hdr, sizeof(hdr));
  memcpy(hb + sizeof(hdr), chunks.data(), chunks.size() * sizeof(HttpChunk));
  uint8_t* hr = hb + head;
  memcpy(hr, runs.data(), runs.size() * sizeof(HttpRawRun));
  uint8_t* hcur = hr + runs.size() * sizeof(HttpRawRun);
  memcpy(hcur, cursors.data(), cursors.size() * 4);
  auto* d_runs = (HttpRawRun*)c.sl->dev_buf(11, std::max<size_t>(runs.size(), 1) * sizeof(HttpRawRun));
  auto* d_cursor = (uint32_t*)c.sl->dev_buf(12, cursors.size() * 4);
  hip_check(hipMemcpyAsync(batch, hb, head, hipMemcpyHostToDevice, c.st), "H2D");
  hip_check(hipMemcpyAsync(d_runs, hr, runs.size() * sizeof(HttpRawRun), hipMemcpyHostToDevice, c.st), "H2D");
  hip_check(hipMemcpyAsync(d_cursor, hcur, cursors.size() * 4, hipMemcpyHostToDevice, c.st), "H2D");
  uint8_t* arena = (uint8_t*)c.sl->dev_buf(13, std::max<unsigned long long>(ovf_bytes, 16));
  auto* order = (uint32_t*)c.sl->dev_buf(14, nslots * 4);  // padding entries: written by the build kernel
  auto* ttab = (HttpTile*)(batch + hdr.ttab_off);
  uint8_t* tdata = batch + hdr.tiles_off;
  const bool lists = c.in == RawInput::Lists;
  hip_check(launch_http_raw_rank(s.raw, lists, c.n, c.rinfo, d_cursor, c.bbase, order, c.st, c.cus),
            "raw rank kernel launch");
  hip_check(launch_http_raw_build(s.raw, d_runs, (uint32_t)runs.size(), tiles, ttab, tdata, order, c.sbuf, arena,
                                  c.ovf + 1, c.st, c.cus),
            "raw build kernel launch");
  hip_check(launch_http(s.dev, batch, nslots, arena, c.d_out, c.st, c.cus, order), "http kernel launch");
  return true;
}

// A call (or half) run start to end on its stream; halves when it is too
// large for one pass.
void raw_sequential(RawCall c) {
  if (!c.n) return;
  if (!raw_scan_phase(c) || !raw_rest_phase(c)) {
    const size_t h = c.n / 2;
    raw_sequential(c.half(0, h));
    raw_sequential(c.half(h, c.n - h));
    return;
  }
  // the workspace belongs to the lease: done before it is handed back
  hip_check(hipStreamSynchronize(c.st), "hipStreamSynchronize");
}

// Requests per sub-batch: the layout's bounds (slots, tiles, directory) are
// reserved for the worst case of a sub-batch — every request in one bucket,
// every string 8 units long — so the reservation is sized by requests, never
// by what the scan finds (no host round trip); 2^25 requests reserve ~4.8 GB
// of tile data on the 10K-rule set.
constexpr size_t kRawSubBatch = (size_t)1 << 25;
constexpr size_t kRawSubBatchMax = (size_t)1 << 27;  // CILIUM_GPU_RAW_SUBBATCH's ceiling

uint32_t floor_pow2(uint32_t x) {
  uint32_t p = 1;
  while (p * 2 <= x) p *= 2;
  return p;
}

// One sub-batch of the device-layout path, enqueued on `st`: clear the
// counters and tile table, scan, seal, http_kernel, walk.  The workspace is
// the slot's buffers 19..26 (the default sequence's are 8..18).
void raw_dl_subbatch(const HttpSnapshot& s, StagingSlot& sl, int cus, bool lists, const uint8_t* d_raw,
                  const uint64_t* d_off, size_t m, const uint32_t* d_policy, const uint8_t* d_ingress,
                  const uint16_t* d_port, const uint32_t* d_remote, uint8_t* d_out, hipStream_t st) {
  // slot counters striped per workgroup (RawLayoutDev.stripes): a bucket
  // key's requests take slots from `stripes` counters, so the returning
  // atomics of a hot key do not serialize on one address (8: measured best
  // of 4/8/16 on config 5, profiles/r05m_stripes.txt)
  uint32_t S = 8;
  if (const char* v = getenv("CILIUM_GPU_RAW_STRIPES")) S = floor_pow2((uint32_t)std::max(1, std::min(64, atoi(v))));
  const uint32_t np = (uint32_t)s.progs.size(), K = (np + 2) * kRawUnits * S;
  // tiles per chunk: the chunk table's 64 when the sub-batch fills several
  // chunks per bucket, fewer for small ones (each bucket's last chunk is
  // partly empty)
  const uint32_t ext = floor_pow2((uint32_t)std::min<size_t>(kChunkTiles, std::max<size_t>(1, m / (64 * (size_t)K))));
  uint32_t cshift = 6;
  while ((1u << cshift) < 64 * ext) ++cshift;
  const size_t per_chunk = (size_t)64 * ext;
  // directory entries per (key, stripe): the requests one stripe's
  // workgroups can take slots for — the scan's grid-stride share plus the
  // deferred kernel's (every request at most once in either)
  const size_t T = kRawScanThreads, itT = (m + T - 1) / T;
  auto share = [&](size_t grid) {
    grid = std::max<size_t>(grid, 1);
    return ((grid + S - 1) / S) * ((itT + grid - 1) / grid) * T;
  };
  const size_t per_stripe = std::min(m, share(http_raw_dl_grid(s.raw, lists, m, cus))) +
                            std::min(m, share((size_t)std::max(1, cus) * 2));
  const uint32_t dpk = (uint32_t)((std::min(m, per_stripe) + per_chunk - 1) / per_chunk);
  // every chunk holds a slot: at most m of them, and at most one partly
  // filled per (key, stripe)
  const uint32_t maxchunks = (uint32_t)std::min<size_t>(m, (m + per_chunk - 1) / per_chunk + K);
  const size_t maxtiles = (size_t)maxchunks * ext;
  if (maxtiles * kRawTileGran >= (1ull << 32)) fail(CG_INVALID_ARGUMENT, "raw batch layout too large");
  // batch: header, chunk table, tile table, tile data (1 KiB aligned)
  const uint64_t ttab_off = sizeof(HttpBatchHeader) + (uint64_t)sizeof(HttpChunk) * maxchunks;
  const uint64_t tiles_off = (ttab_off + sizeof(HttpTile) * maxtiles + 1023) & ~(uint64_t)1023;
  const uint64_t total = tiles_off + (uint64_t)maxtiles * kRawTileGran * 512;
  const size_t ctl_bytes = (size_t)K * kRawCntStride * 4 + kRawCtlWords * 4;
  const size_t dir_bytes = (size_t)K * dpk * 8;
  // the directory: fresh memory is cleared once (entries carry the
  // sub-batch tag, so a live one is never confused with an old one)
  const bool fresh_dir = !sl.dev[20].get() || sl.dev[20].size() < dir_bytes;
  RawLayoutDev L{};
  uint8_t* ctl = (uint8_t*)sl.dev_buf(19, ctl_bytes);
  L.kcnt = (uint32_t*)ctl;
  L.ctl = (uint32_t*)(ctl + (size_t)K * kRawCntStride * 4);
  L.dir = (unsigned long long*)sl.dev_buf(20, dir_bytes);
  if (fresh_dir) hip_check(hipMemsetAsync(L.dir, 0, sl.dev[20].size(), st), "hipMemsetAsync");
  uint8_t* batch = (uint8_t*)sl.dev_buf(21, total);
  L.ttab = (HttpTile*)(batch + ttab_off);
  L.tiles = batch + tiles_off;
  L.chunks = (HttpChunk*)sl.dev_buf(22, (size_t)maxchunks * sizeof(HttpChunk));
  L.order = (uint32_t*)sl.dev_buf(23, maxtiles * 64 * 4);
  L.walk = (uint32_t*)sl.dev_buf(24, m * 4);
  L.dlist = (uint32_t*)sl.dev_buf(25, m * 4);
  L.late = (unsigned long long*)sl.dev_buf(26, m * 8);
  // polls of a chunk id before a lane gives up (~15 ms: a legitimate wait is
  // microseconds); CILIUM_GPU_RAW_SPIN lowers it so tests reach the late path
  L.spin = 1u << 14;
  if (const char* v = getenv("CILIUM_GPU_RAW_SPIN")) L.spin = (uint32_t)std::min<unsigned long long>(L.spin, strtoull(v, nullptr, 10));
  L.dpk = dpk;
  L.ext = ext;
  L.cshift = cshift;
  L.seq = ++sl.raw_seq;
  if (!L.seq) L.seq = ++sl.raw_seq;  // 0 is the cleared directory's tag
  L.maxchunks = maxchunks;
  L.nkeys = K;
  L.stripes = S;
  hip_check(hipMemsetAsync(ctl, 0, ctl_bytes, st), "hipMemsetAsync");
  hip_check(hipMemsetAsync(L.ttab, 0, sizeof(HttpTile) * maxtiles, st), "hipMemsetAsync");
  hip_check(launch_http_raw_dl_scan(s.raw, lists, d_raw, d_off, m, d_policy, d_ingress, d_port, d_remote, L, st, cus),
            "raw scan kernel launch");
  hip_check(launch_http_raw_seal(s.raw, L, batch, s.epoch, ttab_off, tiles_off, total, st), "raw seal kernel launch");
  // the scan wrote raw bytes: class-mode programs code them as they walk
  hip_check(launch_http(s.dev, batch, maxtiles * 64, nullptr, d_out, st, cus, L.order, nullptr, (uint32_t)m, s.raw.codes),
            "http kernel launch");
  hip_check(launch_http_raw_walk(s.dev, s.raw, lists, d_raw, d_off, d_policy, d_ingress, d_port, d_remote, L, d_out,
                                 st, cus),
            "raw walk kernel launch");
}

// The device-layout path: sub-batches enqueued on `stream`, nothing waited
// for on the host.
void raw_device_layout(const HttpSnapshot& s, StagingSlot& sl, int cus, bool lists, const uint8_t* d_raw,
                       const uint64_t* d_off, size_t n, const uint32_t* d_policy, const uint8_t* d_ingress,
                       const uint16_t* d_port, const uint32_t* d_remote, uint8_t* d_out, void* stream) {
  const hipStream_t st = (hipStream_t)stream;
  // the slot's last raw call may still be queued on another stream: this
  // stream waits for it on the device (no host wait)
  if (sl.raw_ev && sl.raw_stream != stream) hip_check(hipStreamWaitEvent(st, (hipEvent_t)sl.raw_ev, 0), "hipStreamWaitEvent");
  // (CILIUM_GPU_RAW_SUBBATCH: another sub-batch size — smaller for tests, up
  // to 2^27 for the measurements of larger ones)
  size_t sub = kRawSubBatch;
  if (const char* v = getenv("CILIUM_GPU_RAW_SUBBATCH")) sub = std::min(kRawSubBatchMax, std::max<size_t>(64, strtoull(v, nullptr, 10)));
  for (size_t a = 0; a < n; a += sub) {
    const size_t m = std::min(sub, n - a);
    raw_dl_subbatch(s, sl, cus, lists, d_raw, d_off + a, m, d_policy + a, d_ingress + a, d_port + a, d_remote + a,
                 d_out + a, st);
  }
  if (!sl.raw_ev) {
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    sl.raw_ev = e;
  }
  hip_check(hipEventRecord((hipEvent_t)sl.raw_ev, st), "hipEventRecord");
  sl.raw_stream = stream;
}

// The device-layout path is the default (round 5: faster end to end and no
// host synchronization); CILIUM_GPU_RAW_LAYOUT=host selects the round-3
// sequence (read per call).
bool device_layout_selected() {
  const char* v = getenv("CILIUM_GPU_RAW_LAYOUT");
  return !(v && std::string(v) == "host");
}

}  // namespace

void http_verdicts_raw_on(const HttpSnapshot& s, StagingSlot& sl, int cus, RawInput in, const uint8_t* d_raw,
                          const uint64_t* d_off, size_t n, const uint32_t* d_policy, const uint8_t* d_ingress,
                          const uint16_t* d_port, const uint32_t* d_remote, uint8_t* d_out, void* stream) {
  const bool lists = in == RawInput::Lists;
  if (lists ? !s.lists_ok : !s.raw_ok)
    fail(CG_UNSUPPORTED, lists ? "header lists on the device: the snapshot has more than " +
                                     std::to_string(kRawMaxFields) + " header fields"
                               : "raw HTTP/1 heads: the snapshot has more than " + std::to_string(kRawMaxFields) +
                                     " header fields, or is a proxylib snapshot");
  if (!n) return;
  if (device_layout_selected()) {
    raw_device_layout(s, sl, cus, lists, d_raw, d_off, n, d_policy, d_ingress, d_port, d_remote, d_out, stream);
    return;
  }
  raw_sequential(RawCall{&s, &sl, cus, in, d_raw, d_off, n, d_policy, d_remote, d_ingress, d_port, d_out,
                         (hipStream_t)stream});
}

}  // namespace cg
