// http_raw.cc — host side of the raw HTTP/1 path (kernels_http_raw.hip):
// the snapshot's device tables for it, and the launch sequence
//   scan → (bucket counts to the host) → layout → tiles → emit → http_kernel
//   → scatter
// on one stream.  The host step is the layout of a few thousand bucket
// counts (groups, chunk table, bucket cursors); request bytes never leave the
// device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

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
  S.raw_ok = false;
  S.raw = HttpRawDev{};
  const uint32_t F = (uint32_t)S.fields.size();
  if (S.raw_values || F > kRawMaxFields) return;  // proxylib snapshots take escaped values, not heads
  HttpRawDev& R = S.raw;
  R.f_method = R.f_path = R.f_authority = -1;
  const uint32_t cap = next_pow2(std::max<uint32_t>(2 * F, 4));
  std::vector<uint32_t> slots(4 * (size_t)cap, 0);
  std::vector<uint8_t> names;
  for (uint32_t f = 0; f < F; ++f) {
    const std::string& nm = S.fields[f];
    if (nm == ":method") R.f_method = (int32_t)f;
    else if (nm == ":path") R.f_path = (int32_t)f;
    else if (nm == ":authority") R.f_authority = (int32_t)f;
    if (nm.empty() || nm[0] == ':') continue;  // pseudo headers never come from a header line
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
  std::vector<uint8_t> codes(std::max<size_t>(S.progs.size(), 1) * 256);
  for (size_t p = 0; p < S.progs.size(); ++p)
    for (int b = 0; b < 256; ++b)
      codes[p * 256 + b] = (S.progs[p].flags & kProgClass) ? S.prog_code[p][b] : (uint8_t)b;
  S.d_phk.upload_vec(S.phash_keys);
  S.d_phv.upload_vec(S.phash_vals);
  S.d_fslots.upload_vec(slots);
  S.d_fnames.upload_vec(names);
  S.d_codes.upload_vec(codes);
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
  R.codes = S.d_codes.as<uint8_t>();
  S.raw_ok = true;
}

void http_verdicts_raw_on(const HttpSnapshot& s, StagingSlot& sl, int cus, const uint8_t* d_raw,
                          const uint64_t* d_off, size_t n, const uint32_t* d_policy, const uint8_t* d_ingress,
                          const uint16_t* d_port, const uint32_t* d_remote, uint8_t* d_out, void* stream) {
  if (!s.raw_ok)
    fail(CG_UNSUPPORTED, "raw HTTP/1 heads: the snapshot has more than " + std::to_string(kRawMaxFields) +
                             " header fields, or is a proxylib snapshot");
  if (!n) return;
  const hipStream_t st = (hipStream_t)stream;
  const uint32_t np = (uint32_t)s.progs.size(), G = np + 2, K = kRawKeys;
  // workspace: [histogram G*K u32][overflow bytes u64][arena cursor u64]
  const size_t hist_bytes = ((size_t)G * K * 4 + 7) & ~(size_t)7;
  uint8_t* small = (uint8_t*)sl.dev_buf(8, hist_bytes + 16);
  uint32_t* hist = (uint32_t*)small;
  auto* ovf = (unsigned long long*)(small + hist_bytes);
  hip_check(hipMemsetAsync(small, 0, hist_bytes + 16, st), "hipMemsetAsync");
  void* rinfo = sl.dev_buf(9, n * 8);
  // per-block bucket counts → per-block slot offsets (when the bucket
  // counters fit the kernels' LDS), else one global histogram
  const bool lds_keys = http_raw_lds_keys(s.raw);
  const uint32_t nblk = (uint32_t)http_raw_grid(n, cus);
  uint32_t* bcount = lds_keys ? (uint32_t*)sl.dev_buf(16, (size_t)G * K * nblk * 4) : hist;
  uint32_t* bbase = lds_keys ? (uint32_t*)sl.dev_buf(17, (size_t)G * K * nblk * 4) : nullptr;
  auto* spans = (uint32_t*)sl.dev_buf(18, (size_t)std::max(s.raw.nfields, 1u) * n * 4);
  hip_check(launch_http_raw_scan(s.raw, d_raw, d_off, n, d_policy, d_ingress, d_port, bcount, rinfo, spans, ovf, st,
                                 cus),
            "raw scan kernel launch");
  if (lds_keys)
    hip_check(launch_http_raw_prefix(bcount, G * K, nblk, bbase, hist, st), "raw prefix kernel launch");
  uint8_t* hh = (uint8_t*)sl.host_buf(8, hist_bytes + 16);
  hip_check(hipMemcpyAsync(hh, small, hist_bytes + 8, hipMemcpyDeviceToHost, st), "D2H");
  hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  const uint32_t* hc = (const uint32_t*)hh;
  unsigned long long ovf_bytes;
  memcpy(&ovf_bytes, hh + hist_bytes, 8);
  if (ovf_bytes / 16 >= (1ull << 24)) {
    // the meta word holds arena offsets / 16 in 24 bits: a batch whose long
    // strings need more than 256 MiB of arena runs as two halves (one head
    // is at most kRawMaxHead bytes, so halving always ends)
    if (n < 2) fail(CG_INVALID_ARGUMENT, "overflow arena beyond 256 MiB");
    const size_t h = n / 2;
    http_verdicts_raw_on(s, sl, cus, d_raw, d_off, h, d_policy, d_ingress, d_port, d_remote, d_out, stream);
    http_verdicts_raw_on(s, sl, cus, d_raw, d_off + h, n - h, d_policy + h, d_ingress + h, d_port + h, d_remote + h,
                         d_out + h, stream);
    return;
  }
  // ---- layout: groups in program order (then allow, deny), 64-slot tiles,
  // chunks of <= kChunkTiles tiles, a cursor per (group, bucket)
  std::vector<HttpRawGroup> groups;
  std::vector<HttpChunk> chunks;
  std::vector<uint32_t> cursors((size_t)G * K, 0);
  uint32_t tiles = 0;
  for (uint32_t g = 0; g < G; ++g) {
    HttpRawGroup gr{};
    uint32_t cnt = 0;
    for (uint32_t k = 0; k < K; ++k) {
      gr.bstart[k] = cnt;
      cnt += hc[(size_t)g * K + k];
    }
    gr.bstart[K] = cnt;
    if (!cnt) continue;
    gr.tile0 = tiles;
    gr.count = cnt;
    gr.prog = g < np ? g : g == np ? kProgAllow : kProgDeny;
    for (uint32_t k = 0; k < K; ++k) cursors[(size_t)g * K + k] = tiles * CG_HTTP_TILE + gr.bstart[k];
    const uint32_t t = (cnt + CG_HTTP_TILE - 1) / CG_HTTP_TILE;
    for (uint32_t k = 0; k < t; k += kChunkTiles) chunks.push_back({gr.prog, tiles + k, std::min(kChunkTiles, t - k), 0});
    tiles += t;
    groups.push_back(gr);
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
  hdr.total_bytes = hdr.tiles_off + (uint64_t)tiles * kRawTileGranules * 512;
  hdr.arena_bytes = ovf_bytes;
  uint8_t* batch = (uint8_t*)sl.dev_buf(10, hdr.total_bytes);
  const size_t head = hdr.ttab_off;
  uint8_t* hb = (uint8_t*)sl.host_buf(9, head + groups.size() * sizeof(HttpRawGroup) + cursors.size() * 4);
  memcpy(hb, &hdr, sizeof(hdr));
  memcpy(hb + sizeof(hdr), chunks.data(), chunks.size() * sizeof(HttpChunk));
  uint8_t* hg = hb + head;
  memcpy(hg, groups.data(), groups.size() * sizeof(HttpRawGroup));
  uint8_t* hcur = hg + groups.size() * sizeof(HttpRawGroup);
  memcpy(hcur, cursors.data(), cursors.size() * 4);
  auto* d_groups = (HttpRawGroup*)sl.dev_buf(11, std::max<size_t>(groups.size(), 1) * sizeof(HttpRawGroup));
  auto* d_cursor = (uint32_t*)sl.dev_buf(12, cursors.size() * 4);
  hip_check(hipMemcpyAsync(batch, hb, head, hipMemcpyHostToDevice, st), "H2D");
  hip_check(hipMemcpyAsync(d_groups, hg, groups.size() * sizeof(HttpRawGroup), hipMemcpyHostToDevice, st), "H2D");
  hip_check(hipMemcpyAsync(d_cursor, hcur, cursors.size() * 4, hipMemcpyHostToDevice, st), "H2D");
  uint8_t* arena = (uint8_t*)sl.dev_buf(13, std::max<unsigned long long>(ovf_bytes, 16));
  auto* order = (uint32_t*)sl.dev_buf(14, nslots * 4);
  uint8_t* vslot = (uint8_t*)sl.dev_buf(15, nslots);
  auto* ttab = (HttpTile*)(batch + hdr.ttab_off);
  uint8_t* tdata = batch + hdr.tiles_off;
  hip_check(launch_http_raw_tiles(d_groups, (uint32_t)groups.size(), tiles, ttab, tdata, order, st),
            "raw tiles kernel launch");
  hip_check(launch_http_raw_emit(s.raw, d_raw, d_off, n, d_ingress, d_remote, rinfo, d_cursor, bbase, ttab, tdata,
                                 order, arena, ovf + 1, spans, st, cus),
            "raw emit kernel launch");
  hip_check(launch_http(s.dev, batch, nslots, arena, vslot, st, cus), "http kernel launch");
  hip_check(launch_http_raw_scatter(order, vslot, nslots, d_out, st, cus), "raw scatter kernel launch");
  // the workspace belongs to the lease: done before it is handed back
  hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
}

}  // namespace cg
