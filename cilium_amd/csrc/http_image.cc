// http_image.cc — a compiled HTTP policy snapshot as a flat byte image:
// cg_http_policy_export writes it, cg_http_policy_import publishes it on
// another handle (another GPU or process) without recompiling.  SURVEY
// §8(e): the host compiles once and every GPU uploads an identical image;
// it is also the serialized table cache of §5 (checkpoint / resume).
//
// Layout (little-endian): magic "CGHI", version, then the snapshot's members
// in declaration order — counts before arrays, POD arrays as raw bytes, strings
// as u32 length + bytes — and an FNV-1a 64 checksum of everything before it.
// Images are only exchanged between builds of the same library (the POD
// layouts of dev_types.h); the version word and the size checks reject
// anything else with CG_POLICY_REJECTED.
#include <cstring>
#include <string>
#include <vector>

#include "comb.h"
#include "http.h"

namespace cg {

namespace {

constexpr uint32_t kImageMagic = 0x49484743u;  // "CGHI"
constexpr uint32_t kImageVersion = 1u | (uint32_t)sizeof(HttpProg) << 8 | (uint32_t)sizeof(HttpPart) << 16 |
                                   (uint32_t)sizeof(cg_http_rule_info) << 24;

uint64_t fnv64(const uint8_t* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

struct Writer {
  std::vector<uint8_t> b;
  void raw(const void* p, size_t n) {
    const uint8_t* q = static_cast<const uint8_t*>(p);
    b.insert(b.end(), q, q + n);
  }
  void u32(uint32_t v) { raw(&v, 4); }
  void u64(uint64_t v) { raw(&v, 8); }
  void str(const std::string& s) {
    u32((uint32_t)s.size());
    raw(s.data(), s.size());
  }
  template <class T>
  void vec(const std::vector<T>& v) {
    u64(v.size());
    raw(v.data(), v.size() * sizeof(T));
  }
};

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  void raw(void* dst, size_t n) {
    if ((size_t)(e - p) < n) fail(CG_POLICY_REJECTED, "policy image: truncated");
    memcpy(dst, p, n);
    p += n;
  }
  uint32_t u32() {
    uint32_t v;
    raw(&v, 4);
    return v;
  }
  uint64_t u64() {
    uint64_t v;
    raw(&v, 8);
    return v;
  }
  std::string str() {
    const uint32_t n = u32();
    if ((size_t)(e - p) < n) fail(CG_POLICY_REJECTED, "policy image: truncated");
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
  template <class T>
  void vec(std::vector<T>* v) {
    const uint64_t n = u64();
    if (n > (uint64_t)(e - p) / sizeof(T)) fail(CG_POLICY_REJECTED, "policy image: truncated");
    v->resize((size_t)n);
    raw(v->data(), (size_t)n * sizeof(T));
  }
};

}  // namespace

std::vector<uint8_t> http_image_export(const HttpSnapshot& s) {
  Writer w;
  w.u32(kImageMagic);
  w.u32(kImageVersion);
  w.u32(s.raw_values ? 1u : 0u);
  w.u32((uint32_t)s.fields.size());
  for (const auto& f : s.fields) w.str(f);
  w.u32((uint32_t)s.policy_index.size());
  for (const auto& [name, idx] : s.policy_index) {
    w.str(name);
    w.u32(idx);
  }
  w.u32(s.npolicies);
  w.vec(s.progs);
  w.vec(s.parts);
  w.vec(s.cells);
  w.vec(s.phash_keys);
  w.vec(s.phash_vals);
  w.u32(s.phash_mask);
  w.vec(s.dflt);
  w.vec(s.prog_key);
  w.vec(s.prog_code);
  w.vec(s.rule_info);
  w.u64(s.total_states);
  w.u64(s.total_exceptions);
  w.u64(s.total_rules);
  w.u64(s.total_remote_slots);
  w.u64(fnv64(w.b.data(), w.b.size()));
  return std::move(w.b);
}

// Every index the kernels and the host walker follow, checked before an
// imported image is published: the image crosses a trust boundary (the
// checkpoint/resume cache, another process) and its FNV checksum is no MAC.
void validate_image(const HttpSnapshot& s) {
  auto bad = [](const char* what) { fail(CG_POLICY_REJECTED, std::string("policy image: ") + what); };
  const size_t np = s.progs.size(), nc = s.cells.size();
  auto prog_ref_ok = [&](uint32_t v) { return v < np || v == kProgAllow || v == kProgDeny; };
  if (s.phash_keys.size() != (size_t)s.phash_mask + 1 || s.phash_vals.size() != s.phash_keys.size())
    bad("bad program hash");
  bool empty_slot = false;
  for (size_t i = 0; i < s.phash_keys.size(); ++i) {
    empty_slot |= s.phash_keys[i] == 0xFFFFFFFFu;
    if (s.phash_keys[i] != 0xFFFFFFFFu && !prog_ref_ok(s.phash_vals[i])) bad("program hash value out of range");
  }
  if (!empty_slot) bad("program hash has no empty slot");  // lookups would probe forever
  if (s.dflt.size() < (size_t)s.npolicies * 2 || s.prog_code.size() != np || s.prog_key.size() > np)
    bad("inconsistent tables");
  for (uint32_t v : s.dflt)
    if (!prog_ref_ok(v)) bad("default program out of range");
  for (const auto& [name, idx] : s.policy_index)
    if (idx >= s.npolicies) bad("policy index out of range");
  for (size_t pi = 0; pi < np; ++pi) {
    const HttpProg& pg = s.progs[pi];
    if ((size_t)pg.part_begin + pg.part_count > s.parts.size() || (size_t)pg.cell_begin + pg.cell_count > nc)
      bad("program out of range");
    if (pg.flags & kProgAllowAll) continue;  // never walked
    const uint64_t W = pg.mask_words, blk = pg.cell_count;
    if (W == 0 || W > (1u << 16)) bad("bad mask width");
    if ((uint64_t)pg.rule_base + pg.nrules > s.rule_info.size() || pg.nrules > 64 * W) bad("rule range out of range");
    const uint32_t* b = s.cells.data() + pg.cell_begin;
    // a PNPR mask at block offset o: inside the block, no bit past nrules
    auto mask_ok = [&](uint64_t o, bool check_bits) {
      if (o + 2 * W > blk) return false;
      if (check_bits)
        for (uint64_t w = 0; w < W; ++w) {
          const uint64_t m = (uint64_t)b[o + 2 * w] | (uint64_t)b[o + 2 * w + 1] << 32;
          for (uint32_t bit = 0; bit < 64; ++bit)
            if (((m >> bit) & 1) && w * 64 + bit >= pg.nrules) return false;
        }
      return true;
    };
    if (!mask_ok(pg.always_off, true) || !mask_ok(pg.default_remote, false)) bad("program mask out of range");
    if (pg.flags & kProgRemoteDirect) {
      if (pg.rdir_len > kRdirMaxSpan || (uint64_t)pg.rdir_off + (pg.rdir_len + 1) / 2 > blk)
        bad("remote direct array out of range");
      const uint16_t* d = (const uint16_t*)(b + pg.rdir_off);
      for (uint32_t i = 0; i < pg.rdir_len; ++i)
        if (!mask_ok(d[i], false)) bad("remote row out of range");
    } else {
      if (pg.rtab_nb == 0 || (uint64_t)pg.rtab_off + (uint64_t)kRtabBucketCells * pg.rtab_nb > blk)
        bad("remote table out of range");
      for (uint32_t k = 0; k < pg.rtab_nb; ++k)
        for (uint32_t sl = 0; sl < 4; ++sl) {
          const uint32_t* bk = b + pg.rtab_off + kRtabBucketCells * k;
          if (bk[sl] != kNoRow && !mask_ok(bk[4 + sl], false)) bad("remote row out of range");
        }
    }
    // the largest code a class-mode string byte can carry
    uint32_t max_code = 255;
    if (pg.flags & kProgClass) {
      max_code = 0;
      for (uint8_t c : s.prog_code[pi]) {
        if (c & 3) bad("class code not a cell offset");
        max_code = std::max<uint32_t>(max_code, c);
      }
    }
    const bool rebased = pg.flags & kProgRebased;
    const uint64_t limit = rebased ? (uint64_t)pg.cell_begin + pg.cell_count : nc;
    for (uint32_t k = 0; k < pg.part_count; ++k) {
      const HttpPart& pt = s.parts[pg.part_begin + k];
      if (pt.mode != 0 && pt.mode != kPartClass) bad("bad part mode");
      const bool scaled = pt.mode == kPartClass;
      if (scaled != ((pg.flags & kProgClass) != 0)) bad("class mode mismatch");
      if ((rebased && pt.walk_off != pg.cell_begin) || pt.cell_off < pt.walk_off ||
          (uint64_t)pt.cell_off + pt.ncells > limit)
        bad("part out of range");
      // a state's header cell and every cell a step from it can read
      auto state_ok = [&](uint64_t st) {
        if (scaled && (st & 3)) return false;
        const uint64_t lo = scaled ? st >> 2 : st, hi = scaled ? (st + max_code) >> 2 : st + 255;
        return lo >= 1 && pt.walk_off + hi < limit;
      };
      if (!state_ok(pt.start) || !state_ok(pt.dead)) bad("part state out of range");
      for (uint64_t i = pt.cell_off; i < (uint64_t)pt.cell_off + pt.ncells; ++i) {
        const uint32_t c = s.cells[i];
        if (c == kCombEmpty) continue;
        if ((c & 0xFFFF) == 0xFFFF) {  // header: accept label
          const uint32_t lab = c >> 16;
          if (lab != kCombNoLabel && !mask_ok((uint64_t)pt.acc_off + (uint64_t)lab * 2 * W, true))
            bad("accept label out of range");
        } else if (!state_ok(c >> 16)) {
          bad("transition out of range");
        }
      }
    }
  }
}

std::shared_ptr<HttpSnapshot> http_image_import(const uint8_t* p, size_t n) {
  if (!p || n < 16) fail(CG_POLICY_REJECTED, "policy image: too short");
  uint64_t sum;
  memcpy(&sum, p + n - 8, 8);
  if (sum != fnv64(p, n - 8)) fail(CG_POLICY_REJECTED, "policy image: checksum mismatch");
  Reader r{p, p + n - 8};
  if (r.u32() != kImageMagic) fail(CG_POLICY_REJECTED, "policy image: bad magic");
  if (r.u32() != kImageVersion) fail(CG_POLICY_REJECTED, "policy image: built by another library version");
  auto snap = std::make_shared<HttpSnapshot>();
  HttpSnapshot& s = *snap;
  s.raw_values = r.u32() != 0;
  const uint32_t nf = r.u32();
  if (nf > (1u << 20)) fail(CG_POLICY_REJECTED, "policy image: bad field count");
  for (uint32_t i = 0; i < nf; ++i) s.fields.push_back(r.str());
  const uint32_t np = r.u32();
  for (uint32_t i = 0; i < np; ++i) {
    std::string name = r.str();
    s.policy_index[name] = r.u32();
  }
  s.npolicies = r.u32();
  r.vec(&s.progs);
  r.vec(&s.parts);
  r.vec(&s.cells);
  r.vec(&s.phash_keys);
  r.vec(&s.phash_vals);
  s.phash_mask = r.u32();
  r.vec(&s.dflt);
  r.vec(&s.prog_key);
  r.vec(&s.prog_code);
  r.vec(&s.rule_info);
  s.total_states = r.u64();
  s.total_exceptions = r.u64();
  s.total_rules = r.u64();
  s.total_remote_slots = r.u64();
  if (r.p != r.e) fail(CG_POLICY_REJECTED, "policy image: trailing bytes");
  validate_image(s);
  s.epoch = http_next_epoch();
  return snap;
}

}  // namespace cg
