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
  // structural checks the kernels rely on
  if (s.phash_keys.size() != (size_t)s.phash_mask + 1 || s.phash_vals.size() != s.phash_keys.size())
    fail(CG_POLICY_REJECTED, "policy image: bad program hash");
  if (s.dflt.size() < (size_t)s.npolicies * 2 || s.prog_code.size() != s.progs.size() ||
      s.prog_key.size() > s.progs.size())
    fail(CG_POLICY_REJECTED, "policy image: inconsistent tables");
  for (const auto& pg : s.progs)
    if ((size_t)pg.part_begin + pg.part_count > s.parts.size() || (size_t)pg.cell_begin + pg.cell_count > s.cells.size())
      fail(CG_POLICY_REJECTED, "policy image: program out of range");
  for (const auto& pt : s.parts)
    if ((size_t)pt.walk_off + pt.ncells > s.cells.size() && pt.ncells)
      fail(CG_POLICY_REJECTED, "policy image: part out of range");
  s.epoch = http_next_epoch();
  return snap;
}

}  // namespace cg
