// http_parse.cc — HTTP/1.x request heads from raw bytes into the packer's
// header lists (the Envoy codec step in front of
// AccessFilter::decodeHeaders, envoy/cilium_l7policy.cc:127-170).
//
// The codec is Envoy's http_parser (external, not vendored: parity for this
// step is unpinned).  What it hands the filter, restated:
//   request-line  method SP request-target SP "HTTP/" DIGIT "." DIGIT CRLF
//                 → :method, :path (the target as sent, query included)
//   header-field  field-name ":" OWS field-value OWS CRLF, names are tokens,
//                 values hold no control byte but HTAB (IS_HEADER_CHAR)
//                 → the header; "Host" becomes :authority
//   CRLF          ends the head; a head without it is incomplete.
// A request the codec would reject never reaches the filter (Envoy answers
// 400): its header list is a single entry the packer flags malformed, so it
// is denied whatever policy index the caller packs it with.
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cilium_gpu.h"
#include "common.h"

namespace {

bool tchar(uint8_t c) {  // RFC 7230 token
  if (c >= '0' && c <= '9') return true;
  if ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') return true;
  return c && strchr("!#$%&'*+-.^_`|~", c) != nullptr;
}

bool header_char(uint8_t c) { return c == '\t' || (c >= 0x20 && c != 0x7F); }

// Parses one head; appends "name\0value\0" pairs to out.  false = rejected.
bool parse_head(const uint8_t* p, size_t n, std::string& out) {
  // Envoy's default max_request_headers_kb (60 KiB) rejects longer heads;
  // the device parser (kernels_http_raw.hip) applies the same bound
  if (n > 61440) return false;
  size_t i = 0;
  auto line_end = [&](size_t from) -> size_t {
    for (size_t k = from; k + 1 < n; ++k)
      if (p[k] == '\r' && p[k + 1] == '\n') return k;
    return std::string::npos;
  };
  const size_t rl = line_end(0);
  if (rl == std::string::npos) return false;
  // method
  size_t m = 0;
  while (m < rl && tchar(p[m])) ++m;
  if (m == 0 || m >= rl || p[m] != ' ') return false;
  // request-target
  size_t t0 = m + 1, t = t0;
  while (t < rl && p[t] > 0x20 && p[t] != 0x7F) ++t;
  if (t == t0 || t >= rl || p[t] != ' ') return false;
  // version
  const size_t v = t + 1;
  if (rl - v != 8 || memcmp(p + v, "HTTP/", 5) != 0 || p[v + 5] < '0' || p[v + 5] > '9' || p[v + 6] != '.' ||
      p[v + 7] < '0' || p[v + 7] > '9')
    return false;
  std::string method((const char*)p, m), path((const char*)p + t0, t - t0), authority, rest;
  bool have_host = false;
  i = rl + 2;
  while (true) {
    const size_t le = line_end(i);
    if (le == std::string::npos) return false;  // incomplete head
    if (le == i) break;                          // empty line: end of head
    size_t c = i;
    while (c < le && tchar(p[c])) ++c;
    if (c == i || c >= le || p[c] != ':') return false;
    size_t a = c + 1, b = le;
    while (a < b && (p[a] == ' ' || p[a] == '\t')) ++a;
    while (b > a && (p[b - 1] == ' ' || p[b - 1] == '\t')) --b;
    for (size_t k = a; k < b; ++k)
      if (!header_char(p[k])) return false;
    std::string name((const char*)p + i, c - i), value((const char*)p + a, b - a);
    std::string lname = name;
    for (auto& ch : lname)
      if (ch >= 'A' && ch <= 'Z') ch = (char)(ch - 'A' + 'a');
    if (lname == "host") {
      if (!have_host) authority = value;  // the first value is the one the filter sees
      have_host = true;
    } else {
      rest += name;
      rest.push_back('\0');
      rest += value;
      rest.push_back('\0');
    }
    i = le + 2;
  }
  auto add = [&](const char* k, const std::string& val) {
    out += k;
    out.push_back('\0');
    out += val;
    out.push_back('\0');
  };
  add(":method", method);
  add(":path", path);
  if (have_host) add(":authority", authority);
  out += rest;
  return true;
}

}  // namespace

extern "C" {

int cg_http_parse_heads(const uint8_t* raw, const uint64_t* raw_off, size_t n, uint8_t* hdr_blob, size_t blob_cap,
                        uint64_t* hdr_off, size_t* blob_used, uint8_t* ok) {
  if (n && (!raw || !raw_off)) return CG_INVALID_ARGUMENT;
  std::string blob;
  std::vector<uint64_t> off{0};
  std::vector<uint8_t> good(n);
  for (size_t r = 0; r < n; ++r) {
    if (raw_off[r + 1] < raw_off[r]) return CG_INVALID_ARGUMENT;
    std::string one;
    good[r] = parse_head(raw + raw_off[r], (size_t)(raw_off[r + 1] - raw_off[r]), one);
    // a rejected head carries one entry whose value holds DEL, a byte the
    // packer's codec rule flags CG_HTTP_F_MALFORMED: it is denied even when
    // the caller ignores ok[] (or its port has no HTTP rules)
    blob += good[r] ? one : std::string(":cg-rejected\0\x7f\0", 15);
    off.push_back(blob.size());
  }
  if (blob_used) *blob_used = blob.size();
  if (!hdr_blob) return CG_OK;  // size query
  if (blob.size() > blob_cap || !hdr_off) return CG_INVALID_ARGUMENT;
  memcpy(hdr_blob, blob.data(), blob.size());
  memcpy(hdr_off, off.data(), off.size() * sizeof(uint64_t));
  if (ok) memcpy(ok, good.data(), n);
  return CG_OK;
}

}  // extern "C"
