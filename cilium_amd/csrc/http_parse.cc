// http_parse.cc — HTTP/1.x request heads from raw bytes into the packer's
// header lists (what stands in front of
// AccessFilter::decodeHeaders, envoy/cilium_l7policy.cc:127-170).
//
// Two steps of Envoy run before the filter, restated here (neither is
// vendored; oracle/http1_ref.py lists the sources and what stays unpinned):
//  * the HTTP/1 codec, nodejs http_parser v2.8 (strict build):
//      request-line  [CR|LF]* method SP+ request-target SP "HTTP/1.1" EOL
//                    method from http_parser's method table; target bytes
//                    0x21-0x7E (strict normal_url_char)
//      header-field  token ":" OWS value OWS EOL; value bytes HTAB,
//                    0x20-0x7E, 0x80-0xFF (IS_HEADER_CHAR)
//      EOL           CR LF or a bare LF (a CR not followed by LF is an
//                    error); an empty line ends the head
//      Content-Length  a non-empty value is digits then SP only, at most
//                    once, bounded as h_content_length bounds it
//  * the connection manager's checks (conn_manager_impl.cc decodeHeaders):
//    only HTTP/1.1 (426 otherwise: accept_http_10 is off,
//    pkg/envoy/envoy/api/v2/core/protocol.pb.go:108-112, and Cilium's
//    listener sets no protocol options, pkg/envoy/server.go:172-215), Host
//    required (400), :path starting with '/' (404).
// What the filter then sees: :method, :path (the target as sent), Host as
// :authority (first value), the other headers in order, values OWS-trimmed.
// A request stopped before the filter is denied: its header list is a single
// entry the packer flags malformed, whatever policy index the caller packs
// it with.
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cilium_gpu.h"
#include "common.h"

namespace {

bool tchar(uint8_t c) {  // RFC 7230 token (http_parser tokens[])
  if (c >= '0' && c <= '9') return true;
  if ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') return true;
  return c && strchr("!#$%&'*+-.^_`|~", c) != nullptr;
}

bool header_char(uint8_t c) { return c == '\t' || (c >= 0x20 && c != 0x7F); }

// http_parser.h HTTP_METHOD_MAP (v2.8)
bool known_method(const uint8_t* p, size_t n) {
  static const char* const kMethods[] = {
      "DELETE",   "GET",        "HEAD",       "POST",     "PUT",       "CONNECT",     "OPTIONS", "TRACE",  "COPY",
      "LOCK",     "MKCOL",      "MOVE",       "PROPFIND", "PROPPATCH", "SEARCH",      "UNLOCK",  "BIND",   "REBIND",
      "UNBIND",   "ACL",        "REPORT",     "MKACTIVITY", "CHECKOUT", "MERGE",      "M-SEARCH", "NOTIFY", "SUBSCRIBE",
      "UNSUBSCRIBE", "PATCH",   "PURGE",      "MKCALENDAR", "LINK",    "UNLINK"};
  for (const char* m : kMethods)
    if (strlen(m) == n && memcmp(m, p, n) == 0) return true;
  return false;
}

bool ieq(const uint8_t* p, size_t n, const char* lower) {
  if (strlen(lower) != n) return false;
  for (size_t k = 0; k < n; ++k) {
    uint8_t c = p[k];
    if (c >= 'A' && c <= 'Z') c = (uint8_t)(c - 'A' + 'a');
    if (c != (uint8_t)lower[k]) return false;
  }
  return true;
}

// Parses one head; appends "name\0value\0" pairs to out.  false = stopped
// before the filter.
bool parse_head(const uint8_t* p, size_t n, std::string& out) {
  // Envoy's default max_request_headers_kb (60 KiB) rejects longer heads;
  // the device parser (kernels_http_raw.hip) applies the same bound
  if (n > 61440) return false;
  // [b, e) of the line starting at `from` and the start of the next one: a
  // line ends at LF, one CR before it is not part of it, a CR elsewhere is
  // an error (http_parser's *_almost_done states)
  auto next_line = [&](size_t from, size_t& e, size_t& nx) -> bool {
    const void* lf = memchr(p + from, '\n', n - from);
    if (!lf) return false;  // incomplete head
    const size_t l = (size_t)((const uint8_t*)lf - p);
    e = (l > from && p[l - 1] == '\r') ? l - 1 : l;
    nx = l + 1;
    return memchr(p + from, '\r', e - from) == nullptr;
  };
  size_t i = 0;
  while (i < n && (p[i] == '\r' || p[i] == '\n')) ++i;  // s_start_req
  size_t rl, nx;
  if (!next_line(i, rl, nx)) return false;
  // method
  size_t m = i;
  while (m < rl && tchar(p[m])) ++m;
  if (m >= rl || p[m] != ' ' || !known_method(p + i, m - i)) return false;
  // request-target after one or more SP: '/' then bytes 0x21-0x7E
  size_t t0 = m;
  while (t0 < rl && p[t0] == ' ') ++t0;
  size_t t = t0;
  while (t < rl && p[t] > 0x20 && p[t] < 0x7F) ++t;
  if (t == t0 || p[t0] != '/' || t >= rl || p[t] != ' ') return false;
  // version: HTTP/1.1 only
  if (rl - (t + 1) != 8 || memcmp(p + t + 1, "HTTP/1.1", 8) != 0) return false;
  std::string method((const char*)p + i, m - i), path((const char*)p + t0, t - t0), authority, rest;
  bool have_host = false, have_cl = false;
  i = nx;
  while (true) {
    size_t le;
    if (!next_line(i, le, nx)) return false;
    if (le == i) break;  // empty line: end of head
    size_t c = i;
    while (c < le && tchar(p[c])) ++c;
    if (c == i || c >= le || p[c] != ':') return false;
    size_t a = c + 1, b = le;
    while (a < b && (p[a] == ' ' || p[a] == '\t')) ++a;
    const size_t raw_a = a;
    while (b > a && (p[b - 1] == ' ' || p[b - 1] == '\t')) --b;
    for (size_t k = a; k < b; ++k)
      if (!header_char(p[k])) return false;
    if (ieq(p + i, c - i, "content-length") && raw_a < le) {  // h_content_length
      if (have_cl) return false;
      have_cl = true;
      uint64_t cl = 0;
      size_t k = raw_a;
      for (; k < le && p[k] >= '0' && p[k] <= '9'; ++k) {
        if (cl > (UINT64_MAX - 10) / 10) return false;
        cl = cl * 10 + (uint64_t)(p[k] - '0');
      }
      if (k == raw_a) return false;
      for (; k < le; ++k)
        if (p[k] != ' ') return false;
    }
    std::string name((const char*)p + i, c - i), value((const char*)p + a, b - a);
    if (ieq(p + i, c - i, "host")) {
      if (!have_host) authority = value;  // the first value is the one the filter sees
      have_host = true;
    } else {
      rest += name;
      rest.push_back('\0');
      rest += value;
      rest.push_back('\0');
    }
    i = nx;
  }
  if (!have_host) return false;  // conn_manager_impl: 400 without Host
  auto add = [&](const char* k, const std::string& val) {
    out += k;
    out.push_back('\0');
    out += val;
    out.push_back('\0');
  };
  add(":method", method);
  add(":path", path);
  add(":authority", authority);
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
