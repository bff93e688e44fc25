// go_text.h — Go runtime string semantics the proxylib parsers rely on
// (Go 1.10, the reference's runtime):
//   utf8.DecodeRune          invalid / overlong / surrogate sequences decode
//                            as U+FFFD of width 1
//   utf8.EncodeRune
//   unicode.IsSpace          the Latin-1 and White_Space sets
//   unicode.ToLower          simple case mapping (go_lower_table.h)
//   strings.ToLower          ASCII fast path, else strings.Map(unicode.ToLower):
//                            bytes before the first changed rune are kept as
//                            they are, runes after it re-encoded (an invalid
//                            byte there becomes EF BF BD)
//   strings.Fields / bytes.Fields  runs of !unicode.IsSpace over decoded runes
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "go_lower_table.h"

namespace cg {
namespace go {

constexpr uint32_t kRuneError = 0xFFFD;

inline uint32_t decode_rune(const uint8_t* p, size_t n, size_t* w) {
  const uint8_t c = p[0];
  *w = 1;
  if (c < 0x80) return c;
  auto cont = [&](size_t i) { return i < n && (p[i] & 0xC0) == 0x80; };
  if (c >= 0xC2 && c <= 0xDF && cont(1)) {
    *w = 2;
    return (uint32_t)(c & 0x1F) << 6 | (p[1] & 0x3F);
  }
  if (c >= 0xE0 && c <= 0xEF && cont(1) && cont(2)) {
    if (c == 0xE0 && p[1] < 0xA0) return kRuneError;  // overlong
    if (c == 0xED && p[1] > 0x9F) return kRuneError;  // surrogate
    *w = 3;
    return (uint32_t)(c & 0x0F) << 12 | (uint32_t)(p[1] & 0x3F) << 6 | (p[2] & 0x3F);
  }
  if (c >= 0xF0 && c <= 0xF4 && cont(1) && cont(2) && cont(3)) {
    if (c == 0xF0 && p[1] < 0x90) return kRuneError;
    if (c == 0xF4 && p[1] > 0x8F) return kRuneError;
    *w = 4;
    return (uint32_t)(c & 0x07) << 18 | (uint32_t)(p[1] & 0x3F) << 12 | (uint32_t)(p[2] & 0x3F) << 6 | (p[3] & 0x3F);
  }
  return kRuneError;
}

inline void encode_rune(std::string& out, uint32_t r) {
  if (r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) r = kRuneError;
  if (r < 0x80) {
    out += (char)r;
  } else if (r < 0x800) {
    out += (char)(0xC0 | r >> 6);
    out += (char)(0x80 | (r & 0x3F));
  } else if (r < 0x10000) {
    out += (char)(0xE0 | r >> 12);
    out += (char)(0x80 | (r >> 6 & 0x3F));
    out += (char)(0x80 | (r & 0x3F));
  } else {
    out += (char)(0xF0 | r >> 18);
    out += (char)(0x80 | (r >> 12 & 0x3F));
    out += (char)(0x80 | (r >> 6 & 0x3F));
    out += (char)(0x80 | (r & 0x3F));
  }
}

inline bool is_space(uint32_t r) {
  switch (r) {
    case '\t': case '\n': case '\v': case '\f': case '\r': case ' ': case 0x85: case 0xA0:
    case 0x1680: case 0x2028: case 0x2029: case 0x202F: case 0x205F: case 0x3000:
      return true;
    default:
      return r >= 0x2000 && r <= 0x200A;
  }
}

inline uint32_t to_lower(uint32_t r) {
  if (r < 0x80) return (r >= 'A' && r <= 'Z') ? r + 32 : r;
  size_t lo = 0, hi = sizeof(kGoLower) / sizeof(kGoLower[0]);
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (kGoLower[mid].hi < r) lo = mid + 1;
    else hi = mid;
  }
  if (lo < sizeof(kGoLower) / sizeof(kGoLower[0])) {
    const GoCaseRange& g = kGoLower[lo];
    if (r >= g.lo && r <= g.hi && (r - g.lo) % g.stride == 0) return (uint32_t)((int32_t)r + g.delta);
  }
  return r;
}

// strings.ToLower (Go 1.10 strings.go / strings.Map)
inline std::string to_lower(std::string_view s) {
  bool ascii = true;
  for (unsigned char c : s)
    if (c >= 0x80) {
      ascii = false;
      break;
    }
  if (ascii) {
    std::string o(s);
    for (char& c : o)
      if (c >= 'A' && c <= 'Z') c = (char)(c + 32);
    return o;
  }
  const uint8_t* p = (const uint8_t*)s.data();
  const size_t n = s.size();
  size_t i = 0;
  while (i < n) {  // the first rune the mapping changes
    size_t w;
    const uint32_t c = decode_rune(p + i, n - i, &w);
    if (to_lower(c) != c) break;
    i += w;
  }
  if (i == n) return std::string(s);
  std::string out(s.substr(0, i));
  while (i < n) {
    size_t w;
    const uint32_t c = decode_rune(p + i, n - i, &w);
    encode_rune(out, to_lower(c));
    i += w;
  }
  return out;
}

// strings.Fields / bytes.Fields
inline std::vector<std::string> fields(std::string_view s) {
  std::vector<std::string> out;
  const uint8_t* p = (const uint8_t*)s.data();
  size_t i = 0, start = 0;
  bool in = false;
  while (i < s.size()) {
    size_t w;
    const uint32_t r = decode_rune(p + i, s.size() - i, &w);
    if (is_space(r)) {
      if (in) out.emplace_back(s.substr(start, i - start));
      in = false;
    } else if (!in) {
      in = true;
      start = i;
    }
    i += w;
  }
  if (in) out.emplace_back(s.substr(start));
  return out;
}

}  // namespace go
}  // namespace cg
