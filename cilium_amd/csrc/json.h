// json.h — minimal JSON reader for policy updates (NPDS protobuf-JSON form
// and the Kafka L7DataMap form).  Strings decode \uXXXX to UTF-8; integers
// keep full 64-bit precision.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "common.h"

namespace cg {

struct Json {
  enum Type { NUL, BOOL, NUM, STR, ARR, OBJ } type = NUL;
  bool b = false;
  bool is_int = false;
  bool neg = false;
  uint64_t u = 0;  // magnitude when is_int
  double d = 0;
  std::string s;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;

  const Json* get(const std::string& k) const {
    if (type != OBJ) return nullptr;
    for (const auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  uint64_t as_u64(const char* what) const {
    if (type == STR) {  // protobuf-JSON encodes 64-bit ints as strings
      uint64_t v = 0;
      if (s.empty()) fail(CG_POLICY_REJECTED, std::string("bad integer for ") + what);
      for (char c : s) {
        if (c < '0' || c > '9') fail(CG_POLICY_REJECTED, std::string("bad integer for ") + what);
        v = v * 10 + (c - '0');
      }
      return v;
    }
    if (type != NUM || !is_int || neg) fail(CG_POLICY_REJECTED, std::string("expected unsigned integer for ") + what);
    return u;
  }
  int64_t as_i64(const char* what) const {
    if (type == STR) {  // protobuf-JSON encodes 64-bit ints as strings
      const bool minus = !s.empty() && s[0] == '-';
      uint64_t v = 0;
      if (s.size() == (size_t)minus) fail(CG_POLICY_REJECTED, std::string("bad integer for ") + what);
      for (size_t i = minus; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9' || v > (uint64_t)1 << 63) fail(CG_POLICY_REJECTED, std::string("bad integer for ") + what);
        v = v * 10 + (s[i] - '0');
      }
      if (v > (minus ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1)) fail(CG_POLICY_REJECTED, std::string("int64 out of range for ") + what);
      return minus ? (int64_t)(0 - v) : (int64_t)v;
    }
    if (type != NUM || !is_int || u > (neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1))
      fail(CG_POLICY_REJECTED, std::string("expected int64 for ") + what);
    return neg ? (int64_t)(0 - u) : (int64_t)u;
  }
  const std::string& as_str(const char* what) const {
    if (type != STR) fail(CG_POLICY_REJECTED, std::string("expected string for ") + what);
    return s;
  }
};

class JsonParser {
 public:
  JsonParser(const char* p, size_t n) : p_(p), e_(p + n) {}
  Json parse() {
    Json v = value(0);
    ws();
    if (p_ != e_) bad("trailing data");
    return v;
  }

 private:
  const char* p_;
  const char* e_;
  [[noreturn]] void bad(const char* m) { fail(CG_POLICY_REJECTED, std::string("json: ") + m); }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  bool lit(const char* w) {
    size_t n = strlen(w);
    if ((size_t)(e_ - p_) >= n && memcmp(p_, w, n) == 0) {
      p_ += n;
      return true;
    }
    return false;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) {
      o += (char)cp;
    } else if (cp < 0x800) {
      o += (char)(0xC0 | (cp >> 6));
      o += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      o += (char)(0xE0 | (cp >> 12));
      o += (char)(0x80 | ((cp >> 6) & 0x3F));
      o += (char)(0x80 | (cp & 0x3F));
    } else {
      o += (char)(0xF0 | (cp >> 18));
      o += (char)(0x80 | ((cp >> 12) & 0x3F));
      o += (char)(0x80 | ((cp >> 6) & 0x3F));
      o += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (e_ - p_ < 4) bad("bad \\u");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else bad("bad \\u");
    }
    return v;
  }
  std::string str() {
    // p_ at opening quote
    ++p_;
    std::string o;
    while (true) {
      if (p_ >= e_) bad("unterminated string");
      char c = *p_++;
      if (c == '"') break;
      if (c != '\\') {
        o += c;
        continue;
      }
      if (p_ >= e_) bad("bad escape");
      char x = *p_++;
      switch (x) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(o, cp);
          break;
        }
        default: bad("bad escape");
      }
    }
    return o;
  }
  Json value(int depth) {
    if (depth > 64) bad("nesting too deep");
    ws();
    if (p_ >= e_) bad("unexpected end");
    Json v;
    char c = *p_;
    if (c == '{') {
      v.type = Json::OBJ;
      ++p_;
      ws();
      if (p_ < e_ && *p_ == '}') {
        ++p_;
        return v;
      }
      while (true) {
        ws();
        if (p_ >= e_ || *p_ != '"') bad("expected key");
        std::string k = str();
        ws();
        if (p_ >= e_ || *p_ != ':') bad("expected ':'");
        ++p_;
        v.obj.emplace_back(std::move(k), value(depth + 1));
        ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == '}') {
          ++p_;
          break;
        }
        bad("expected ',' or '}'");
      }
    } else if (c == '[') {
      v.type = Json::ARR;
      ++p_;
      ws();
      if (p_ < e_ && *p_ == ']') {
        ++p_;
        return v;
      }
      while (true) {
        v.arr.push_back(value(depth + 1));
        ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == ']') {
          ++p_;
          break;
        }
        bad("expected ',' or ']'");
      }
    } else if (c == '"') {
      v.type = Json::STR;
      v.s = str();
    } else if (lit("true")) {
      v.type = Json::BOOL;
      v.b = true;
    } else if (lit("false")) {
      v.type = Json::BOOL;
    } else if (lit("null")) {
      v.type = Json::NUL;
    } else {
      const char* st = p_;
      if (*p_ == '-') ++p_;
      bool digits = false, frac = false;
      while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' ||
                         *p_ == '+' || *p_ == '-')) {
        if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') frac = true;
        if (*p_ >= '0' && *p_ <= '9') digits = true;
        ++p_;
      }
      if (!digits) bad("bad value");
      std::string t(st, p_);
      v.type = Json::NUM;
      v.d = strtod(t.c_str(), nullptr);
      if (!frac) {
        v.is_int = true;
        v.neg = t[0] == '-';
        uint64_t m = 0;
        for (size_t i = v.neg ? 1 : 0; i < t.size(); ++i) {
          uint64_t nm = m * 10 + (t[i] - '0');
          if (nm / 10 != m) bad("integer overflow");
          m = nm;
        }
        v.u = m;
      }
    }
    return v;
  }
};

}  // namespace cg
