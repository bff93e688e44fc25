// regex.h — regex → minimized byte DFA compiler (host side).
//
// Semantics follow what the reference enforces for HTTP header matchers:
// Envoy's HeaderUtility::matchHeaders with `regex_match`, i.e. a std::regex
// (ECMAScript grammar, libstdc++, char = signed byte) applied with
// std::regex_match — a FULL-string match (envoy/cilium_network_policy.h:68-71,
// Envoy pinned at f936fc60 in envoy/WORKSPACE:10-16).  Go's regexp is only
// used by the agent to validate Path/Method (pkg/policy/api/http.go:66-84).
// An unanchored "search" mode serves proxylib parsers, which call Go
// regexp.MatchString (proxylib/r2d2/r2d2parser.go:80).
//
// Supported subset: literals, escapes (\d\D\w\W\s\S \f\n\r\t\v \0 \xHH
// \uHHHH≤0xFF \cX, identity escapes), '.', bracket classes with ranges and
// negation, groups (...) and (?:...), alternation, quantifiers * + ? {n}
// {n,} {n,m} (greedy or lazy — the same language), anchors ^ $.
// Rejected with CG_UNSUPPORTED: backreferences, lookaround, \b \B.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "common.h"

namespace cg {

struct ByteSet {
  uint64_t w[4] = {0, 0, 0, 0};
  void set(int b) { w[b >> 6] |= 1ULL << (b & 63); }
  bool test(int b) const { return (w[b >> 6] >> (b & 63)) & 1; }
  void set_range(int lo, int hi) {
    for (int b = lo; b <= hi; ++b) set(b);
  }
  void invert() {
    for (auto& x : w) x = ~x;
  }
  void merge(const ByteSet& o) {
    for (int i = 0; i < 4; ++i) w[i] |= o.w[i];
  }
  void intersect(const ByteSet& o) {
    for (int i = 0; i < 4; ++i) w[i] &= o.w[i];
  }
  bool empty() const { return !(w[0] | w[1] | w[2] | w[3]); }
  static ByteSet all() {
    ByteSet s;
    s.invert();
    return s;
  }
};

// Deterministic automaton over bytes.  State 0 is the dead state
// (non-accepting, every byte → 0).  trans has size()*256 entries.
struct ByteDfa {
  int start = 1;
  std::vector<int32_t> trans;
  std::vector<uint8_t> accept;
  int size() const { return (int)accept.size(); }
  int next(int s, int b) const { return trans[(size_t)s * 256 + b]; }
};

enum class MatchMode { Full, Search };

// Compile `re` to a minimized DFA accepting exactly the strings over
// `alphabet` (bytes outside it lead to the dead state) that the regex
// matches in `mode`.  Throws Error{CG_UNSUPPORTED | CG_POLICY_REJECTED}.
ByteDfa compile_regex(const std::string& re, const ByteSet& alphabet, MatchMode mode,
                      int max_states = 1 << 16);
// Strings equal to `s` (exact_match).
ByteDfa dfa_literal(const std::string& s, const ByteSet& alphabet);
// alphabet* (present_match on a field, or "no constraint").
ByteDfa dfa_star(const ByteSet& alphabet);
ByteDfa dfa_intersect(const ByteDfa& a, const ByteDfa& b);
// The same language over escaped strings: every byte b <= 3 of a string is
// written as the pair {kEscByte, kEscBase + b} (proxylib field values, whose
// bytes are arbitrary, while 0x00-0x02 structure the request string).
constexpr int kEscByte = 0x03, kEscBase = 0x10;
ByteDfa dfa_escape_low(const ByteDfa& d);
// Strings starting with `s` (then any bytes of the alphabet).
ByteDfa dfa_prefix(const std::string& s, const ByteSet& alphabet);
// Strings ending with `s` (KMP automaton over the alphabet).
ByteDfa dfa_suffix(const std::string& s, const ByteSet& alphabet);
// alphabet* minus L(d): Envoy's invert_match over the strings a field can hold.
ByteDfa dfa_complement(const ByteDfa& d, const ByteSet& alphabet);
// Strings that Envoy's StringUtil::atol (strtol base 10 over the whole value,
// ERANGE rejected) reads as an integer x with start <= x < end
// (HeaderMatcher.range_match, envoy.type.Int64Range).
ByteDfa dfa_int_range(int64_t start, int64_t end, const ByteSet& alphabet);
// A list of escaped items, each followed by the separator pair {kEscByte,
// kEscSep} (which no escaped string contains): (item SEP)*, every item in
// the language of the escaped DFA `item` (memcached key lists).
constexpr int kEscSep = 0x14;
ByteDfa dfa_list(const ByteDfa& item);
// Moore partition refinement + canonical BFS renumbering (dead=0, start=1):
// equal languages give identical tables.
ByteDfa dfa_minimize(const ByteDfa& d);
// Simulate (tests/diagnostics only).
bool dfa_run(const ByteDfa& d, const std::string& s);

// Parse-only check (used by PortRuleHTTP sanitize mirror).
bool regex_syntax_ok(const std::string& re, std::string* err);

}  // namespace cg
