// regex.h — regex → minimized byte DFA compiler (host side).
//
// Two flavours, each with the semantics of the engine the reference runs:
//
// * Full match (MatchMode::Full): Envoy's HeaderUtility::matchHeaders with
//   `regex_match`, i.e. a std::regex (ECMAScript grammar, libstdc++, char =
//   signed byte, "C" locale) applied with std::regex_match — a FULL-string
//   match (envoy/cilium_network_policy.h:68-71, Envoy pinned at f936fc60 in
//   envoy/WORKSPACE:10-16).  Supported: literals, escapes (\d\D\w\W\s\S
//   \f\n\r\t\v \0 \xHH \uHHHH (low byte, as assigned to a char) \cX,
//   identity escapes), '.', bracket expressions with ranges, negation,
//   [:class:], [.collating-element.] and [=equivalence-class=], groups
//   (...) (?:...), alternation, quantifiers * + ? {n} {n,} {n,m} (greedy or
//   lazy: the same language), anchors ^ $ and word boundaries \b \B.
//   Rejected with CG_UNSUPPORTED (std::regex accepts them, a DFA cannot
//   express them): backreferences and lookahead.
//
// * Search (MatchMode::Search): Go 1.10 regexp.MatchString, as proxylib's
//   parsers call it (proxylib/r2d2/r2d2parser.go:80,103,
//   cassandra/cassandraparser.go:89,113, memcached/parser.go:91,132) —
//   RE2 syntax with the Perl flags (regexp/syntax), matched over UTF-8
//   runes where each invalid byte is one U+FFFD rune (regex_go.cc).
//   Every Go-valid pattern compiles, within the NFA/DFA size budgets.
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

// Parse-only check: Ecma = std::regex's grammar (what Envoy compiles), Go =
// regexp.Compile's (PortRuleHTTP.Sanitize, pkg/policy/api/http.go:66-84).
enum class RegexFlavour { Ecma, Go };
bool regex_syntax_ok(const std::string& re, std::string* err, RegexFlavour flavour = RegexFlavour::Ecma);

}  // namespace cg
