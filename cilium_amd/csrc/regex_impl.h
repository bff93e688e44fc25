// regex_impl.h — shared back end of the two regex front ends (regex.cc:
// ECMAScript / std::regex for Envoy's regex_match; regex_go.cc: Go regexp
// for proxylib's MatchString).  Internal to the host compiler.
//
// Both front ends lower a pattern to a Prog: an AST over *symbols* — bytes
// for ECMAScript (std::regex<char> reads bytes), rune classes for Go (Go
// reads UTF-8 runes, an invalid byte being one U+FFFD rune).  A Decoder turns
// the input bytes into symbols: the identity for bytes, a UTF-8 decoder that
// follows utf8.DecodeRune for runes.  build_dfa() runs subset construction
// over (NFA state set, previous-symbol kind, decoder state) and returns a
// minimized byte DFA, so the GPU walks bytes either way.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "regex.h"

namespace cg {
namespace rx {

struct SymSet {
  std::vector<uint64_t> w;
  SymSet() = default;
  explicit SymSet(int nsym) : w((size_t)(nsym + 63) / 64, 0) {}
  void set(int s) { w[(size_t)s >> 6] |= 1ULL << (s & 63); }
  bool test(int s) const { return (w[(size_t)s >> 6] >> (s & 63)) & 1; }
  bool operator==(const SymSet& o) const { return w == o.w; }
};

// Empty-width assertions.  Begin* look at the previous symbol only and are
// settled when reached; End*/word boundaries also need the next symbol and
// stay pending in a DFA state until it (or the end of input) arrives.
enum Assert : uint8_t { kBeginText, kEndText, kBeginLine, kEndLine, kWordB, kNotWordB };

struct Node {
  enum Kind : uint8_t { EMPTY, SET, CAT, ALT, REP, ASSERT };
  Kind kind = EMPTY;
  uint8_t as = 0;
  int set = -1;  // SET: index into Prog::sets
  int min = 0, max = 0;  // REP; max < 0 = unbounded
  std::vector<int> kids;
};

struct Prog {
  int nsym = 256;
  std::vector<SymSet> sets;
  std::vector<Node> nodes;
  int root = -1;
  std::vector<uint8_t> word, newline;  // per symbol: is a word character / is '\n'

  int add(Node n) {
    nodes.push_back(std::move(n));
    return (int)nodes.size() - 1;
  }
  int add_set(const SymSet& s) {
    sets.push_back(s);
    Node n;
    n.kind = Node::SET;
    n.set = (int)sets.size() - 1;
    return add(n);
  }
};

// Deterministic byte → symbol-sequence machine.  State 0 is "between
// symbols"; a transition emits 0..4 symbols; at the end of input a state
// still holding `pending[q]` bytes emits that many `flush` symbols.
struct Decoder {
  int nstates = 1;
  std::vector<int32_t> next;    // [q * 256 + b]
  std::vector<uint8_t> nemit;   // [q * 256 + b]
  std::vector<uint16_t> emit;   // [(q * 256 + b) * 4 + k]
  std::vector<uint8_t> pending; // [q]
  int flush = 0;
};

Decoder identity_decoder();
// A minimized DFA over bytes: match-anywhere (search) or whole-string
// (full) semantics of p, bytes outside `alphabet` dead.
ByteDfa build_dfa(Prog p, const Decoder& dec, const ByteSet& alphabet, bool search, int max_states);

// Go front end (regex_go.cc): parse `re` as Go 1.10 regexp/syntax (Perl
// flags) and lower it to runes classes + the UTF-8 decoder.  Throws Error.
void go_compile(const std::string& re, Prog* prog, Decoder* dec);
void go_syntax_check(const std::string& re);

}  // namespace rx
}  // namespace cg
