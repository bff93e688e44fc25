// regex.cc — the ECMAScript front end (Envoy's std::regex), the shared
// assertion-aware subset construction (regex_impl.h) and the DFA utilities.
// See regex.h for the semantics contract; regex_go.cc is the Go front end.
#include "regex.h"

#include <algorithm>
#include <deque>
#include <map>
#include <tuple>
#include <unordered_map>

#include "regex_impl.h"

namespace cg {

namespace {

struct VecHash {
  size_t operator()(const std::vector<int>& v) const {
    uint64_t h = 0x9e3779b97f4a7c15ULL ^ v.size();
    for (int x : v) h = mix64(h ^ (uint64_t)(uint32_t)x);
    return (size_t)h;
  }
};

constexpr int kMaxRepeat = 1000;

// ------------------------------------------------ ECMAScript byte classes --
// libstdc++ regex_traits<char> in the "C" locale: ctype<char>::is on the
// byte as unsigned char (bytes >= 0x80 belong to no class).
enum CType : uint16_t {
  kUpper = 1, kLower = 2, kAlpha = 4, kDigit = 8, kXdigit = 16, kSpace = 32, kPrint = 64, kGraph = 128,
  kCntrl = 256, kPunct = 512, kAlnum = 1024, kBlank = 2048, kUnder = 4096,
};
bool c_is(int b, uint16_t mask) {
  if (b >= 0x80) return false;
  const bool upper = b >= 'A' && b <= 'Z', lower = b >= 'a' && b <= 'z', digit = b >= '0' && b <= '9';
  const bool alpha = upper || lower, space = b == ' ' || (b >= '\t' && b <= '\r');
  const bool print = b >= 0x20 && b < 0x7f, graph = b > 0x20 && b < 0x7f;
  uint16_t m = 0;
  if (upper) m |= kUpper;
  if (lower) m |= kLower;
  if (alpha) m |= kAlpha;
  if (digit) m |= kDigit;
  if (digit || (b >= 'a' && b <= 'f') || (b >= 'A' && b <= 'F')) m |= kXdigit;
  if (space) m |= kSpace;
  if (print) m |= kPrint;
  if (graph) m |= kGraph;
  if (b < 0x20 || b == 0x7f) m |= kCntrl;
  if (graph && !alpha && !digit) m |= kPunct;
  if (alpha || digit) m |= kAlnum;
  if (b == ' ' || b == '\t') m |= kBlank;
  return (m & mask) || ((mask & kUnder) && b == '_');
}
ByteSet ctype_set(uint16_t mask) {
  ByteSet s;
  for (int b = 0; b < 256; ++b)
    if (c_is(b, mask)) s.set(b);
  return s;
}
ByteSet set_digit() { return ctype_set(kDigit); }
ByteSet set_word() { return ctype_set(kAlnum | kUnder); }
ByteSet set_space() { return ctype_set(kSpace); }  // [\t\n\v\f\r ]
ByteSet set_dot() {
  // libstdc++ _AnyMatcher<ecma>: any char except '\n' and '\r'
  ByteSet s = ByteSet::all();
  s.w['\n' >> 6] &= ~(1ULL << ('\n' & 63));
  s.w['\r' >> 6] &= ~(1ULL << ('\r' & 63));
  return s;
}

// regex_traits::lookup_classname (case-insensitive name)
bool class_by_name(std::string n, uint16_t* mask) {
  for (auto& c : n)
    if (c >= 'A' && c <= 'Z') c = c - 'A' + 'a';
  static const std::pair<const char*, uint16_t> kNames[] = {
      {"d", kDigit},      {"w", kAlnum | kUnder}, {"s", kSpace},   {"alnum", kAlnum}, {"alpha", kAlpha},
      {"blank", kBlank},  {"cntrl", kCntrl},      {"digit", kDigit}, {"graph", kGraph}, {"lower", kLower},
      {"print", kPrint},  {"punct", kPunct},      {"space", kSpace}, {"upper", kUpper}, {"xdigit", kXdigit}};
  for (auto& e : kNames)
    if (n == e.first) {
      *mask = e.second;
      return true;
    }
  return false;
}

// regex_traits::lookup_collatename: the POSIX names of the 128 ASCII
// characters (exact spelling; the index is the character)
int collate_by_name(const std::string& n) {
  static const char* const kNames[128] = {
      "NUL", "SOH", "STX", "ETX", "EOT", "ENQ", "ACK", "alert", "backspace", "tab", "newline", "vertical-tab",
      "form-feed", "carriage-return", "SO", "SI", "DLE", "DC1", "DC2", "DC3", "DC4", "NAK", "SYN", "ETB", "CAN",
      "EM", "SUB", "ESC", "IS4", "IS3", "IS2", "IS1", "space", "exclamation-mark", "quotation-mark", "number-sign",
      "dollar-sign", "percent-sign", "ampersand", "apostrophe", "left-parenthesis", "right-parenthesis",
      "asterisk", "plus-sign", "comma", "hyphen", "period", "slash", "zero", "one", "two", "three", "four", "five",
      "six", "seven", "eight", "nine", "colon", "semicolon", "less-than-sign", "equals-sign", "greater-than-sign",
      "question-mark", "commercial-at", "A", "B", "C", "D", "E", "F", "G", "H", "I", "J", "K", "L", "M", "N", "O",
      "P", "Q", "R", "S", "T", "U", "V", "W", "X", "Y", "Z", "left-square-bracket", "backslash",
      "right-square-bracket", "circumflex", "underscore", "grave-accent", "a", "b", "c", "d", "e", "f", "g", "h",
      "i", "j", "k", "l", "m", "n", "o", "p", "q", "r", "s", "t", "u", "v", "w", "x", "y", "z",
      "left-curly-bracket", "vertical-line", "right-curly-bracket", "tilde", "DEL"};
  for (int i = 0; i < 128; ++i)
    if (n == kNames[i]) return i;
  return -1;
}

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

rx::SymSet to_sym(const ByteSet& b) {
  rx::SymSet s(256);
  for (int i = 0; i < 4; ++i) s.w[i] = b.w[i];
  return s;
}

// ECMAScript grammar as libstdc++ (GCC 11, this image's std::regex — the
// oracle's engine) scans and compiles it (bits/regex_scanner.tcc,
// regex_compiler.tcc), lowered to a Prog over bytes.
class EcmaParser {
 public:
  EcmaParser(const std::string& re, rx::Prog& prog) : s_(re), g_(prog) {}

  int parse() {
    int r = parse_alt();
    if (p_ != s_.size()) err(CG_POLICY_REJECTED, "unmatched ')'");
    // std::regex accepts the pattern; a construct in it is beyond a DFA
    if (!unsupported_.empty()) fail(CG_UNSUPPORTED, "regex \"" + s_ + "\": " + unsupported_);
    return r;
  }

 private:
  const std::string& s_;
  rx::Prog& g_;
  size_t p_ = 0;
  int depth_ = 0;
  // capture groups: started so far (libstdc++ _M_subexpr_count - 1) and
  // still open (_M_paren_stack), for the validity of a backreference
  int ncap_ = 0;
  std::vector<int> open_caps_;
  std::string unsupported_;  // first construct a DFA cannot express

  [[noreturn]] void err(int code, const std::string& m) {
    fail(code, "regex \"" + s_ + "\": " + m + " at offset " + std::to_string(p_));
  }
  bool eof() const { return p_ >= s_.size(); }
  char peek() const { return s_[p_]; }

  int mkset(const ByteSet& s) { return g_.add_set(to_sym(s)); }
  int mkassert(uint8_t as) {
    rx::Node n;
    n.kind = rx::Node::ASSERT;
    n.as = as;
    return g_.add(n);
  }

  int parse_alt() {
    if (++depth_ > 200) err(CG_UNSUPPORTED, "nesting too deep");
    std::vector<int> alts{parse_cat()};
    while (!eof() && peek() == '|') {
      ++p_;
      alts.push_back(parse_cat());
    }
    --depth_;
    if (alts.size() == 1) return alts[0];
    rx::Node a;
    a.kind = rx::Node::ALT;
    a.kids = alts;
    return g_.add(a);
  }

  int parse_cat() {
    std::vector<int> items;
    while (!eof() && peek() != '|' && peek() != ')') items.push_back(parse_quant());
    if (items.empty()) return g_.add(rx::Node{});
    if (items.size() == 1) return items[0];
    rx::Node a;
    a.kind = rx::Node::CAT;
    a.kids = items;
    return g_.add(a);
  }

  bool parse_int(int* v) {
    size_t st = p_;
    long x = 0;
    while (!eof() && peek() >= '0' && peek() <= '9') {
      x = x * 10 + (peek() - '0');
      if (x > 100000000) err(CG_UNSUPPORTED, "repeat count too large");
      ++p_;
    }
    *v = (int)x;
    return p_ > st;
  }

  int parse_quant() {
    bool assertion = false;
    int atom = parse_atom(&assertion);
    while (!eof()) {
      char c = peek();
      int mn, mx;
      if (c == '*') {
        mn = 0, mx = -1, ++p_;
      } else if (c == '+') {
        mn = 1, mx = -1, ++p_;
      } else if (c == '?') {
        mn = 0, mx = 1, ++p_;
      } else if (c == '{') {
        ++p_;
        if (!parse_int(&mn)) err(CG_POLICY_REJECTED, "bad brace");
        mx = mn;
        if (!eof() && peek() == ',') {
          ++p_;
          if (!parse_int(&mx)) mx = -1;
        }
        if (eof() || peek() != '}') err(CG_POLICY_REJECTED, "bad brace");
        ++p_;
        if (mx >= 0 && mx < mn) err(CG_POLICY_REJECTED, "bad brace range");
        if (mn > kMaxRepeat || mx > kMaxRepeat) err(CG_UNSUPPORTED, "repeat count > 1000");
      } else {
        break;
      }
      // A quantifier must follow an atom, not an assertion (libstdc++
      // error_badrepeat).  libstdc++ accepts stacked quantifiers ("a**",
      // "a?+") as nested repeats; a trailing '?' only marks one lazy.
      if (assertion) err(CG_POLICY_REJECTED, "nothing to repeat");
      if (!eof() && peek() == '?') ++p_;
      rx::Node a;
      a.kind = rx::Node::REP;
      a.kids = {atom};
      a.min = mn;
      a.max = mx;
      atom = g_.add(a);
    }
    return atom;
  }

  // Class escape \d\D\w\W\s\S (the scanner's quoted_class token).
  bool class_escape(char c, ByteSet* out) {
    switch (c) {
      case 'd': *out = set_digit(); return true;
      case 'w': *out = set_word(); return true;
      case 's': *out = set_space(); return true;
      case 'D': *out = set_digit(); out->invert(); return true;
      case 'W': *out = set_word(); out->invert(); return true;
      case 'S': *out = set_space(); out->invert(); return true;
      default: return false;
    }
  }

  // _M_eat_escape_ecma for an escape that yields one character (p_ at the
  // char after '\'); class escapes and \b \B are handled by the callers.
  int char_escape(bool in_class) {
    if (eof()) err(CG_POLICY_REJECTED, "trailing backslash");
    char c = s_[p_++];
    switch (c) {
      case '0': return 0;  // NUL; following digits are ordinary
      case 'b': return '\b';  // in a bracket only (callers)
      case 'f': return '\f';
      case 'n': return '\n';
      case 'r': return '\r';
      case 't': return '\t';
      case 'v': return '\v';
      case 'x':
      case 'u': {
        const int nd = c == 'x' ? 2 : 4;
        int v = 0;
        for (int i = 0; i < nd; ++i) {
          if (eof() || hexval(peek()) < 0) err(CG_POLICY_REJECTED, "bad \\x / \\u escape");
          v = v * 16 + hexval(s_[p_++]);
        }
        return v & 0xFF;  // assigned to a char: Ł reads as 0x41
      }
      case 'c':
        // libstdc++ reads "\cX" as the character X itself, for any X
        if (eof()) err(CG_POLICY_REJECTED, "bad \\c escape");
        return (unsigned char)s_[p_++];
      default:
        if (c >= '1' && c <= '9') {
          // a backreference token (all following digits): "Unexpected
          // character" inside a bracket; outside one valid iff the group
          // exists and is closed (_M_insert_backref) — then std::regex
          // supports it and a DFA does not
          if (in_class) err(CG_POLICY_REJECTED, "backreference in bracket");
          long idx = c - '0';
          while (!eof() && peek() >= '0' && peek() <= '9') {
            idx = idx * 10 + (s_[p_++] - '0');
            if (idx > 0x7fffffff) err(CG_POLICY_REJECTED, "invalid back reference");
          }
          if (idx > ncap_) err(CG_POLICY_REJECTED, "back-reference index exceeds group count");
          for (int o : open_caps_)
            if (o == idx) err(CG_POLICY_REJECTED, "back-reference to an open group");
          if (unsupported_.empty()) unsupported_ = "backreference";
          return -1;
        }
        return (unsigned char)c;  // identity escape
    }
  }

  // _M_eat_class: the name up to the first `ch`, then "ch]"
  std::string eat_class_name(char ch) {
    size_t e = s_.find(ch, p_);
    if (e == std::string::npos || e + 1 >= s_.size() || s_[e + 1] != ']')
      err(CG_POLICY_REJECTED, "unterminated [: [. or [= in bracket");
    std::string n = s_.substr(p_, e - p_);
    p_ = e + 2;
    return n;
  }

  // A bracket expression as _M_expression_term walks it: a cached last
  // character (the possible start of a range), or a class just added.
  int parse_class() {
    bool neg = false;
    if (!eof() && peek() == '^') {
      neg = true;
      ++p_;
    }
    ByteSet set;
    enum { NONE, CHAR, CLASS } last = NONE;
    int last_c = 0;
    auto push_char = [&](int ch) {
      if (last == CHAR) set.set(last_c);
      last = CHAR;
      last_c = ch;
    };
    auto push_class = [&]() {
      if (last == CHAR) set.set(last_c);
      last = CLASS;
    };
    // One scanner token; kinds: 'c' char (ord/hex), 'q' quoted class,
    // '.' collating symbol, ':' class name, '=' equivalence class, '-'
    // dash, ']' end.
    struct Tok {
      char kind;
      int ch;
      ByteSet set;
    };
    auto next_tok = [&]() -> Tok {
      if (eof()) err(CG_POLICY_REJECTED, "unterminated [");
      const char c = s_[p_++];
      Tok t{'c', (unsigned char)c, ByteSet{}};
      if (c == '-') {
        t.kind = '-';
      } else if (c == ']') {
        t.kind = ']';
      } else if (c == '[') {
        if (eof()) err(CG_POLICY_REJECTED, "unexpected '[' at end of bracket");
        const char k = peek();
        if (k == '.' || k == ':' || k == '=') {
          ++p_;
          const std::string n = eat_class_name(k);
          t.kind = k;
          if (k == ':') {
            uint16_t mask;
            if (!class_by_name(n, &mask)) err(CG_POLICY_REJECTED, "invalid character class [:" + n + ":]");
            t.set = ctype_set(mask);
          } else {
            const int e = collate_by_name(n);
            if (e < 0) err(CG_POLICY_REJECTED, "invalid collating element");
            if (k == '.') {
              t.ch = e;
            } else {
              // transform_primary: equal after tolower
              auto low = [](int b) { return b >= 'A' && b <= 'Z' ? b + 32 : b; };
              for (int b = 0; b < 256; ++b)
                if (low(b) == low(e)) t.set.set(b);
            }
          }
        }
      } else if (c == '\\') {
        if (!eof() && class_escape(peek(), &t.set)) {
          ++p_;
          t.kind = 'q';
        } else {
          t.ch = char_escape(true);
        }
      }
      return t;
    };
    for (;;) {
      Tok t = next_tok();
      if (t.kind == ']') break;
      if (t.kind == '.' || t.kind == 'c') {
        push_char(t.ch);
      } else if (t.kind == ':' || t.kind == '=' || t.kind == 'q') {
        push_class();
        set.merge(t.set);
      } else {  // '-'
        if (!eof() && peek() == ']') {
          ++p_;
          push_char('-');
          break;
        }
        if (last == CLASS) err(CG_POLICY_REJECTED, "invalid start of range");
        if (last == CHAR) {
          Tok e = next_tok();
          int hi;
          if (e.kind == 'c') hi = e.ch;
          else if (e.kind == '-') hi = '-';
          else err(CG_POLICY_REJECTED, "invalid end of range");
          // libstdc++ compares the range ends as (signed) char
          const int slo = (int8_t)last_c, shi = (int8_t)hi;
          if (slo > shi) err(CG_POLICY_REJECTED, "invalid range");
          for (int v = slo; v <= shi; ++v) set.set((uint8_t)(int8_t)v);
          last = NONE;
        } else {
          push_char('-');  // ECMAScript: a dash outside a range is a char
        }
      }
    }
    if (last == CHAR) set.set(last_c);
    if (neg) set.invert();
    return mkset(set);
  }

  int parse_atom(bool* assertion) {
    char c = s_[p_++];
    switch (c) {
      case '(': {
        int cap = 0;
        if (!eof() && peek() == '?') {
          if (p_ + 1 < s_.size() && s_[p_ + 1] == ':') {
            p_ += 2;
          } else if (p_ + 1 < s_.size() && (s_[p_ + 1] == '=' || s_[p_ + 1] == '!')) {
            p_ += 2;
            *assertion = true;  // libstdc++ _M_assertion: no quantifier may follow
            if (unsupported_.empty()) unsupported_ = "lookahead";
          } else {
            err(CG_POLICY_REJECTED, "bad group");
          }
        } else {
          cap = ++ncap_;
          open_caps_.push_back(cap);
        }
        int r = parse_alt();
        if (eof() || peek() != ')') err(CG_POLICY_REJECTED, "missing ')'");
        ++p_;
        if (cap) open_caps_.pop_back();
        return r;
      }
      case ')': err(CG_POLICY_REJECTED, "unmatched ')'");
      case '[': return parse_class();
      case '.': return mkset(set_dot());
      case '^': *assertion = true; return mkassert(rx::kBeginText);
      case '$': *assertion = true; return mkassert(rx::kEndText);
      case '*':
      case '+':
      case '?':
      case '{': --p_; err(CG_POLICY_REJECTED, "nothing to repeat");
      case '\\': {
        if (!eof() && (peek() == 'b' || peek() == 'B')) {
          *assertion = true;
          return mkassert(s_[p_++] == 'b' ? rx::kWordB : rx::kNotWordB);
        }
        ByteSet esc;
        if (!eof() && class_escape(peek(), &esc)) {
          ++p_;
          return mkset(esc);
        }
        const int ch = char_escape(false);
        if (ch < 0) return g_.add(rx::Node{});  // backreference (unsupported_ is set)
        ByteSet s;
        s.set(ch);
        return mkset(s);
      }
      default: {
        ByteSet s;
        s.set((unsigned char)c);
        return mkset(s);
      }
    }
  }
};

void ecma_compile(const std::string& re, rx::Prog* g) {
  g->nsym = 256;
  g->root = EcmaParser(re, *g).parse();
  g->word.assign(256, 0);
  g->newline.assign(256, 0);
  const ByteSet w = set_word();
  for (int b = 0; b < 256; ++b) g->word[b] = w.test(b);
  g->newline['\n'] = 1;
}

// ---------------------------------------------------------------- NFA ----
struct NState {
  enum Type : uint8_t { SET, EPS, SPLIT, ASSERT, MATCH };
  Type type = EPS;
  uint8_t as = 0;
  int out = -1, out1 = -1;
  int set = -1;
};

constexpr int kMaxNfa = 200000;

class NfaBuilder {
 public:
  explicit NfaBuilder(const rx::Prog& g) : g_(g) {}
  std::vector<NState> st;

  int add(NState::Type t) {
    if ((int)st.size() >= kMaxNfa) fail(CG_UNSUPPORTED, "regex too large after repeat expansion");
    NState s;
    s.type = t;
    st.push_back(s);
    return (int)st.size() - 1;
  }
  struct Frag {
    int in, out;  // out: EPS state whose out is unset
  };
  Frag eps() {
    int e = add(NState::EPS);
    return {e, e};
  }
  Frag cat(Frag a, Frag b) {
    st[a.out].out = b.in;
    return {a.in, b.out};
  }
  Frag build(int id) {
    const rx::Node& n = g_.nodes[id];
    switch (n.kind) {
      case rx::Node::EMPTY: return eps();
      case rx::Node::SET: {
        int s = add(NState::SET);
        st[s].set = n.set;
        int e = add(NState::EPS);
        st[s].out = e;
        return {s, e};
      }
      case rx::Node::ASSERT: {
        int s = add(NState::ASSERT);
        st[s].as = n.as;
        int e = add(NState::EPS);
        st[s].out = e;
        return {s, e};
      }
      case rx::Node::CAT: {
        Frag f = build(n.kids[0]);
        for (size_t i = 1; i < n.kids.size(); ++i) f = cat(f, build(n.kids[i]));
        return f;
      }
      case rx::Node::ALT: {
        int e = add(NState::EPS);
        int entry = -1, prev_split = -1;
        for (size_t i = 0; i < n.kids.size(); ++i) {
          Frag f = build(n.kids[i]);
          st[f.out].out = e;
          if (i + 1 < n.kids.size()) {
            int sp = add(NState::SPLIT);
            st[sp].out = f.in;
            if (prev_split < 0) entry = sp;
            else st[prev_split].out1 = sp;
            prev_split = sp;
          } else {
            if (prev_split < 0) entry = f.in;
            else st[prev_split].out1 = f.in;
          }
        }
        return {entry, e};
      }
      case rx::Node::REP: {
        Frag f = eps();
        for (int i = 0; i < n.min; ++i) f = cat(f, build(n.kids[0]));
        if (n.max < 0) {
          Frag body = build(n.kids[0]);
          int sp = add(NState::SPLIT);
          int e = add(NState::EPS);
          st[sp].out = body.in;
          st[sp].out1 = e;
          st[body.out].out = sp;
          f = cat(f, Frag{sp, e});
        } else {
          for (int i = n.min; i < n.max; ++i) {
            Frag body = build(n.kids[0]);
            int sp = add(NState::SPLIT);
            int e = add(NState::EPS);
            st[sp].out = body.in;
            st[sp].out1 = e;
            st[body.out].out = e;
            f = cat(f, Frag{sp, e});
          }
        }
        return f;
      }
    }
    return eps();
  }

 private:
  const rx::Prog& g_;
};

// ------------------------------------------------- subset construction ---
// DFA state = (kept NFA states, kind of the previous symbol, decoder state).
// Kept: SET and MATCH states, and lookahead assertions (End*, word
// boundaries) waiting for the next symbol.  Begin* assertions are settled
// when reached, from the previous symbol's kind.
enum PrevKind : int { kStart = 0, kNl = 1, kWord = 2, kOther = 3 };

class Subset {
 public:
  Subset(const std::vector<NState>& st, const rx::Prog& g, const rx::Decoder& dec, const ByteSet& alpha)
      : st_(st), g_(g), dec_(dec), alpha_(alpha), mark_(st.size(), 0) {
    for (const auto& s : st_) {
      if (s.type != NState::ASSERT) continue;
      if (s.as == rx::kBeginText || s.as == rx::kBeginLine) need_begin_ = true;
      if (s.as == rx::kBeginLine) need_nl_ = true;
      if (s.as == rx::kWordB || s.as == rx::kNotWordB) need_word_ = true;
    }
  }

  ByteDfa run(int start, int max_states) {
    // symbols that every SET and the assertions treat alike share a class
    std::vector<int> symcls(g_.nsym);
    {
      std::map<std::vector<uint8_t>, int> sig2id;
      std::vector<int> sets_used;
      for (const auto& s : st_)
        if (s.type == NState::SET) sets_used.push_back(s.set);
      std::sort(sets_used.begin(), sets_used.end());
      sets_used.erase(std::unique(sets_used.begin(), sets_used.end()), sets_used.end());
      for (int y = 0; y < g_.nsym; ++y) {
        std::vector<uint8_t> sig;
        sig.reserve(sets_used.size() + 2);
        for (int k : sets_used) sig.push_back(g_.sets[k].test(y));
        sig.push_back(g_.word[y]);
        sig.push_back(g_.newline[y]);
        symcls[y] = sig2id.emplace(sig, (int)sig2id.size()).first->second;
      }
    }
    // byte classes: equal alphabet membership and, from every decoder
    // state, equal next state and equal emitted symbol classes
    std::vector<int> bcls(256);
    std::vector<int> rep;
    {
      std::map<std::vector<int>, int> sig2id;
      for (int b = 0; b < 256; ++b) {
        std::vector<int> sig{alpha_.test(b)};
        for (int q = 0; q < dec_.nstates; ++q) {
          const size_t k = (size_t)q * 256 + b;
          sig.push_back(dec_.next[k]);
          sig.push_back(dec_.nemit[k]);
          for (int e = 0; e < dec_.nemit[k]; ++e) sig.push_back(symcls[dec_.emit[k * 4 + e]]);
        }
        auto it = sig2id.emplace(sig, (int)sig2id.size());
        bcls[b] = it.first->second;
        if (it.second) rep.push_back(b);
      }
    }

    std::unordered_map<std::vector<int>, int, VecHash> ids;
    std::vector<std::vector<int>> keys;
    ByteDfa d;
    d.trans.assign(256, 0);
    d.accept.push_back(0);
    keys.push_back({});

    auto intern = [&](std::vector<int> kept, int pk, int q) -> int {
      if (kept.empty()) return 0;
      kept.push_back(-1 - canon(pk));
      kept.push_back(-16 - q);
      auto it = ids.find(kept);
      if (it != ids.end()) return it->second;
      if ((int)keys.size() >= max_states) fail(CG_UNSUPPORTED, "regex DFA exceeds state budget");
      const int id = (int)keys.size();
      ids.emplace(kept, id);
      keys.push_back(std::move(kept));
      d.trans.resize((size_t)(id + 1) * 256, 0);
      d.accept.push_back(0);
      return id;
    };

    std::vector<int> s0 = closure({start}, kStart, false, -1);
    const int first = intern(s0, kStart, 0);
    if (first == 0) {  // no string can match
      d.accept.push_back(0);
      d.trans.resize(2 * 256, 0);
      d.start = 1;
      return d;
    }
    std::deque<int> work{first};
    std::vector<bool> done(2, false);
    while (!work.empty()) {
      const int ds = work.front();
      work.pop_front();
      if ((int)done.size() <= ds) done.resize(ds + 1, false);
      if (done[ds]) continue;
      done[ds] = true;
      std::vector<int> key = keys[ds];
      const int q = -16 - key.back();
      key.pop_back();
      const int pk = -1 - key.back();
      key.pop_back();
      // acceptance: the decoder's pending bytes flush as symbols, then the
      // end of input settles the pending assertions
      {
        std::vector<int> k = key;
        int p = pk;
        for (int i = 0; i < dec_.pending[q] && !k.empty(); ++i) {
          k = step(k, p, dec_.flush);
          p = kind(dec_.flush);
        }
        if (!k.empty()) {
          std::vector<int> r = closure(k, p, true, -1);
          for (int x : r)
            if (st_[x].type == NState::MATCH) d.accept[ds] = 1;
        }
      }
      for (size_t c = 0; c < rep.size(); ++c) {
        const int b = rep[c];
        int target = 0;
        if (alpha_.test(b)) {
          const size_t kk = (size_t)q * 256 + b;
          std::vector<int> k = key;
          int p = pk;
          for (int e = 0; e < dec_.nemit[kk] && !k.empty(); ++e) {
            const int y = dec_.emit[kk * 4 + e];
            k = step(k, p, y);
            p = kind(y);
          }
          target = intern(k, p, dec_.next[kk]);
          if (target && ((int)done.size() <= target || !done[target])) work.push_back(target);
        }
        for (int bb = 0; bb < 256; ++bb)
          if (bcls[bb] == (int)c) d.trans[(size_t)ds * 256 + bb] = target;
      }
    }
    d.start = first;
    return d;
  }

 private:
  const std::vector<NState>& st_;
  const rx::Prog& g_;
  const rx::Decoder& dec_;
  ByteSet alpha_;
  std::vector<uint32_t> mark_;
  uint32_t gen_ = 0;
  bool need_begin_ = false, need_nl_ = false, need_word_ = false;

  int kind(int y) const { return g_.newline[y] ? kNl : g_.word[y] ? kWord : kOther; }
  int canon(int pk) const {
    if (pk == kStart && !need_begin_) return kOther;
    if (pk == kNl && !need_nl_) return kOther;
    if (pk == kWord && !need_word_) return kOther;
    return pk;
  }
  // next: a symbol, or -1 = end of input (when `known`)
  bool holds(uint8_t as, int pk, int next) const {
    const bool pw = pk == kWord, nw = next >= 0 && g_.word[next];
    switch (as) {
      case rx::kBeginText: return pk == kStart;
      case rx::kBeginLine: return pk == kStart || pk == kNl;
      case rx::kEndText: return next < 0;
      case rx::kEndLine: return next < 0 || g_.newline[next];
      case rx::kWordB: return pw != nw;
      case rx::kNotWordB: return pw == nw;
    }
    return false;
  }

  // epsilon closure at a position whose previous symbol has kind pk; with
  // `known`, the next symbol (or the end) settles every assertion
  std::vector<int> closure(const std::vector<int>& seeds, int pk, bool known, int next) {
    ++gen_;
    std::vector<int> stack(seeds.rbegin(), seeds.rend());
    std::vector<int> kept;
    while (!stack.empty()) {
      const int s = stack.back();
      stack.pop_back();
      if (s < 0 || mark_[s] == gen_) continue;
      mark_[s] = gen_;
      const NState& n = st_[s];
      switch (n.type) {
        case NState::SET:
        case NState::MATCH: kept.push_back(s); break;
        case NState::EPS: stack.push_back(n.out); break;
        case NState::SPLIT:
          stack.push_back(n.out1);
          stack.push_back(n.out);
          break;
        case NState::ASSERT: {
          const bool look = n.as != rx::kBeginText && n.as != rx::kBeginLine;
          if (look && !known) kept.push_back(s);
          else if (holds(n.as, pk, next)) stack.push_back(n.out);
          break;
        }
      }
    }
    std::sort(kept.begin(), kept.end());
    return kept;
  }

  // consume symbol y from the kept set k (previous kind pk)
  std::vector<int> step(const std::vector<int>& k, int pk, int y) {
    std::vector<int> r = closure(k, pk, true, y);
    std::vector<int> moved;
    for (int x : r)
      if (st_[x].type == NState::SET && g_.sets[st_[x].set].test(y)) moved.push_back(st_[x].out);
    if (moved.empty()) return {};
    return closure(moved, kind(y), false, -1);
  }
};

}  // namespace

namespace rx {

Decoder identity_decoder() {
  Decoder d;
  d.nstates = 1;
  d.next.assign(256, 0);
  d.nemit.assign(256, 1);
  d.emit.assign(256 * 4, 0);
  for (int b = 0; b < 256; ++b) d.emit[(size_t)b * 4] = (uint16_t)b;
  d.pending.assign(1, 0);
  return d;
}

ByteDfa build_dfa(Prog g, const Decoder& dec, const ByteSet& alphabet, bool search, int max_states) {
  // one extra symbol set: every symbol (search's surrounding loops)
  SymSet all(g.nsym);
  for (int y = 0; y < g.nsym; ++y) all.set(y);
  g.sets.push_back(all);
  const int all_id = (int)g.sets.size() - 1;
  NfaBuilder b(g);
  NfaBuilder::Frag f = b.build(g.root);
  const int match = b.add(NState::MATCH);
  int start = f.in;
  if (search) {
    // (any symbol)* re (any symbol)* — a begin assertion inside re still
    // holds only at offset 0 (the previous kind is kStart only there)
    int pre = b.add(NState::SPLIT);
    int pre_set = b.add(NState::SET);
    b.st[pre_set].set = all_id;
    b.st[pre_set].out = pre;
    b.st[pre].out = pre_set;
    b.st[pre].out1 = f.in;
    int post = b.add(NState::SPLIT);
    int post_set = b.add(NState::SET);
    b.st[post_set].set = all_id;
    b.st[post_set].out = post;
    b.st[post].out = post_set;
    b.st[post].out1 = match;
    b.st[f.out].out = post;
    start = pre;
  } else {
    b.st[f.out].out = match;
  }
  Subset sub(b.st, g, dec, alphabet);
  return dfa_minimize(sub.run(start, max_states));
}

}  // namespace rx

bool regex_syntax_ok(const std::string& re, std::string* errmsg, RegexFlavour flavour) {
  try {
    if (flavour == RegexFlavour::Go) {
      rx::go_syntax_check(re);
    } else {
      rx::Prog g;
      EcmaParser(re, g).parse();
    }
    return true;
  } catch (const Error& e) {
    if (errmsg) *errmsg = e.msg;
    return false;
  }
}

ByteDfa compile_regex(const std::string& re, const ByteSet& alphabet, MatchMode mode, int max_states) {
  rx::Prog g;
  rx::Decoder dec;
  if (mode == MatchMode::Search) {
    rx::go_compile(re, &g, &dec);
  } else {
    ecma_compile(re, &g);
    dec = rx::identity_decoder();
  }
  return rx::build_dfa(g, dec, alphabet, mode == MatchMode::Search, max_states);
}

ByteDfa dfa_literal(const std::string& s, const ByteSet& alphabet) {
  ByteDfa d;
  int n = (int)s.size();
  d.accept.assign(n + 2, 0);
  d.trans.assign((size_t)(n + 2) * 256, 0);
  bool ok = true;
  for (int i = 0; i < n; ++i) {
    uint8_t b = (uint8_t)s[i];
    if (!alphabet.test(b)) ok = false;
    d.trans[(size_t)(i + 1) * 256 + b] = i + 2;
  }
  d.accept[n + 1] = ok ? 1 : 0;
  d.start = 1;
  return dfa_minimize(d);
}

ByteDfa dfa_star(const ByteSet& alphabet) {
  ByteDfa d;
  d.accept = {0, 1};
  d.trans.assign(2 * 256, 0);
  for (int b = 0; b < 256; ++b)
    if (alphabet.test(b)) d.trans[256 + b] = 1;
  d.start = 1;
  return d;
}

ByteDfa dfa_prefix(const std::string& s, const ByteSet& alphabet) {
  ByteDfa d;
  const int n = (int)s.size();
  d.accept.assign(n + 2, 0);
  d.trans.assign((size_t)(n + 2) * 256, 0);
  bool ok = true;
  for (int i = 0; i < n; ++i) {
    const uint8_t b = (uint8_t)s[i];
    if (!alphabet.test(b)) ok = false;
    d.trans[(size_t)(i + 1) * 256 + b] = i + 2;
  }
  if (ok) {
    d.accept[n + 1] = 1;
    for (int b = 0; b < 256; ++b)
      if (alphabet.test(b)) d.trans[(size_t)(n + 1) * 256 + b] = n + 1;
  }
  d.start = 1;
  return dfa_minimize(d);
}

ByteDfa dfa_suffix(const std::string& s, const ByteSet& alphabet) {
  const int n = (int)s.size();
  for (unsigned char c : s)
    if (!alphabet.test(c)) {  // no string over the alphabet ends with s
      ByteDfa d;
      d.accept.assign(2, 0);
      d.trans.assign(2 * 256, 0);
      return d;
    }
  // KMP failure function; automaton state q (0..n) = longest prefix of s
  // that is a suffix of the input, as ByteDfa state q + 1 (0 stays dead)
  std::vector<int> fail_(n + 1, 0);
  for (int i = 1, k = 0; i < n; ++i) {
    while (k && s[i] != s[k]) k = fail_[k];
    if (s[i] == s[k]) ++k;
    fail_[i + 1] = k;
  }
  ByteDfa d;
  d.accept.assign(n + 2, 0);
  d.trans.assign((size_t)(n + 2) * 256, 0);
  d.accept[n + 1] = 1;
  for (int q = 0; q <= n; ++q)
    for (int b = 0; b < 256; ++b) {
      if (!alphabet.test(b)) continue;
      int k = q;
      if (k == n) k = fail_[n];
      while (k && (uint8_t)s[k] != b) k = fail_[k];
      if (k < n && (uint8_t)s[k] == b) ++k;
      d.trans[(size_t)(q + 1) * 256 + b] = k + 1;
    }
  d.start = 1;
  return dfa_minimize(d);
}

ByteDfa dfa_complement(const ByteDfa& d, const ByteSet& alphabet) {
  // live states keep their rows with acceptance flipped; moves into the dead
  // state go to an accepting sink T instead (bytes outside the alphabet
  // still die: those strings are not field values)
  const int n = d.size(), T = n;
  ByteDfa o;
  o.accept.assign(n + 1, 0);
  o.trans.assign((size_t)(n + 1) * 256, 0);
  for (int s = 1; s < n; ++s) {
    o.accept[s] = !d.accept[s];
    for (int b = 0; b < 256; ++b) {
      if (!alphabet.test(b)) continue;
      const int t = d.next(s, b);
      o.trans[(size_t)s * 256 + b] = t ? t : T;
    }
  }
  o.accept[T] = 1;
  for (int b = 0; b < 256; ++b)
    if (alphabet.test(b)) o.trans[(size_t)T * 256 + b] = T;
  o.start = d.start;
  return dfa_minimize(o);
}

namespace {

// A DFA under construction: rows of 256 targets (0 = dead).
struct DfaBuild {
  ByteDfa d;
  DfaBuild() {
    d.accept.assign(1, 0);
    d.trans.assign(256, 0);
  }
  int add(bool acc) {
    d.accept.push_back(acc);
    d.trans.resize(d.trans.size() + 256, 0);
    return d.size() - 1;
  }
  void set(int s, int b, int t) { d.trans[(size_t)s * 256 + b] = t; }
};

// Magnitude automaton: any number of leading '0's, then the significant
// digits of m, accepting m in [lo, hi] (the all-zeros string is m = 0, needs
// at least one digit).  States after k significant digits of prefix p are
// (k, p vs lo's first k digits, p vs hi's first k digits) — the comparison
// decides for numbers of lo's / hi's length, any other length in between is
// in range.  Returns the entry state.
int build_magnitude(DfaBuild& B, uint64_t lo, uint64_t hi) {
  const bool zero_ok = lo == 0;
  const uint64_t plo = lo == 0 ? 1 : lo;
  const std::string L = std::to_string(plo), H = std::to_string(hi);
  const bool any_pos = hi >= plo;
  const int entry = B.add(false);
  const int zeros = B.add(zero_ok);
  for (int b = '0'; b <= '0'; ++b) {
    B.set(entry, b, zeros);
    B.set(zeros, b, zeros);
  }
  if (!any_pos) return entry;
  std::map<std::tuple<int, int, int>, int> ids;
  std::vector<std::tuple<int, int, int>> work;
  auto state = [&](int k, int cl, int ch) -> int {
    // numbers longer than hi never come back into range
    if (k > (int)H.size()) return 0;
    auto key = std::make_tuple(k, cl, ch);
    auto it = ids.find(key);
    if (it != ids.end()) return it->second;
    const bool ge = k > (int)L.size() || (k == (int)L.size() && cl >= 0);
    const bool le = k < (int)H.size() || (k == (int)H.size() && ch <= 0);
    const int id = B.add(ge && le);
    ids.emplace(key, id);
    work.push_back(key);
    return id;
  };
  auto cmp = [](int a, int b) { return a < b ? -1 : a > b ? 1 : 0; };
  for (int dgt = 1; dgt <= 9; ++dgt) {
    const int t = state(1, cmp('0' + dgt, L[0]), cmp('0' + dgt, H[0]));
    B.set(entry, '0' + dgt, t);
    B.set(zeros, '0' + dgt, t);
  }
  while (!work.empty()) {
    auto [k, cl, ch] = work.back();
    work.pop_back();
    const int s = ids[std::make_tuple(k, cl, ch)];
    for (int dgt = 0; dgt <= 9; ++dgt) {
      const int c = '0' + dgt;
      const int ncl = cl != 0 || k >= (int)L.size() ? cl : cmp(c, L[k]);
      const int nch = ch != 0 || k >= (int)H.size() ? ch : cmp(c, H[k]);
      B.set(s, c, state(k + 1, ncl, nch));
    }
  }
  return entry;
}

}  // namespace

ByteDfa dfa_int_range(int64_t start, int64_t end, const ByteSet& alphabet) {
  DfaBuild B;
  const int st = B.add(false);  // start: leading isspace bytes loop here
  if (start < end) {
    const int64_t last = end - 1;  // inclusive
    const bool has_pos = last >= 0, has_neg = start < 0;
    int pos = 0, neg = 0;
    if (has_pos) pos = build_magnitude(B, start < 0 ? 0 : (uint64_t)start, (uint64_t)last);
    if (has_neg) {
      // |x| for the negative part; "-0..." reads as 0, in range iff 0 is
      // (when the range also holds non-negatives, last >= 0 and |x| >= 1)
      const uint64_t mlo = last < 0 ? (uint64_t)(-(last + 1)) + 1 : 1;
      const uint64_t mhi = (uint64_t)(-(start + 1)) + 1;
      neg = build_magnitude(B, has_pos ? 0 : mlo, mhi);
    } else if (start == 0) {
      neg = build_magnitude(B, 0, 0);  // only "-0..." (= 0) reads in range
    }
    for (int b : {' ', '\t', '\n', '\v', '\f', '\r'}) B.set(st, b, st);
    if (has_pos) {
      B.set(st, '+', pos);
      for (int b = '0'; b <= '9'; ++b) B.set(st, b, B.d.next(pos, b));
    }
    if (neg) B.set(st, '-', neg);
  }
  B.d.start = st;
  ByteDfa d = B.d;
  for (int s = 0; s < d.size(); ++s)
    for (int b = 0; b < 256; ++b)
      if (!alphabet.test(b)) d.trans[(size_t)s * 256 + b] = 0;
  return dfa_minimize(d);
}

ByteDfa dfa_list(const ByteDfa& item) {
  // item states keep their rows; an accepting state's move on kEscByte goes
  // to a fresh state Y(s) that continues the item on kEscBase..+3 (as the
  // old escape state did) and ends it on kEscSep, back to a fresh start S'
  // that copies the item's start row and is the only accepting state
  const int n = item.size();
  std::vector<int> acc;
  for (int s = 1; s < n; ++s)
    if (item.accept[s]) acc.push_back(s);
  const int sp = n + (int)acc.size();
  ByteDfa o;
  o.accept.assign((size_t)sp + 1, 0);
  o.trans.assign((size_t)(sp + 1) * 256, 0);
  for (int s = 1; s < n; ++s)
    for (int b = 0; b < 256; ++b) o.trans[(size_t)s * 256 + b] = item.next(s, b);
  for (size_t k = 0; k < acc.size(); ++k) {
    const int s = acc[k], y = n + (int)k;
    const int e = item.next(s, kEscByte);
    if (e)
      for (int b = kEscBase; b < kEscBase + 4; ++b) o.trans[(size_t)y * 256 + b] = item.next(e, b);
    o.trans[(size_t)y * 256 + kEscSep] = sp;
    o.trans[(size_t)s * 256 + kEscByte] = y;
  }
  for (int b = 0; b < 256; ++b) o.trans[(size_t)sp * 256 + b] = o.trans[(size_t)item.start * 256 + b];
  o.accept[sp] = 1;
  o.start = sp;
  return dfa_minimize(o);
}

ByteDfa dfa_escape_low(const ByteDfa& d) {
  // state s keeps its transitions on bytes >= 4; bytes 0..3 move to an escape
  // state e(s) reached on kEscByte, whose transitions on kEscBase + b are
  // s's old transitions on b.  The escaped encoding is injective and prefix
  // free, so the language maps one to one.
  const int n = d.size();
  ByteDfa o;
  o.start = d.start;
  o.accept = d.accept;
  o.accept.resize((size_t)2 * n, 0);
  o.trans.assign((size_t)2 * n * 256, 0);
  for (int s = 1; s < n; ++s) {
    for (int b = 4; b < 256; ++b) o.trans[(size_t)s * 256 + b] = d.next(s, b);
    bool any = false;
    for (int b = 0; b < 4; ++b) {
      o.trans[(size_t)(n + s) * 256 + kEscBase + b] = d.next(s, b);
      any |= d.next(s, b) != 0;
    }
    if (any) o.trans[(size_t)s * 256 + kEscByte] = n + s;
  }
  return dfa_minimize(o);
}

ByteDfa dfa_intersect(const ByteDfa& a, const ByteDfa& b) {
  std::unordered_map<uint64_t, int> ids;
  std::vector<std::pair<int, int>> pairs{{0, 0}};
  ByteDfa d;
  d.accept = {0};
  d.trans.assign(256, 0);
  auto get = [&](int x, int y) -> int {
    if (x == 0 || y == 0) return 0;
    uint64_t k = ((uint64_t)(uint32_t)x << 32) | (uint32_t)y;
    auto it = ids.find(k);
    if (it != ids.end()) return it->second;
    int id = (int)pairs.size();
    if (id > (1 << 20)) fail(CG_UNSUPPORTED, "matcher intersection too large");
    ids.emplace(k, id);
    pairs.push_back({x, y});
    d.accept.push_back(a.accept[x] && b.accept[y]);
    d.trans.resize((size_t)(id + 1) * 256, 0);
    return id;
  };
  int s = get(a.start, b.start);
  for (size_t i = 1; i < pairs.size(); ++i) {
    auto [x, y] = pairs[i];
    for (int c = 0; c < 256; ++c) {
      int t = get(a.next(x, c), b.next(y, c));
      d.trans[i * 256 + c] = t;
    }
  }
  d.start = s;
  if (s == 0) {
    d.accept.push_back(0);
    d.trans.resize(2 * 256, 0);
    d.start = 1;
  }
  return dfa_minimize(d);
}

ByteDfa dfa_minimize(const ByteDfa& d) {
  int n = d.size();
  // byte classes of the input table
  std::vector<int> bcls(256);
  std::vector<int> rep;
  {
    std::unordered_map<std::vector<int>, int, VecHash> col2id;
    std::vector<int> col(n);
    for (int b = 0; b < 256; ++b) {
      for (int s = 0; s < n; ++s) col[s] = d.trans[(size_t)s * 256 + b];
      auto it = col2id.emplace(col, (int)col2id.size());
      bcls[b] = it.first->second;
      if (it.second) rep.push_back(b);
    }
  }
  int k = (int)rep.size();
  // Moore refinement
  std::vector<int> blk(n);
  for (int s = 0; s < n; ++s) blk[s] = d.accept[s] ? 1 : 0;
  int nblk = 0;
  for (;;) {
    std::unordered_map<std::vector<int>, int, VecHash> sig2id;
    std::vector<int> nb(n);
    std::vector<int> sig(k + 1);
    for (int s = 0; s < n; ++s) {
      sig[0] = blk[s];
      for (int c = 0; c < k; ++c) sig[c + 1] = blk[d.trans[(size_t)s * 256 + rep[c]]];
      auto it = sig2id.emplace(sig, (int)sig2id.size());
      nb[s] = it.first->second;
    }
    int cnt = (int)sig2id.size();
    blk.swap(nb);
    if (cnt == nblk) break;
    nblk = cnt;
  }
  // canonical BFS numbering: dead block → 0, start block → 1
  std::vector<int> newid(nblk, -1);
  std::vector<int> order;  // block representatives (a state) in new-id order
  int dead_blk = blk[0];
  newid[dead_blk] = 0;
  order.push_back(0);
  std::vector<int> rep_state(nblk, -1);
  for (int s = 0; s < n; ++s)
    if (rep_state[blk[s]] < 0) rep_state[blk[s]] = s;
  ByteDfa out;
  if (blk[d.start] == dead_blk) {
    out.accept = {0, 0};
    out.trans.assign(2 * 256, 0);
    out.start = 1;
    return out;
  }
  std::deque<int> q;
  newid[blk[d.start]] = 1;
  order.push_back(rep_state[blk[d.start]]);
  q.push_back(blk[d.start]);
  while (!q.empty()) {
    int bb = q.front();
    q.pop_front();
    int s = rep_state[bb];
    for (int b = 0; b < 256; ++b) {
      int t = blk[d.trans[(size_t)s * 256 + b]];
      if (newid[t] < 0) {
        newid[t] = (int)order.size();
        order.push_back(rep_state[t]);
        q.push_back(t);
      }
    }
  }
  int m = (int)order.size();
  out.accept.assign(m, 0);
  out.trans.assign((size_t)m * 256, 0);
  for (int i = 1; i < m; ++i) {
    int s = order[i];
    out.accept[i] = d.accept[s];
    for (int b = 0; b < 256; ++b) out.trans[(size_t)i * 256 + b] = newid[blk[d.trans[(size_t)s * 256 + b]]];
  }
  out.start = 1;
  return out;
}

bool dfa_run(const ByteDfa& d, const std::string& s) {
  int st = d.start;
  for (unsigned char c : s) {
    st = d.next(st, c);
    if (st == 0) return false;
  }
  return d.accept[st];
}

}  // namespace cg
