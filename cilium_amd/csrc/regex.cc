// regex.cc — ECMAScript-subset parser, Thompson NFA, subset construction,
// minimization.  See regex.h for the semantics contract.
#include "regex.h"

#include <algorithm>
#include <deque>
#include <map>
#include <tuple>
#include <unordered_map>

namespace cg {

namespace {

// ---------------------------------------------------------------- AST ----
struct Ast {
  enum Kind { EMPTY, SET, CAT, ALT, REP, BOL, EOL };
  Kind kind = EMPTY;
  ByteSet set;
  std::vector<int> kids;
  int min = 0, max = 0;  // REP; max < 0 = unbounded
};

constexpr int kMaxRepeat = 1000;

ByteSet set_digit() {
  ByteSet s;
  s.set_range('0', '9');
  return s;
}
ByteSet set_word() {
  ByteSet s;
  s.set_range('0', '9');
  s.set_range('a', 'z');
  s.set_range('A', 'Z');
  s.set('_');
  return s;
}
// Two flavours share the parser: Envoy's std::regex (ECMAScript, full
// match) and Go's regexp (RE2 syntax, proxylib's MatchString search).  They
// differ, on bytes, in '.' and '\s'.
ByteSet set_space(bool go) {
  // libstdc++ ctype<char> "space" in the C locale; Go RE2 \s is [\t\n\f\r ]
  // (no \v: regexp/syntax perl_groups.go)
  ByteSet s;
  for (int c : {' ', '\t', '\n', '\f', '\r'}) s.set(c);
  if (!go) s.set('\v');
  return s;
}
ByteSet set_dot(bool go) {
  // libstdc++ _AnyMatcher<ecma>: any char except '\n' and '\r'; Go RE2
  // without the s flag: any char except '\n'
  ByteSet s = ByteSet::all();
  s.w['\n' >> 6] &= ~(1ULL << ('\n' & 63));
  if (!go) s.w['\r' >> 6] &= ~(1ULL << ('\r' & 63));
  return s;
}

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

class Parser {
 public:
  Parser(const std::string& re, std::vector<Ast>& nodes, bool go = false) : s_(re), n_(nodes), go_(go) {}

  int parse() {
    int r = parse_alt();
    if (p_ != s_.size()) err(CG_POLICY_REJECTED, "unmatched ')'");
    return r;
  }

 private:
  const std::string& s_;
  std::vector<Ast>& n_;
  bool go_ = false;  // Go RE2 flavour (search mode)
  size_t p_ = 0;
  int depth_ = 0;

  [[noreturn]] void err(int code, const std::string& m) {
    fail(code, "regex \"" + s_ + "\": " + m + " at offset " + std::to_string(p_));
  }
  bool eof() const { return p_ >= s_.size(); }
  char peek() const { return s_[p_]; }

  int mk(Ast a) {
    n_.push_back(std::move(a));
    return (int)n_.size() - 1;
  }
  int mkset(const ByteSet& s) {
    Ast a;
    a.kind = Ast::SET;
    a.set = s;
    return mk(a);
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
    Ast a;
    a.kind = Ast::ALT;
    a.kids = alts;
    return mk(a);
  }

  int parse_cat() {
    std::vector<int> items;
    while (!eof() && peek() != '|' && peek() != ')') items.push_back(parse_quant());
    if (items.empty()) return mk(Ast{});
    if (items.size() == 1) return items[0];
    Ast a;
    a.kind = Ast::CAT;
    a.kids = items;
    return mk(a);
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
    bool quantified = false;
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
      Ast a;
      a.kind = Ast::REP;
      a.kids = {atom};
      a.min = mn;
      a.max = mx;
      atom = mk(a);
      quantified = true;
    }
    return atom;
  }

  // Class escape inside or outside brackets; returns true and fills `out`
  // for \d\D\w\W\s\S, else false (p_ unchanged).
  bool class_escape(char c, ByteSet* out) {
    switch (c) {
      case 'd': *out = set_digit(); return true;
      case 'w': *out = set_word(); return true;
      case 's': *out = set_space(go_); return true;
      case 'D': *out = set_digit(); out->invert(); return true;
      case 'W': *out = set_word(); out->invert(); return true;
      case 'S': *out = set_space(go_); out->invert(); return true;
      default: return false;
    }
  }

  // Character escape after '\' (p_ at the char after '\').  Returns the byte.
  int char_escape(bool in_class) {
    if (eof()) err(CG_POLICY_REJECTED, "trailing backslash");
    char c = s_[p_++];
    switch (c) {
      case 'f': return '\f';
      case 'n': return '\n';
      case 'r': return '\r';
      case 't': return '\t';
      case 'v': return '\v';
      case 'b':
        if (in_class) return '\b';
        err(CG_UNSUPPORTED, "word boundary \\b");
      case 'B': err(CG_UNSUPPORTED, "word boundary \\B");
      case '0':
        if (!eof() && peek() >= '0' && peek() <= '9') err(CG_UNSUPPORTED, "octal escape");
        return 0;
      case 'x': {
        if (p_ + 2 > s_.size()) err(CG_POLICY_REJECTED, "bad \\x escape");
        int h = hexval(s_[p_]), l = hexval(s_[p_ + 1]);
        if (h < 0 || l < 0) err(CG_POLICY_REJECTED, "bad \\x escape");
        p_ += 2;
        return h * 16 + l;
      }
      case 'u': {
        if (p_ + 4 > s_.size()) err(CG_POLICY_REJECTED, "bad \\u escape");
        int v = 0;
        for (int i = 0; i < 4; ++i) {
          int d = hexval(s_[p_ + i]);
          if (d < 0) err(CG_POLICY_REJECTED, "bad \\u escape");
          v = v * 16 + d;
        }
        p_ += 4;
        if (v > 0xFF) err(CG_UNSUPPORTED, "\\u escape beyond one byte");
        return v;
      }
      case 'c': {
        if (eof() || !((peek() >= 'a' && peek() <= 'z') || (peek() >= 'A' && peek() <= 'Z')))
          err(CG_POLICY_REJECTED, "bad \\c escape");
        // libstdc++ (the engine Envoy ran) matches "\cX" as the letter X
        // itself, not the control character; measured against std::regex.
        return (unsigned char)s_[p_++];
      }
      default:
        if (c >= '1' && c <= '9') err(CG_UNSUPPORTED, "backreference");
        return (unsigned char)c;  // identity escape
    }
  }

  int parse_class() {
    // p_ just after '['
    bool neg = false;
    if (!eof() && peek() == '^') {
      neg = true;
      ++p_;
    }
    ByteSet set;
    for (;;) {
      if (eof()) err(CG_POLICY_REJECTED, "unterminated [");
      char c = peek();
      // ECMAScript (libstdc++ _M_scan_in_bracket): ']' always closes the
      // bracket, so "[]" matches nothing and "[^]" matches any byte.
      if (c == ']') {
        ++p_;
        break;
      }
      // one class atom
      int lo = -1;
      ByteSet esc;
      ++p_;
      if (c == '\\') {
        if (!eof() && class_escape(peek(), &esc)) {
          ++p_;
          set.merge(esc);
          if (!eof() && peek() == '-' && p_ + 1 < s_.size() && s_[p_ + 1] != ']')
            err(CG_POLICY_REJECTED, "class escape in range");
          continue;
        }
        lo = char_escape(true);
      } else if (c == '[' && !eof() && (peek() == ':' || peek() == '.' || peek() == '=')) {
        err(CG_UNSUPPORTED, "POSIX bracket expression");
      } else {
        lo = (unsigned char)c;
      }
      // range?
      if (!eof() && peek() == '-' && p_ + 1 < s_.size() && s_[p_ + 1] != ']') {
        ++p_;
        char d = s_[p_++];
        int hi;
        if (d == '\\') {
          if (!eof() && class_escape(peek(), &esc)) err(CG_POLICY_REJECTED, "class escape in range");
          hi = char_escape(true);
        } else {
          hi = (unsigned char)d;
        }
        // libstdc++ compares the range ends as (signed) char.
        int slo = (int8_t)lo, shi = (int8_t)hi;
        if (slo > shi) err(CG_POLICY_REJECTED, "invalid range");
        for (int v = slo; v <= shi; ++v) set.set((uint8_t)(int8_t)v);
      } else {
        set.set(lo);
      }
    }
    if (neg) set.invert();
    return mkset(set);
  }

  int parse_atom(bool* assertion) {
    char c = s_[p_++];
    switch (c) {
      case '(': {
        if (!eof() && peek() == '?') {
          if (p_ + 1 < s_.size() && s_[p_ + 1] == ':') {
            p_ += 2;
          } else if (p_ + 1 < s_.size() && (s_[p_ + 1] == '=' || s_[p_ + 1] == '!')) {
            err(CG_UNSUPPORTED, "lookahead");
          } else {
            err(CG_POLICY_REJECTED, "bad group");
          }
        }
        int r = parse_alt();
        if (eof() || peek() != ')') err(CG_POLICY_REJECTED, "missing ')'");
        ++p_;
        return r;
      }
      case ')': err(CG_POLICY_REJECTED, "unmatched ')'");
      case '[': return parse_class();
      case '.': return mkset(set_dot(go_));
      case '^': {
        *assertion = true;
        Ast a;
        a.kind = Ast::BOL;
        return mk(a);
      }
      case '$': {
        *assertion = true;
        Ast a;
        a.kind = Ast::EOL;
        return mk(a);
      }
      case '*':
      case '+':
      case '?':
      case '{': --p_; err(CG_POLICY_REJECTED, "nothing to repeat");
      case '\\': {
        ByteSet esc;
        if (!eof() && class_escape(peek(), &esc)) {
          ++p_;
          return mkset(esc);
        }
        ByteSet s;
        s.set(char_escape(false));
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

// ---------------------------------------------------------------- NFA ----
struct NState {
  enum Type : uint8_t { SET, EPS, SPLIT, BOL, EOL, MATCH };
  Type type = EPS;
  int out = -1, out1 = -1;
  ByteSet set;
};

constexpr int kMaxNfa = 200000;

class NfaBuilder {
 public:
  NfaBuilder(const std::vector<Ast>& ast) : a_(ast) {}
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
    const Ast& n = a_[id];
    switch (n.kind) {
      case Ast::EMPTY: return eps();
      case Ast::SET: {
        int s = add(NState::SET);
        st[s].set = n.set;
        int e = add(NState::EPS);
        st[s].out = e;
        return {s, e};
      }
      case Ast::BOL:
      case Ast::EOL: {
        int s = add(n.kind == Ast::BOL ? NState::BOL : NState::EOL);
        int e = add(NState::EPS);
        st[s].out = e;
        return {s, e};
      }
      case Ast::CAT: {
        Frag f = build(n.kids[0]);
        for (size_t i = 1; i < n.kids.size(); ++i) f = cat(f, build(n.kids[i]));
        return f;
      }
      case Ast::ALT: {
        int e = add(NState::EPS);
        int entry = -1;
        // chain of SPLITs
        int prev_split = -1;
        for (size_t i = 0; i < n.kids.size(); ++i) {
          Frag f = build(n.kids[i]);
          st[f.out].out = e;
          if (i + 1 < n.kids.size()) {
            int sp = add(NState::SPLIT);
            st[sp].out = f.in;
            if (prev_split < 0)
              entry = sp;
            else
              st[prev_split].out1 = sp;
            prev_split = sp;
          } else {
            if (prev_split < 0)
              entry = f.in;
            else
              st[prev_split].out1 = f.in;
          }
        }
        return {entry, e};
      }
      case Ast::REP: {
        Frag f = eps();
        for (int i = 0; i < n.min; ++i) f = cat(f, build(n.kids[0]));
        if (n.max < 0) {
          // star
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
  const std::vector<Ast>& a_;
};

struct VecHash {
  size_t operator()(const std::vector<int>& v) const {
    uint64_t h = 0x9e3779b97f4a7c15ULL ^ v.size();
    for (int x : v) h = mix64(h ^ (uint64_t)(uint32_t)x);
    return (size_t)h;
  }
};

class Subset {
 public:
  Subset(const std::vector<NState>& st, int start, const ByteSet& alpha)
      : st_(st), start_(start), alpha_(alpha), mark_(st.size(), 0) {}

  ByteDfa run(int max_states) {
    // byte classes: partition 0..255 by every SET state's set and the alphabet
    std::vector<ByteSet> sets;
    for (const auto& s : st_)
      if (s.type == NState::SET) sets.push_back(s.set);
    sets.push_back(alpha_);
    std::vector<int> cls(256, 0);
    {
      std::map<std::vector<bool>, int> sig2id;
      for (int b = 0; b < 256; ++b) {
        std::vector<bool> sig(sets.size());
        for (size_t i = 0; i < sets.size(); ++i) sig[i] = sets[i].test(b);
        auto it = sig2id.emplace(sig, (int)sig2id.size()).first;
        cls[b] = it->second;
      }
    }
    int ncls = 0;
    for (int b = 0; b < 256; ++b) ncls = std::max(ncls, cls[b] + 1);
    std::vector<int> rep(ncls, -1);
    for (int b = 0; b < 256; ++b)
      if (rep[cls[b]] < 0) rep[cls[b]] = b;

    // DFA states: key = (is_start flag folded in as -1 marker) + kept NFA states.
    std::unordered_map<std::vector<int>, int, VecHash> ids;
    std::vector<std::vector<int>> sets_of;
    std::vector<uint8_t> is_start;
    ByteDfa d;
    d.trans.assign(256, 0);  // dead
    d.accept.push_back(0);
    sets_of.push_back({});
    is_start.push_back(0);

    std::vector<int> s0 = closure({start_}, true);
    std::vector<int> key0 = s0;
    key0.insert(key0.begin(), -1);
    ids[key0] = 1;
    sets_of.push_back(s0);
    is_start.push_back(1);
    d.trans.resize(2 * 256, 0);
    d.accept.push_back(accepts(s0, true));

    std::deque<int> work{1};
    std::vector<int> moved;
    while (!work.empty()) {
      int ds = work.front();
      work.pop_front();
      std::vector<int> cur = sets_of[ds];
      for (int c = 0; c < ncls; ++c) {
        int b = rep[c];
        int target = 0;
        if (alpha_.test(b)) {
          moved.clear();
          for (int ns : cur)
            if (st_[ns].type == NState::SET && st_[ns].set.test(b)) moved.push_back(st_[ns].out);
          if (!moved.empty()) {
            std::vector<int> nx = closure(moved, false);
            if (!nx.empty()) {
              auto it = ids.find(nx);
              if (it == ids.end()) {
                if ((int)sets_of.size() >= max_states)
                  fail(CG_UNSUPPORTED, "regex DFA exceeds state budget");
                target = (int)sets_of.size();
                ids.emplace(nx, target);
                sets_of.push_back(nx);
                is_start.push_back(0);
                d.trans.resize((size_t)(target + 1) * 256, 0);
                d.accept.push_back(accepts(nx, false));
                work.push_back(target);
              } else {
                target = it->second;
              }
            }
          }
        }
        for (int bb = 0; bb < 256; ++bb)
          if (cls[bb] == c) d.trans[(size_t)ds * 256 + bb] = target;
      }
    }
    d.start = 1;
    return d;
  }

 private:
  const std::vector<NState>& st_;
  int start_;
  ByteSet alpha_;
  std::vector<uint32_t> mark_;
  uint32_t gen_ = 0;

  // epsilon closure; keeps SET, EOL and MATCH states (sorted, unique).
  std::vector<int> closure(const std::vector<int>& seeds, bool at_start) {
    ++gen_;
    std::vector<int> stack(seeds.begin(), seeds.end());
    std::vector<int> kept;
    while (!stack.empty()) {
      int s = stack.back();
      stack.pop_back();
      if (s < 0 || mark_[s] == gen_) continue;
      mark_[s] = gen_;
      const NState& n = st_[s];
      switch (n.type) {
        case NState::SET:
        case NState::MATCH:
        case NState::EOL: kept.push_back(s); break;
        case NState::EPS: stack.push_back(n.out); break;
        case NState::SPLIT:
          stack.push_back(n.out);
          stack.push_back(n.out1);
          break;
        case NState::BOL:
          if (at_start) stack.push_back(n.out);
          break;
      }
    }
    std::sort(kept.begin(), kept.end());
    return kept;
  }

  // Is MATCH reachable at end of input from this set?
  uint8_t accepts(const std::vector<int>& set, bool at_start) {
    ++gen_;
    std::vector<int> stack(set.begin(), set.end());
    while (!stack.empty()) {
      int s = stack.back();
      stack.pop_back();
      if (s < 0 || mark_[s] == gen_) continue;
      mark_[s] = gen_;
      const NState& n = st_[s];
      switch (n.type) {
        case NState::MATCH: return 1;
        case NState::SET: break;
        case NState::EOL:
        case NState::EPS: stack.push_back(n.out); break;
        case NState::SPLIT:
          stack.push_back(n.out);
          stack.push_back(n.out1);
          break;
        case NState::BOL:
          if (at_start) stack.push_back(n.out);
          break;
      }
    }
    return 0;
  }
};

}  // namespace

bool regex_syntax_ok(const std::string& re, std::string* errmsg) {
  try {
    std::vector<Ast> nodes;
    Parser(re, nodes).parse();
    return true;
  } catch (const Error& e) {
    if (errmsg) *errmsg = e.msg;
    return false;
  }
}

ByteDfa compile_regex(const std::string& re, const ByteSet& alphabet, MatchMode mode,
                      int max_states) {
  std::vector<Ast> nodes;
  int root = Parser(re, nodes, mode == MatchMode::Search).parse();
  NfaBuilder b(nodes);
  NfaBuilder::Frag f = b.build(root);
  int match = b.add(NState::MATCH);
  int start = f.in;
  if (mode == MatchMode::Search) {
    // (any byte)* re (any byte)*  — a '^' inside re still only matches at
    // offset 0 (closure follows BOL edges only in the start set).
    int pre = b.add(NState::SPLIT);
    int pre_set = b.add(NState::SET);
    b.st[pre_set].set = ByteSet::all();
    b.st[pre_set].out = pre;
    b.st[pre].out = pre_set;
    b.st[pre].out1 = f.in;
    int post = b.add(NState::SPLIT);
    int post_set = b.add(NState::SET);
    b.st[post_set].set = ByteSet::all();
    b.st[post_set].out = post;
    b.st[post].out = post_set;
    b.st[post].out1 = match;
    b.st[f.out].out = post;
    start = pre;
  } else {
    b.st[f.out].out = match;
  }
  Subset sub(b.st, start, alphabet);
  ByteDfa d = sub.run(max_states);
  return dfa_minimize(d);
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
