// regex_go.cc — the Go regexp front end: Go 1.10 regexp/syntax with the
// Perl flags regexp.Compile uses (syntax.Perl = ClassNL | OneLine | PerlX |
// UnicodeGroups), matched as regexp.MatchString matches: over runes decoded
// by utf8.DecodeRune, where an invalid byte is one U+FFFD rune.
//
// Callers in the reference: proxylib/r2d2/r2d2parser.go:80,103,
// proxylib/cassandra/cassandraparser.go:89,113,
// proxylib/memcached/parser.go:91,132 (MustCompile + MatchString / Match);
// PortRuleHTTP.Sanitize validates with the same syntax
// (pkg/policy/api/http.go:66-84).
//
// Lowering: the pattern's rune sets partition the code points into classes
// (the symbols of a Prog); a byte → symbol decoder restates DecodeRune
// (a lead byte whose sequence fails is one U+FFFD and decoding restarts at
// the next byte), its pending states merged by what they can still emit.
// regex.cc's subset construction then yields a byte DFA.
#include <algorithm>
#include <map>

#include "go_unicode10.h"
#include "regex_impl.h"

namespace cg {
namespace rx {

namespace {

using RS = std::vector<std::pair<uint32_t, uint32_t>>;  // sorted, disjoint, inclusive
constexpr uint32_t kMaxRune = 0x10FFFF;
constexpr uint32_t kRuneError = 0xFFFD;

void rs_norm(RS& r) {
  std::sort(r.begin(), r.end());
  RS o;
  for (auto& x : r) {
    if (!o.empty() && x.first <= o.back().second + 1) o.back().second = std::max(o.back().second, x.second);
    else o.push_back(x);
  }
  r.swap(o);
}
bool rs_has(const RS& r, uint32_t c) {
  auto it = std::upper_bound(r.begin(), r.end(), std::make_pair(c, kMaxRune + 1));
  return it != r.begin() && (it - 1)->second >= c;
}
RS rs_neg(RS r) {
  rs_norm(r);
  RS o;
  uint32_t next = 0;
  for (auto& x : r) {
    if (x.first > next) o.push_back({next, x.first - 1});
    next = x.second + 1;
  }
  if (next <= kMaxRune) o.push_back({next, kMaxRune});
  return o;
}
void rs_add(RS& r, const RS& o) { r.insert(r.end(), o.begin(), o.end()); }

// simple case folding orbits (unicode.SimpleFold), Unicode 10.0
struct Orbits {
  std::vector<std::vector<uint32_t>> orbits;
  std::vector<std::pair<uint32_t, int>> member;  // sorted (rune, orbit)
  Orbits() {
    int k = 0;
    for (int o = 0; o < gou::kNumFoldOrbits; ++o) {
      const int n = (int)gou::kFoldOrbits[k++];
      std::vector<uint32_t> v(gou::kFoldOrbits + k, gou::kFoldOrbits + k + n);
      k += n;
      for (uint32_t c : v) member.push_back({c, (int)orbits.size()});
      orbits.push_back(std::move(v));
    }
    std::sort(member.begin(), member.end());
  }
  const std::vector<uint32_t>* of(uint32_t c) const {
    auto it = std::lower_bound(member.begin(), member.end(), std::make_pair(c, -1));
    if (it == member.end() || it->first != c) return nullptr;
    return &orbits[it->second];
  }
};
const Orbits& orbits() {
  static const Orbits o;
  return o;
}
// appendFoldedRange over a whole set: every orbit meeting the set joins it
RS rs_fold(RS r) {
  rs_norm(r);
  RS add;
  for (const auto& o : orbits().orbits) {
    bool hit = false;
    for (uint32_t c : o) hit = hit || rs_has(r, c);
    if (hit)
      for (uint32_t c : o) add.push_back({c, c});
  }
  rs_add(r, add);
  rs_norm(r);
  return r;
}

RS table_rs(const gou::Table& t) {
  RS r;
  for (int i = 0; i < t.n; ++i) r.push_back({t.r[i].lo, t.r[i].hi});
  return r;
}
// unicodeTable (regexp/syntax/parse.go): "Any", then unicode.Categories,
// then unicode.Scripts (case-sensitive names)
bool unicode_table(const std::string& name, RS* out) {
  if (name == "Any") {
    *out = {{0, kMaxRune}};
    return true;
  }
  for (const auto& t : gou::kCategories)
    if (name == t.name) {
      *out = table_rs(t);
      return true;
    }
  for (const auto& t : gou::kScripts)
    if (name == t.name) {
      *out = table_rs(t);
      return true;
    }
  return false;
}

RS ascii(std::initializer_list<std::pair<uint32_t, uint32_t>> l) { return RS(l); }
// perlGroup / posixGroup (regexp/syntax/perl_groups.go)
bool perl_group(uint32_t c, RS* cls, int* sign) {
  switch (c) {
    case 'd': *cls = ascii({{'0', '9'}}); *sign = 1; return true;
    case 'D': *cls = ascii({{'0', '9'}}); *sign = -1; return true;
    case 's': *cls = ascii({{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}}); *sign = 1; return true;
    case 'S': *cls = ascii({{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}}); *sign = -1; return true;
    case 'w': *cls = ascii({{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}); *sign = 1; return true;
    case 'W': *cls = ascii({{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}); *sign = -1; return true;
  }
  return false;
}
bool posix_group(const std::string& name, RS* cls) {
  static const std::map<std::string, RS> kG = {
      {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
      {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
      {"ascii", {{0, 0x7F}}},
      {"blank", {{'\t', '\t'}, {' ', ' '}}},
      {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
      {"digit", {{'0', '9'}}},
      {"graph", {{'!', '~'}}},
      {"lower", {{'a', 'z'}}},
      {"print", {{' ', '~'}}},
      {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
      {"space", {{'\t', '\r'}, {' ', ' '}}},
      {"upper", {{'A', 'Z'}}},
      {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
      {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}},
  };
  auto it = kG.find(name);
  if (it == kG.end()) return false;
  *cls = it->second;
  return true;
}

bool is_alnum(uint32_t c) { return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }
int unhex(uint32_t c) {
  if (c >= '0' && c <= '9') return (int)c - '0';
  if (c >= 'a' && c <= 'f') return (int)c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return (int)c - 'A' + 10;
  return -1;
}

// utf8.DecodeRune: (rune, width); an invalid sequence is (U+FFFD, 1)
std::pair<uint32_t, int> decode_rune(const uint8_t* p, size_t n) {
  const uint8_t b0 = p[0];
  if (b0 < 0x80) return {b0, 1};
  int need;
  uint8_t lo = 0x80, hi = 0xBF;
  if (b0 >= 0xC2 && b0 <= 0xDF) need = 2;
  else if (b0 >= 0xE0 && b0 <= 0xEF) need = 3;
  else if (b0 >= 0xF0 && b0 <= 0xF4) need = 4;
  else return {kRuneError, 1};
  if (b0 == 0xE0) lo = 0xA0;
  if (b0 == 0xED) hi = 0x9F;
  if (b0 == 0xF0) lo = 0x90;
  if (b0 == 0xF4) hi = 0x8F;
  if (n < (size_t)need) return {kRuneError, 1};
  if (p[1] < lo || p[1] > hi) return {kRuneError, 1};
  uint32_t r = b0 & (need == 2 ? 0x1F : need == 3 ? 0x0F : 0x07);
  r = (r << 6) | (p[1] & 0x3F);
  for (int i = 2; i < need; ++i) {
    if (p[i] < 0x80 || p[i] > 0xBF) return {kRuneError, 1};
    r = (r << 6) | (p[i] & 0x3F);
  }
  return {r, need};
}

struct GNode {
  enum Kind : uint8_t { EMPTY, SET, CAT, ALT, REP, ASSERT };
  Kind kind = EMPTY;
  uint8_t as = 0;
  RS set;
  std::vector<int> kids;
  int min = 0, max = 0;
};

struct Flags {
  bool fold = false, dotnl = false, oneline = true, nongreedy = false;
};

class GoParser {
 public:
  GoParser(const std::string& re, std::vector<GNode>& nodes) : src_(re), n_(nodes) {
    // regexp/syntax reads the pattern rune by rune and rejects invalid
    // UTF-8 wherever it meets it (nextRune, checkUTF8); every byte is read
    const uint8_t* p = (const uint8_t*)re.data();
    for (size_t i = 0; i < re.size();) {
      auto [r, w] = decode_rune(p + i, re.size() - i);
      if (r == kRuneError && w == 1) err("invalid UTF-8");
      r_.push_back(r);
      i += w;
    }
  }

  int parse() {
    Flags f;
    const int root = parse_alt(f);
    if (p_ < r_.size()) err("unexpected )");
    return root;
  }

 private:
  std::string src_;
  std::vector<uint32_t> r_;
  size_t p_ = 0;
  std::vector<GNode>& n_;
  int depth_ = 0;

  [[noreturn]] void err(const std::string& m) {
    fail(CG_POLICY_REJECTED, "Go regexp \"" + src_ + "\": " + m + " (rune " + std::to_string(p_) + ")");
  }
  bool eof() const { return p_ >= r_.size(); }
  uint32_t peek(size_t k = 0) const { return p_ + k < r_.size() ? r_[p_ + k] : 0xFFFFFFFF; }

  int mk(GNode n) {
    n_.push_back(std::move(n));
    return (int)n_.size() - 1;
  }
  int mkset(RS s) {
    rs_norm(s);
    GNode n;
    n.kind = GNode::SET;
    n.set = std::move(s);
    return mk(std::move(n));
  }
  int mkassert(uint8_t as) {
    GNode n;
    n.kind = GNode::ASSERT;
    n.as = as;
    return mk(std::move(n));
  }
  int literal(uint32_t c, const Flags& f) {
    RS s{{c, c}};
    if (f.fold)
      if (auto* o = orbits().of(c))
        for (uint32_t x : *o) s.push_back({x, x});
    return mkset(s);
  }

  int parse_alt(Flags& f) {
    if (++depth_ > 1000) fail(CG_UNSUPPORTED, "Go regexp nesting too deep");
    std::vector<int> alts{parse_cat(f)};
    while (!eof() && peek() == '|') {
      ++p_;
      alts.push_back(parse_cat(f));
    }
    --depth_;
    if (alts.size() == 1) return alts[0];
    GNode a;
    a.kind = GNode::ALT;
    a.kids = alts;
    return mk(std::move(a));
  }

  // parseInt: digits without a leading zero; > 1e8 reads as -1
  bool parse_int(size_t* q, int* v) {
    if (*q >= r_.size() || r_[*q] < '0' || r_[*q] > '9') return false;
    if (*q + 1 < r_.size() && r_[*q] == '0' && r_[*q + 1] >= '0' && r_[*q + 1] <= '9') return false;
    long n = 0;
    bool big = false;
    while (*q < r_.size() && r_[*q] >= '0' && r_[*q] <= '9') {
      if (!big) {
        if (n >= 100000000) big = true;
        else n = n * 10 + (r_[*q] - '0');
      }
      ++*q;
    }
    *v = big ? -1 : (int)n;
    return true;
  }
  // parseRepeat at '{': {n}, {n,}, {n,m}; false = not a repeat ('{' is a literal)
  bool parse_repeat(int* mn, int* mx) {
    size_t q = p_ + 1;
    if (!parse_int(&q, mn)) return false;
    if (q >= r_.size()) return false;
    if (r_[q] != ',') {
      *mx = *mn;
    } else {
      ++q;
      if (q >= r_.size()) return false;
      if (r_[q] == '}') {
        *mx = -1;
      } else {
        if (!parse_int(&q, mx)) return false;
        if (*mx < 0) *mn = -1;
      }
    }
    if (q >= r_.size() || r_[q] != '}') return false;
    p_ = q + 1;
    return true;
  }

  int parse_cat(Flags& f) {
    std::vector<int> items;
    bool last_repeat = false;
    while (!eof() && peek() != '|' && peek() != ')') {
      const uint32_t c = peek();
      int mn = 0, mx = 0;
      bool rep = false;
      if (c == '*' || c == '+' || c == '?') {
        ++p_;
        mn = c == '+' ? 1 : 0;
        mx = c == '?' ? 1 : -1;
        rep = true;
      } else if (c == '{') {
        if (parse_repeat(&mn, &mx)) {
          if (mn < 0 || mn > 1000 || mx > 1000 || (mx >= 0 && mn > mx)) err("invalid repeat count");
          rep = true;
        }
      }
      if (rep) {
        // a** and a*{2} are errors in Perl mode; a*? is one (lazy) repeat
        if (last_repeat) err("invalid nested repetition operator");
        if (items.empty()) err("missing argument to repetition operator");
        if (!eof() && peek() == '?') ++p_;
        GNode r;
        r.kind = GNode::REP;
        r.kids = {items.back()};
        r.min = mn;
        r.max = mx;
        items.back() = mk(std::move(r));
        last_repeat = true;
        continue;
      }
      last_repeat = false;
      if (c == '{') {  // not a repeat: a literal brace
        ++p_;
        items.push_back(literal('{', f));
        continue;
      }
      if (c == '(') {
        int g;
        if (group(f, &g)) items.push_back(g);
        continue;
      }
      parse_atom(f, items);
    }
    if (items.empty()) return mk(GNode{});
    if (items.size() == 1) return items[0];
    GNode a;
    a.kind = GNode::CAT;
    a.kids = items;
    return mk(std::move(a));
  }

  int group_body(Flags inner) {
    const int g = parse_alt(inner);
    if (eof() || peek() != ')') err("missing closing )");
    ++p_;
    return g;
  }

  // '(' at p_.  Returns false for a flags-only "(?flags)" (no atom).
  bool group(Flags& f, int* out) {
    if (peek(1) != '?') {
      ++p_;
      *out = group_body(f);
      return true;
    }
    // named capture (?P<name>re) (parsePerlFlags; byte length > 4)
    if (p_ + 4 < r_.size() && r_[p_ + 2] == 'P' && r_[p_ + 3] == '<') {
      size_t e = p_ + 4;
      while (e < r_.size() && r_[e] != '>') ++e;
      if (e >= r_.size()) err("invalid named capture");
      if (e == p_ + 4) err("invalid named capture");
      for (size_t k = p_ + 4; k < e; ++k)
        if (r_[k] != '_' && !is_alnum(r_[k])) err("invalid named capture");
      p_ = e + 1;
      *out = group_body(f);
      return true;
    }
    Flags nf = f;
    int sign = 1;
    bool saw = false;
    for (size_t i = p_ + 2; i < r_.size(); ++i) {
      const uint32_t c = r_[i];
      switch (c) {
        case 'i': nf.fold = sign > 0; saw = true; break;
        case 'm': nf.oneline = sign < 0; saw = true; break;
        case 's': nf.dotnl = sign > 0; saw = true; break;
        case 'U': nf.nongreedy = sign > 0; saw = true; break;
        case '-':
          if (sign < 0) err("invalid or unsupported Perl syntax");
          sign = -1;
          saw = false;
          break;
        case ':':
        case ')':
          if (sign < 0 && !saw) err("invalid or unsupported Perl syntax");
          p_ = i + 1;
          if (c == ':') {
            *out = group_body(nf);  // the enclosing flags come back at ')'
            return true;
          }
          f = nf;
          return false;
        default: err("invalid or unsupported Perl syntax");
      }
    }
    err("invalid or unsupported Perl syntax");
  }

  // parseEscape (p_ at '\\'): one rune
  uint32_t parse_escape() {
    ++p_;
    if (eof()) err("trailing backslash at end of expression");
    const uint32_t c = r_[p_++];
    switch (c) {
      case '1': case '2': case '3': case '4': case '5': case '6': case '7':
        if (eof() || peek() < '0' || peek() > '7') break;  // a backreference
        [[fallthrough]];
      case '0': {
        uint32_t r = c - '0';
        for (int i = 1; i < 3; ++i) {
          if (eof() || peek() < '0' || peek() > '7') break;
          r = r * 8 + (r_[p_++] - '0');
        }
        return r;
      }
      case 'x': {
        if (eof()) break;
        uint32_t d = r_[p_++];
        if (d == '{') {
          int nhex = 0;
          uint32_t r = 0;
          for (;;) {
            if (eof()) err("invalid escape sequence");
            d = r_[p_++];
            if (d == '}') break;
            const int v = unhex(d);
            if (v < 0) err("invalid escape sequence");
            r = r * 16 + v;
            if (r > kMaxRune) err("invalid escape sequence");
            ++nhex;
          }
          if (nhex == 0) err("invalid escape sequence");
          return r;
        }
        const int x = unhex(d);
        const int y = eof() ? -1 : unhex(r_[p_++]);
        if (x < 0 || y < 0) break;
        return (uint32_t)(x * 16 + y);
      }
      case 'a': return 7;
      case 'f': return '\f';
      case 'n': return '\n';
      case 'r': return '\r';
      case 't': return '\t';
      case 'v': return '\v';
      default:
        if (c < 0x80 && !is_alnum(c)) return c;  // escaped punctuation is itself
        break;
    }
    err("invalid escape sequence");
  }

  // \pN, \p{Name}, \PN, \p{^Name} (p_ at '\\'); false if not \p / \P
  bool unicode_class(const Flags& f, RS* out) {
    if (peek() != '\\' || (peek(1) != 'p' && peek(1) != 'P')) return false;
    int sign = peek(1) == 'P' ? -1 : 1;
    p_ += 2;
    std::string name;
    if (eof()) err("invalid character class range");
    if (peek() != '{') {
      const uint32_t c = r_[p_++];
      if (c < 0x80) name = std::string(1, (char)c);
      else name = "\x80";  // no table has a non-ASCII name
    } else {
      size_t e = p_;
      while (e < r_.size() && r_[e] != '}') ++e;
      if (e >= r_.size()) err("invalid character class range");
      for (size_t k = p_ + 1; k < e; ++k) name += r_[k] < 0x80 ? (char)r_[k] : '\x80';
      p_ = e + 1;
    }
    if (!name.empty() && name[0] == '^') {
      sign = -sign;
      name = name.substr(1);
    }
    RS tab;
    if (!unicode_table(name, &tab)) err("invalid character class range");
    if (f.fold && name != "Any") tab = rs_fold(tab);  // tab + FoldCategory / FoldScript
    *out = sign > 0 ? tab : rs_neg(tab);
    return true;
  }

  // a Perl or POSIX group as appendGroup adds it: folded, then negated
  RS group_set(RS cls, int sign, const Flags& f) {
    if (f.fold) cls = rs_fold(cls);
    return sign > 0 ? cls : rs_neg(cls);
  }

  // parseClass (p_ at '[')
  int parse_class(const Flags& f) {
    ++p_;
    int sign = 1;
    if (!eof() && peek() == '^') {
      sign = -1;
      ++p_;  // ClassNL is set: no '\n' special case
    }
    RS cls;
    bool first = true;
    for (;;) {
      if (eof()) err("missing closing ]");
      if (peek() == ']' && !first) break;
      first = false;
      // [:alnum:] — only if a ":]" follows, else '[' is a plain char
      if (peek() == '[' && peek(1) == ':') {
        size_t e = p_ + 2;
        while (e + 1 < r_.size() && !(r_[e] == ':' && r_[e + 1] == ']')) ++e;
        if (e + 1 < r_.size()) {
          std::string name;
          for (size_t k = p_ + 2; k < e; ++k) name += r_[k] < 0x80 ? (char)r_[k] : '\x80';
          int gs = 1;
          if (!name.empty() && name[0] == '^') {
            gs = -1;
            name = name.substr(1);
          }
          RS g;
          if (!posix_group(name, &g)) err("invalid character class range");
          rs_add(cls, group_set(g, gs, f));
          p_ = e + 2;
          continue;
        }
      }
      RS u;
      if (unicode_class(f, &u)) {
        rs_add(cls, u);
        continue;
      }
      if (peek() == '\\') {
        RS g;
        int gs;
        if (perl_group(peek(1), &g, &gs)) {
          p_ += 2;
          rs_add(cls, group_set(g, gs, f));
          continue;
        }
      }
      const uint32_t lo = class_char();
      uint32_t hi = lo;
      if (!eof() && peek() == '-' && peek(1) != ']' && p_ + 1 < r_.size()) {
        ++p_;
        hi = class_char();
        if (hi < lo) err("invalid character class range");
      }
      RS rg{{lo, hi}};
      rs_add(cls, f.fold ? rs_fold(rg) : rg);
    }
    ++p_;  // ']'
    return mkset(sign > 0 ? cls : rs_neg(cls));
  }
  uint32_t class_char() {
    if (eof()) err("missing closing ]");
    if (peek() == '\\') return parse_escape();
    return r_[p_++];
  }

  void parse_atom(const Flags& f, std::vector<int>& items) {
    const uint32_t c = peek();
    switch (c) {
      case '^': ++p_; items.push_back(mkassert(f.oneline ? kBeginText : kBeginLine)); return;
      case '$': ++p_; items.push_back(mkassert(f.oneline ? kEndText : kEndLine)); return;
      case '.': {
        ++p_;
        RS s{{0, kMaxRune}};
        if (!f.dotnl) s = {{0, '\n' - 1}, {'\n' + 1, kMaxRune}};
        items.push_back(mkset(s));
        return;
      }
      case '[': items.push_back(parse_class(f)); return;
      case '\\': {
        switch (peek(1)) {
          case 'A': p_ += 2; items.push_back(mkassert(kBeginText)); return;
          case 'b': p_ += 2; items.push_back(mkassert(kWordB)); return;
          case 'B': p_ += 2; items.push_back(mkassert(kNotWordB)); return;
          case 'C': err("invalid escape sequence \\C");
          case 'z': p_ += 2; items.push_back(mkassert(kEndText)); return;
          case 'Q': {
            // \Q...\E: literal text up to \E or the end
            p_ += 2;
            while (!eof()) {
              if (peek() == '\\' && peek(1) == 'E') {
                p_ += 2;
                break;
              }
              items.push_back(literal(r_[p_++], f));
            }
            return;
          }
        }
        RS u;
        if (unicode_class(f, &u)) {
          items.push_back(mkset(u));
          return;
        }
        RS g;
        int gs;
        if (perl_group(peek(1), &g, &gs)) {
          p_ += 2;
          items.push_back(mkset(group_set(g, gs, f)));
          return;
        }
        items.push_back(literal(parse_escape(), f));
        return;
      }
      case '*': case '+': case '?': err("missing argument to repetition operator");
      default: ++p_; items.push_back(literal(c, f)); return;
    }
  }
};

// --------------------------------------------------------- rune classes --
struct Partition {
  std::vector<uint32_t> lo;   // interval starts, ascending; lo[0] = 0
  std::vector<int> cls;       // class of each interval
  std::vector<uint32_t> rep;  // a code point of each class
  int of(uint32_t c) const {
    return cls[std::upper_bound(lo.begin(), lo.end(), c) - lo.begin() - 1];
  }
  // the class of every code point of [a, b], or -1
  int uniform(uint32_t a, uint32_t b) const {
    const size_t i = std::upper_bound(lo.begin(), lo.end(), a) - lo.begin() - 1;
    const uint32_t end = i + 1 < lo.size() ? lo[i + 1] - 1 : kMaxRune;
    return end >= b ? cls[i] : -1;
  }
};

Partition partition(const std::vector<const RS*>& sets) {
  std::vector<uint32_t> cut{0};
  for (const RS* s : sets)
    for (auto& x : *s) {
      cut.push_back(x.first);
      if (x.second < kMaxRune) cut.push_back(x.second + 1);
    }
  std::sort(cut.begin(), cut.end());
  cut.erase(std::unique(cut.begin(), cut.end()), cut.end());
  const size_t ni = cut.size(), words = (sets.size() + 63) / 64;
  std::vector<uint64_t> sig(ni * words, 0);
  for (size_t k = 0; k < sets.size(); ++k)
    for (auto& x : *sets[k]) {
      size_t i = std::lower_bound(cut.begin(), cut.end(), x.first) - cut.begin();
      for (; i < ni && cut[i] <= x.second; ++i) sig[i * words + k / 64] |= 1ULL << (k % 64);
    }
  Partition p;
  p.lo = cut;
  p.cls.resize(ni);
  std::map<std::vector<uint64_t>, int> ids;
  for (size_t i = 0; i < ni; ++i) {
    std::vector<uint64_t> s(sig.begin() + i * words, sig.begin() + (i + 1) * words);
    auto it = ids.emplace(s, (int)ids.size());
    p.cls[i] = it.first->second;
    if (it.second) p.rep.push_back(cut[i]);
  }
  return p;
}

// ---------------------------------------------------- the UTF-8 decoder --
// Pending states are merged bottom-up by a canonical signature of what
// their continuations emit (a constant vector is written compactly).
class DecoderBuilder {
 public:
  explicit DecoderBuilder(const Partition& pt) : pt_(pt) {}

  Decoder build() {
    const int fffd = pt_.of(kRuneError);
    // level-1 states per lead byte
    int l1[256];
    for (int b = 0xC2; b <= 0xDF; ++b) l1[b] = state2(b);
    for (int b = 0xE0; b <= 0xEF; ++b) l1[b] = lead3(b);
    for (int b = 0xF0; b <= 0xF4; ++b) l1[b] = lead4(b);
    Decoder d;
    d.nstates = (int)specs_.size() + 1;
    d.next.assign((size_t)d.nstates * 256, 0);
    d.nemit.assign((size_t)d.nstates * 256, 0);
    d.emit.assign((size_t)d.nstates * 256 * 4, 0);
    d.pending.assign(d.nstates, 0);
    d.flush = fffd;
    auto idle = [&](int b, int* next, std::vector<int>& em) {
      if (b < 0x80) {
        em.push_back(pt_.of((uint32_t)b));
        *next = 0;
      } else if (b >= 0xC2 && b <= 0xF4) {
        *next = l1[b];
      } else {
        em.push_back(fffd);
        *next = 0;
      }
    };
    auto put = [&](int q, int b, int next, const std::vector<int>& em) {
      const size_t k = (size_t)q * 256 + b;
      d.next[k] = next;
      d.nemit[k] = (uint8_t)em.size();
      for (size_t e = 0; e < em.size(); ++e) d.emit[k * 4 + e] = (uint16_t)em[e];
    };
    for (int b = 0; b < 256; ++b) {
      std::vector<int> em;
      int nx;
      idle(b, &nx, em);
      put(0, b, nx, em);
    }
    for (size_t s = 0; s < specs_.size(); ++s) {
      const Spec& sp = specs_[s];
      const int q = (int)s + 1;
      d.pending[q] = (uint8_t)sp.level;
      for (int b = 0; b < 256; ++b) {
        std::vector<int> em;
        int nx = 0;
        if (b >= sp.lo && b <= sp.hi) {
          const int v = sp.act[b - sp.lo];
          if (sp.final) em.push_back(v);
          else nx = v;
        } else {
          // DecodeRune fails: the lead byte is U+FFFD and the pending
          // continuation bytes decode one U+FFFD each; b starts afresh
          for (int i = 0; i < sp.level; ++i) em.push_back(fffd);
          idle(b, &nx, em);
        }
        put(q, b, nx, em);
      }
    }
    return d;
  }

 private:
  // a pending state: `level` bytes held; on a byte in [lo, hi] either the
  // rune completes (final: emit act[b - lo]) or state act[b - lo] follows
  struct Spec {
    int level;
    bool final;
    int lo, hi;
    std::vector<int> act;
  };
  const Partition& pt_;
  std::vector<Spec> specs_;
  std::map<std::vector<int>, int> ids_;

  int intern(int level, bool final, int lo, int hi, const std::vector<int>& act) {
    std::vector<int> key{level, final, lo, hi};
    const bool same = std::all_of(act.begin(), act.end(), [&](int v) { return v == act[0]; });
    if (same) {
      key.push_back(-1);
      key.push_back(act[0]);
    } else {
      key.insert(key.end(), act.begin(), act.end());
    }
    auto it = ids_.find(key);
    if (it != ids_.end()) return it->second;
    specs_.push_back({level, final, lo, hi, act});
    const int id = (int)specs_.size();
    ids_.emplace(key, id);
    return id;
  }
  // the classes of the 64 code points base .. base + 63
  std::vector<int> block(uint32_t base) {
    const int u = pt_.uniform(base, base + 63);
    if (u >= 0) return std::vector<int>(64, u);
    std::vector<int> v(64);
    for (int i = 0; i < 64; ++i) v[i] = pt_.of(base + i);
    return v;
  }
  // a state waiting for the last byte of a rune whose code points start at base
  int last_byte(int level, uint32_t base) { return intern(level, true, 0x80, 0xBF, block(base)); }
  int state2(int lead) { return last_byte(1, (uint32_t)(lead & 0x1F) << 6); }
  int lead3(int lead) {
    const int lo = lead == 0xE0 ? 0xA0 : 0x80, hi = lead == 0xED ? 0x9F : 0xBF;
    std::vector<int> act;
    for (int b1 = lo; b1 <= hi; ++b1) act.push_back(last_byte(2, ((uint32_t)(lead & 0x0F) << 12) | ((b1 & 0x3F) << 6)));
    return intern(1, false, lo, hi, act);
  }
  int lead4(int lead) {
    const int lo = lead == 0xF0 ? 0x90 : 0x80, hi = lead == 0xF4 ? 0x8F : 0xBF;
    std::vector<int> act;
    for (int b1 = lo; b1 <= hi; ++b1) {
      const uint32_t base = ((uint32_t)(lead & 0x07) << 18) | ((b1 & 0x3F) << 12);
      std::vector<int> a2;
      const int u = pt_.uniform(base, base + 4095);
      if (u >= 0) {
        a2.assign(64, intern(3, true, 0x80, 0xBF, std::vector<int>(64, u)));
      } else {
        for (int b2 = 0x80; b2 <= 0xBF; ++b2) a2.push_back(last_byte(3, base | ((b2 & 0x3F) << 6)));
      }
      act.push_back(intern(2, false, 0x80, 0xBF, a2));
    }
    return intern(1, false, lo, hi, act);
  }
};

int lower_node(const std::vector<GNode>& gn, int id, const Partition& pt, int nsym, Prog* g) {
  const GNode& n = gn[id];
  Node o;
  switch (n.kind) {
    case GNode::EMPTY: return g->add(o);
    case GNode::SET: {
      SymSet s(nsym);
      for (int c = 0; c < nsym; ++c)
        if (rs_has(n.set, pt.rep[c])) s.set(c);
      return g->add_set(s);
    }
    case GNode::ASSERT:
      o.kind = Node::ASSERT;
      o.as = n.as;
      return g->add(o);
    case GNode::CAT:
    case GNode::ALT:
    case GNode::REP:
      o.kind = n.kind == GNode::CAT ? Node::CAT : n.kind == GNode::ALT ? Node::ALT : Node::REP;
      o.min = n.min;
      o.max = n.max;
      for (int k : n.kids) o.kids.push_back(lower_node(gn, k, pt, nsym, g));
      return g->add(o);
  }
  return g->add(o);
}

// The runes Go's Prog.Prefix / onePassPrefix would take as the literal
// prefix (leading single-rune literals, through concatenations, groups and
// repeats of at least one), over-approximated at alternations.  Go finds
// candidate match starts by a *byte* search for that prefix, so a U+FFFD
// there matches only the bytes EF BF BD on some paths (the backtracker, the
// one-pass matcher) and also an invalid byte on another (the NFA, when the
// rune at the scan position is U+FFFD): the result then depends on the input
// length and program size, not only on the language.
void leading_literals(const std::vector<GNode>& gn, int id, std::vector<uint32_t>* out, bool* complete) {
  const GNode& n = gn[id];
  switch (n.kind) {
    case GNode::EMPTY: *complete = true; return;
    case GNode::SET:
      if (n.set.size() == 1 && n.set[0].first == n.set[0].second) {
        out->push_back(n.set[0].first);
        *complete = true;
      } else {
        *complete = false;
      }
      return;
    case GNode::CAT:
      for (size_t k = 0; k < n.kids.size(); ++k) {
        bool c = false;
        // a leading \A / ^ is skipped by onePassPrefix
        if (k == 0 && gn[n.kids[0]].kind == GNode::ASSERT && gn[n.kids[0]].as == kBeginText) continue;
        leading_literals(gn, n.kids[k], out, &c);
        if (!c) {
          *complete = false;
          return;
        }
      }
      *complete = true;
      return;
    case GNode::REP: {
      bool c = false;
      if (n.min >= 1) leading_literals(gn, n.kids[0], out, &c);
      *complete = false;
      return;
    }
    case GNode::ALT:
      for (int k : n.kids) {
        bool c = false;
        leading_literals(gn, k, out, &c);
      }
      *complete = false;
      return;
    case GNode::ASSERT: *complete = false; return;
  }
}

}  // namespace

void go_syntax_check(const std::string& re) {
  std::vector<GNode> nodes;
  GoParser(re, nodes).parse();
}

void go_compile(const std::string& re, Prog* g, Decoder* dec) {
  std::vector<GNode> nodes;
  const int root = GoParser(re, nodes).parse();
  {
    std::vector<uint32_t> pre;
    bool c = false;
    leading_literals(nodes, root, &pre, &c);
    if (std::find(pre.begin(), pre.end(), kRuneError) != pre.end())
      fail(CG_UNSUPPORTED, "Go regexp with U+FFFD in its literal prefix (Go's byte prefix search decides)");
  }
  // the partition also separates what the assertions look at: word
  // characters (IsWordChar, ASCII) and '\n'
  const RS word{{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}, nl{{'\n', '\n'}};
  std::vector<const RS*> sets{&word, &nl};
  for (const auto& n : nodes)
    if (n.kind == GNode::SET) sets.push_back(&n.set);
  const Partition pt = partition(sets);
  const int nsym = (int)pt.rep.size();
  if (nsym > 65535) fail(CG_UNSUPPORTED, "Go regexp has too many rune classes");
  g->nsym = nsym;
  g->root = lower_node(nodes, root, pt, nsym, g);
  g->word.assign(nsym, 0);
  g->newline.assign(nsym, 0);
  for (int c = 0; c < nsym; ++c) {
    g->word[c] = rs_has(word, pt.rep[c]);
    g->newline[c] = pt.rep[c] == '\n';
  }
  *dec = DecoderBuilder(pt).build();
}

}  // namespace rx
}  // namespace cg
