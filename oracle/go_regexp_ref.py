"""CPU restatement of Go 1.10 ``regexp`` as proxylib's parsers use it:
``regexp.MustCompile(v)`` then ``MatchString`` / ``Match``
(proxylib/r2d2/r2d2parser.go:80,103, proxylib/cassandra/cassandraparser.go:
89,113, proxylib/memcached/parser.go:91,132) and the syntax check of
``PortRuleHTTP.Sanitize`` (pkg/policy/api/http.go:66-84).

TEST INFRASTRUCTURE ONLY (the checker for tests/ and smoke()); it shares no
code with cilium_amd.  Go's regexp is not in /root/reference (Go 1.10.3 per
contrib/packaging/docker/Dockerfile.runtime:84), so this restates its
published algorithm:

* parsing follows regexp/syntax/parse.go with the Perl flags
  (ClassNL | OneLine | PerlX | UnicodeGroups): the operator stack with
  left-paren / vertical-bar markers, flag groups scoped to the enclosing
  group, repeat rules (no stacked repeats, {n,m} <= 1000, '{' literal when
  not a repeat), escapes (octal, \\x{...}, \\Q...\\E, \\pN), classes (']'
  first, [:posix:], Perl and Unicode groups, folding);
* matching runs Python's backtracking ``re`` over the input decoded the way
  utf8.DecodeRune steps through it (each invalid byte is one U+FFFD), with
  every construct lowered to explicit code point classes and lookarounds —
  no Python flag semantics are relied on.

Unicode tables (categories, scripts, simple-folding orbits of Unicode 10.0)
come from oracle/go_unicode10.json, written by tools/gen_go_unicode.py.

**Parity pinning:** Go's own regexp test vectors are not in the reference;
the syntax cases in tests/golden/go_regex_kat.json are the documented Go
behaviours (regexp/syntax parse_test.go invalid/only-Perl lists as
published), so Go-regexp parity is pinned by those and otherwise
**unpinned** beyond this restatement.
"""
from __future__ import annotations

import json
import os
import re
from functools import lru_cache

MAX_RUNE = 0x10FFFF
RUNE_ERROR = 0xFFFD


class GoSyntaxError(ValueError):
    pass


def decode_rune(b: bytes, i: int) -> tuple[int, int]:
    """utf8.DecodeRune(b[i:]): (rune, width), (U+FFFD, 1) when invalid."""
    c = b[i]
    if c < 0x80:
        return c, 1
    if 0xC2 <= c <= 0xDF:
        need, lo, hi = 2, 0x80, 0xBF
    elif 0xE0 <= c <= 0xEF:
        need, lo, hi = 3, 0xA0 if c == 0xE0 else 0x80, 0x9F if c == 0xED else 0xBF
    elif 0xF0 <= c <= 0xF4:
        need, lo, hi = 4, 0x90 if c == 0xF0 else 0x80, 0x8F if c == 0xF4 else 0xBF
    else:
        return RUNE_ERROR, 1
    if len(b) - i < need or not lo <= b[i + 1] <= hi:
        return RUNE_ERROR, 1
    r = c & (0x1F if need == 2 else 0x0F if need == 3 else 0x07)
    for k in range(1, need):
        if k > 1 and not 0x80 <= b[i + k] <= 0xBF:
            return RUNE_ERROR, 1
        r = (r << 6) | (b[i + k] & 0x3F)
    return r, need


def go_decode(b: bytes) -> str:
    """The rune sequence Go's matcher steps through."""
    out, i = [], 0
    while i < len(b):
        r, w = decode_rune(b, i)
        out.append(chr(r))
        i += w
    return "".join(out)


@lru_cache(maxsize=1)
def _tables():
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "go_unicode10.json")) as f:
        d = json.load(f)
    orbit_of = {}
    for o in d["orbits"]:
        for c in o:
            orbit_of[c] = o
    return d["categories"], d["scripts"], d["orbits"], orbit_of


# ------------------------------------------------------------ rune sets ---
def norm(rs):
    out = []
    for lo, hi in sorted(rs):
        if out and lo <= out[-1][1] + 1:
            out[-1][1] = max(out[-1][1], hi)
        else:
            out.append([lo, hi])
    return out


def negate(rs):
    out, nxt = [], 0
    for lo, hi in norm(rs):
        if lo > nxt:
            out.append([nxt, lo - 1])
        nxt = hi + 1
    if nxt <= MAX_RUNE:
        out.append([nxt, MAX_RUNE])
    return out


def contains(rs, c):
    return any(lo <= c <= hi for lo, hi in rs)


def fold(rs):
    """appendFoldedRange / appendFoldedClass: add every SimpleFold orbit
    member of every rune in the set."""
    rs = norm(rs)
    _, _, orbits, _ = _tables()
    extra = [[c, c] for o in orbits if any(contains(rs, c) for c in o) for c in o]
    return norm(rs + extra)


PERL = {"d": [[48, 57]], "s": [[9, 10], [12, 13], [32, 32]], "w": [[48, 57], [65, 90], [95, 95], [97, 122]]}
POSIX = {"alnum": [[48, 57], [65, 90], [97, 122]], "alpha": [[65, 90], [97, 122]], "ascii": [[0, 127]],
         "blank": [[9, 9], [32, 32]], "cntrl": [[0, 31], [127, 127]], "digit": [[48, 57]], "graph": [[33, 126]],
         "lower": [[97, 122]], "print": [[32, 126]], "punct": [[33, 47], [58, 64], [91, 96], [123, 126]],
         "space": [[9, 13], [32, 32]], "upper": [[65, 90]], "word": [[48, 57], [65, 90], [95, 95], [97, 122]],
         "xdigit": [[48, 57], [65, 70], [97, 102]]}


def unicode_table(name):
    if name == "Any":
        return [[0, MAX_RUNE]]
    cats, scripts, _, _ = _tables()
    if name in cats:
        return [list(x) for x in cats[name]]
    if name in scripts:
        return [list(x) for x in scripts[name]]
    return None


# ---------------------------------------------------------------- parse ---
# nodes: ("set", rs) ("cat", [..]) ("alt", [..]) ("rep", n, min, max)
# ("assert", kind) ("empty",); stack markers: ("(", flags) and ("|",)
BEGIN_TEXT, END_TEXT, BEGIN_LINE, END_LINE, WORD_B, NOT_WORD_B = range(6)


class _Flags:
    __slots__ = ("fold", "dotnl", "oneline")

    def __init__(self, fold=False, dotnl=False, oneline=True):
        self.fold, self.dotnl, self.oneline = fold, dotnl, oneline

    def copy(self):
        return _Flags(self.fold, self.dotnl, self.oneline)


def _isalnum(c):
    return 48 <= c <= 57 or 65 <= c <= 90 or 97 <= c <= 122


def _unhex(c):
    ch = chr(c)
    return int(ch, 16) if ch in "0123456789abcdefABCDEF" else -1


class _Parser:
    def __init__(self, pattern: bytes):
        runes, i = [], 0
        while i < len(pattern):
            r, w = decode_rune(pattern, i)
            if r == RUNE_ERROR and w == 1:
                raise GoSyntaxError("invalid UTF-8")
            runes.append(r)
            i += w
        self.t = runes
        self.i = 0
        self.stack = []
        self.flags = _Flags()

    def err(self, m):
        raise GoSyntaxError(m)

    def peek(self, k=0):
        j = self.i + k
        return self.t[j] if j < len(self.t) else None

    def push(self, node):
        self.stack.append(node)

    def literal(self, c):
        rs = [[c, c]]
        if self.flags.fold:
            _, _, _, orbit_of = _tables()
            rs = norm(rs + [[x, x] for x in orbit_of.get(c, [])])
        self.push(("set", rs))

    def _is_marker(self, x):
        return x[0] in ("(", "|")

    def concat(self):
        items = []
        while self.stack and not self._is_marker(self.stack[-1]):
            items.append(self.stack.pop())
        items.reverse()
        self.push(("cat", items) if len(items) != 1 else items[0])

    def alternate_to_paren(self):
        """Pop branches (and '|' markers) down to a '(' marker; returns
        (alternation node, the marker) — marker None at the bottom."""
        branches = []
        while self.stack and self.stack[-1][0] != "(":
            x = self.stack.pop()
            if x[0] != "|":
                branches.append(x)
        branches.reverse()
        node = branches[0] if len(branches) == 1 else ("alt", branches)
        return node, (self.stack.pop() if self.stack else None)

    def repeat(self, mn, mx, last_repeat):
        if self.peek() == ord("?"):
            self.i += 1
        if last_repeat:
            self.err("invalid nested repetition operator")
        if not self.stack or self._is_marker(self.stack[-1]):
            self.err("missing argument to repetition operator")
        self.stack[-1] = ("rep", self.stack[-1], mn, mx)

    def parse_int(self, j):
        t = self.t
        if j >= len(t) or not 48 <= t[j] <= 57:
            return None, j
        if j + 1 < len(t) and t[j] == 48 and 48 <= t[j + 1] <= 57:
            return None, j
        k, n = j, 0
        while k < len(t) and 48 <= t[k] <= 57:
            k += 1
        digits = "".join(chr(x) for x in t[j:k])
        n = int(digits)
        return (n if n < 10 ** 8 + 0 and len(digits) <= 9 and n <= 10 ** 8 else -1), k

    def parse_repeat(self):
        """parseRepeat at '{': (min, max, end index) or None."""
        t, j = self.t, self.i + 1
        mn, j = self.parse_int(j)
        if mn is None or j >= len(t):
            return None
        if t[j] != ord(","):
            mx = mn
        else:
            j += 1
            if j >= len(t):
                return None
            if t[j] == ord("}"):
                mx = -1
            else:
                mx, j = self.parse_int(j)
                if mx is None:
                    return None
                if mx < 0:
                    mn = -1
        if j >= len(t) or t[j] != ord("}"):
            return None
        return mn, mx, j + 1

    def perl_flags(self):
        t, i = self.t, self.i
        if len(t) - i > 4 and t[i + 2] == ord("P") and t[i + 3] == ord("<"):
            try:
                end = t.index(ord(">"), i)
            except ValueError:
                self.err("invalid named capture")
            name = t[i + 4:end]
            if not name or not all(c == 95 or _isalnum(c) for c in name):
                self.err("invalid named capture")
            self.push(("(", self.flags.copy()))
            self.i = end + 1
            return
        f = self.flags.copy()
        sign, saw = 1, False
        j = i + 2
        while j < len(t):
            c = chr(t[j])
            j += 1
            if c == "i":
                f.fold, saw = sign > 0, True
            elif c == "m":
                f.oneline, saw = sign < 0, True
            elif c == "s":
                f.dotnl, saw = sign > 0, True
            elif c == "U":
                saw = True
            elif c == "-":
                if sign < 0:
                    break
                sign, saw = -1, False
            elif c in ":)":
                if sign < 0 and not saw:
                    break
                if c == ":":
                    self.push(("(", self.flags.copy()))
                self.flags = f
                self.i = j
                return
            else:
                break
        self.err("invalid or unsupported Perl syntax")

    def parse_escape(self):
        """parseEscape with self.i at '\\'; returns one rune."""
        t = self.t
        self.i += 1
        if self.i >= len(t):
            self.err("trailing backslash at end of expression")
        c = t[self.i]
        self.i += 1
        ch = chr(c)
        if ch in "1234567":
            if self.peek() is None or not 48 <= self.peek() <= 55:
                self.err("invalid escape sequence")
        if ch in "01234567":
            r = c - 48
            for _ in range(2):
                if self.peek() is None or not 48 <= self.peek() <= 55:
                    break
                r = r * 8 + t[self.i] - 48
                self.i += 1
            return r
        if ch == "x":
            if self.peek() is None:
                self.err("invalid escape sequence")
            d = t[self.i]
            self.i += 1
            if d == ord("{"):
                nhex, r = 0, 0
                while True:
                    if self.peek() is None:
                        self.err("invalid escape sequence")
                    d = t[self.i]
                    self.i += 1
                    if d == ord("}"):
                        break
                    v = _unhex(d)
                    if v < 0:
                        self.err("invalid escape sequence")
                    r = r * 16 + v
                    if r > MAX_RUNE:
                        self.err("invalid escape sequence")
                    nhex += 1
                if nhex == 0:
                    self.err("invalid escape sequence")
                return r
            x = _unhex(d)
            y = -1
            if self.peek() is not None:
                y = _unhex(t[self.i])
                self.i += 1
            if x < 0 or y < 0:
                self.err("invalid escape sequence")
            return x * 16 + y
        simple = {"a": 7, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11}
        if ch in simple:
            return simple[ch]
        if c < 0x80 and not _isalnum(c):
            return c
        self.err("invalid escape sequence")

    def unicode_class(self):
        """\\pN \\p{Name} \\PN \\p{^Name} at self.i, or None."""
        t = self.t
        if self.peek() != 92 or self.peek(1) not in (ord("p"), ord("P")):
            return None
        sign = -1 if t[self.i + 1] == ord("P") else 1
        self.i += 2
        if self.peek() is None:
            self.err("invalid character class range")
        if self.peek() != ord("{"):
            name = chr(t[self.i])
            self.i += 1
        else:
            try:
                end = t.index(ord("}"), self.i)
            except ValueError:
                self.err("invalid character class range")
            name = "".join(chr(x) for x in t[self.i + 1:end])
            self.i = end + 1
        if name.startswith("^"):
            sign, name = -sign, name[1:]
        tab = unicode_table(name)
        if tab is None:
            self.err("invalid character class range")
        if self.flags.fold:
            tab = fold(tab)
        return tab if sign > 0 else negate(tab)

    def group(self, rs, sign):
        if self.flags.fold:
            rs = fold(rs)
        return rs if sign > 0 else negate(rs)

    def parse_class(self):
        t = self.t
        self.i += 1
        sign = 1
        if self.peek() == ord("^"):
            sign = -1
            self.i += 1
        cls = []
        first = True
        while True:
            if self.peek() is None:
                self.err("missing closing ]")
            if self.peek() == ord("]") and not first:
                break
            first = False
            if self.peek() == ord("[") and self.peek(1) == ord(":"):
                j = self.i + 2
                while j + 1 < len(t) and not (t[j] == ord(":") and t[j + 1] == ord("]")):
                    j += 1
                if j + 1 < len(t):
                    name = "".join(chr(x) for x in t[self.i + 2:j])
                    gs = 1
                    if name.startswith("^"):
                        gs, name = -1, name[1:]
                    if name not in POSIX:
                        self.err("invalid character class range")
                    cls += self.group(POSIX[name], gs)
                    self.i = j + 2
                    continue
            u = self.unicode_class()
            if u is not None:
                cls += u
                continue
            if self.peek() == 92 and self.peek(1) is not None and chr(self.peek(1)).lower() in PERL:
                g = chr(self.peek(1))
                self.i += 2
                cls += self.group(PERL[g.lower()], 1 if g.islower() else -1)
                continue
            lo = self.class_char()
            hi = lo
            if self.peek() == ord("-") and self.peek(1) is not None and self.peek(1) != ord("]"):
                self.i += 1
                hi = self.class_char()
                if hi < lo:
                    self.err("invalid character class range")
            cls += fold([[lo, hi]]) if self.flags.fold else [[lo, hi]]
        self.i += 1
        return ("set", norm(cls) if sign > 0 else negate(cls))

    def class_char(self):
        if self.peek() is None:
            self.err("missing closing ]")
        if self.peek() == 92:
            return self.parse_escape()
        c = self.t[self.i]
        self.i += 1
        return c

    def parse(self):
        t = self.t
        last_repeat = False
        while self.i < len(t):
            c = chr(t[self.i])
            repeat = False
            if c == "(":
                if self.peek(1) == ord("?"):
                    self.perl_flags()
                else:
                    self.push(("(", self.flags.copy()))
                    self.i += 1
            elif c == "|":
                self.concat()
                self.push(("|",))
                self.i += 1
            elif c == ")":
                self.concat()
                node, mark = self.alternate_to_paren()
                if mark is None:
                    self.err("unexpected )")
                self.flags = mark[1]
                self.push(node)
                self.i += 1
            elif c == "^":
                self.push(("assert", BEGIN_TEXT if self.flags.oneline else BEGIN_LINE))
                self.i += 1
            elif c == "$":
                self.push(("assert", END_TEXT if self.flags.oneline else END_LINE))
                self.i += 1
            elif c == ".":
                self.push(("set", [[0, MAX_RUNE]] if self.flags.dotnl else [[0, 9], [11, MAX_RUNE]]))
                self.i += 1
            elif c == "[":
                self.push(self.parse_class())
            elif c in "*+?":
                self.i += 1
                self.repeat({"*": 0, "+": 1, "?": 0}[c], {"*": -1, "+": -1, "?": 1}[c], last_repeat)
                repeat = True
            elif c == "{":
                rp = self.parse_repeat()
                if rp is None:
                    self.literal(ord("{"))
                    self.i += 1
                else:
                    mn, mx, j = rp
                    if mn < 0 or mn > 1000 or mx > 1000 or (mx >= 0 and mn > mx):
                        self.err("invalid repeat count")
                    self.i = j
                    self.repeat(mn, mx, last_repeat)
                    repeat = True
            elif c == "\\":
                nx = self.peek(1)
                nxc = chr(nx) if nx is not None else ""
                if nxc in ("A", "b", "B", "z"):
                    self.push(("assert", {"A": BEGIN_TEXT, "b": WORD_B, "B": NOT_WORD_B, "z": END_TEXT}[nxc]))
                    self.i += 2
                elif nxc == "C":
                    self.err("invalid escape sequence")
                elif nxc == "Q":
                    self.i += 2
                    while self.i < len(t):
                        if t[self.i] == 92 and self.peek(1) == ord("E"):
                            self.i += 2
                            break
                        self.literal(t[self.i])
                        self.i += 1
                else:
                    u = self.unicode_class()
                    if u is not None:
                        self.push(("set", u))
                    elif nxc.lower() in PERL and nxc:
                        self.i += 2
                        self.push(("set", self.group(PERL[nxc.lower()], 1 if nxc.islower() else -1)))
                    else:
                        self.literal(self.parse_escape())
            else:
                self.literal(t[self.i])
                self.i += 1
            last_repeat = repeat
        self.concat()
        node, mark = self.alternate_to_paren()
        if mark is not None:
            self.err("missing closing )")
        return node


# ------------------------------------------------------- Python lowering ---
_WORD = "[0-9A-Za-z_]"


def _cp(c):
    return "\\U%08x" % c


def _py(node) -> str:
    k = node[0]
    if k == "set":
        rs = node[1]
        if not rs:
            return "(?!)"
        return "[" + "".join(_cp(lo) if lo == hi else _cp(lo) + "-" + _cp(hi) for lo, hi in rs) + "]"
    if k == "cat":
        return "(?:" + "".join(_py(x) for x in node[1]) + ")"
    if k == "alt":
        return "(?:" + "|".join(_py(x) for x in node[1]) + ")"
    if k == "rep":
        _, sub, mn, mx = node
        q = "{%d,}" % mn if mx < 0 else "{%d,%d}" % (mn, mx)
        return "(?:" + _py(sub) + ")" + q
    if k == "assert":
        return {BEGIN_TEXT: r"\A", END_TEXT: r"\Z", BEGIN_LINE: r"(?:\A|(?<=\n))", END_LINE: r"(?:\Z|(?=\n))",
                WORD_B: "(?:(?<!%s)(?=%s)|(?<=%s)(?!%s))" % (_WORD, _WORD, _WORD, _WORD),
                NOT_WORD_B: "(?:(?<!%s)(?!%s)|(?<=%s)(?=%s))" % (_WORD, _WORD, _WORD, _WORD)}[node[1]]
    return ""


class GoRegexp:
    """regexp.MustCompile(pattern); .match_string(b) = MatchString."""

    def __init__(self, pattern):
        if isinstance(pattern, str):
            pattern = pattern.encode("utf-8", "surrogateescape")
        self.ast = _Parser(pattern).parse()
        self.py = re.compile(_py(self.ast), re.DOTALL)

    def match_string(self, data) -> bool:
        if isinstance(data, str):
            data = data.encode("utf-8", "surrogateescape")
        return self.py.search(go_decode(data)) is not None


def compile_ok(pattern) -> bool:
    try:
        GoRegexp(pattern)
        return True
    except GoSyntaxError:
        return False
