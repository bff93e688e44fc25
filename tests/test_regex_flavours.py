"""The two regex flavours the reference enforces, each against its own oracle.

* Envoy (``regex_match``, full match): std::regex ECMAScript as libstdc++
  runs it (envoy/cilium_network_policy.h:68-71) — word boundaries, POSIX
  bracket classes, collating elements and equivalence classes, libstdc++'s
  escapes; checked against the oracle's std::regex (oracle/oracle.cc).
* Go (proxylib rules, unanchored): Go 1.10 regexp/syntax with the Perl
  flags, matched over runes with each invalid byte one U+FFFD
  (proxylib/r2d2/r2d2parser.go:80,103, cassandra/cassandraparser.go:89,113,
  memcached/parser.go:91,132); checked against oracle/go_regexp_ref.py and
  the Go known answers of tests/golden/go_regex_kat.json.

CPU tests run the compiled DFAs through cg_diag_regex_match and the
engine's host walkers; the GPU tests run the same constructs through the
kernels (http_kernel for r2d2 / cassandra / memcache and Envoy policies).
"""
import ctypes as C
import random
import unicodedata

import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import proxylib as P
from cilium_amd.policy import PolicyValidationError, PortRuleHTTP
from kat_util import load
from oracle.go_regexp_ref import GoRegexp, GoSyntaxError, go_decode
from oracle.proxylib_ref import ProxylibOracle

GO_KAT = load("go_regex_kat.json")


def _b(p) -> bytes:
    return p.encode("utf-8", "surrogateescape") if isinstance(p, str) else p


def engine(p, s: bytes, go: bool) -> int:
    """1/0 = match / no match; -code when the compiler refuses."""
    p = _b(p)
    res = C.c_uint8()
    buf = np.frombuffer(s, np.uint8) if s else np.zeros(1, np.uint8)
    rc = N.lib.cg_diag_regex_match(p, len(p), buf.ctypes.data, len(s), 1 if go else 0, C.byref(res))
    return -rc if rc else res.value


def go_oracle(p):
    try:
        return GoRegexp(_b(p))
    except GoSyntaxError:
        return None


# ------------------------------------------------------------------ Go ---
def test_go_syntax_kat():
    for p in GO_KAT["invalid"]:
        assert go_oracle(p) is None, p
        assert engine(p, b"", True) == -N.CG_POLICY_REJECTED, p
        with pytest.raises(N.CiliumGPUError):
            N.regex_validate(p, N.CG_REGEX_GO)
    for p in GO_KAT["valid"]:
        assert go_oracle(p) is not None, p
        assert engine(p, b"", True) >= 0, p
        N.regex_validate(p, N.CG_REGEX_GO)


def test_go_match_kat():
    for c in GO_KAT["matches"]:
        s = bytes.fromhex(c["input"])
        if c["match"] is None:  # refused: Go's byte prefix search decides these (regex_go.cc leading_literals)
            assert engine(c["pattern"], s, True) == -N.CG_UNSUPPORTED, c
            continue
        assert go_oracle(c["pattern"]).match_string(s) == c["match"], c
        assert engine(c["pattern"], s, True) == int(c["match"]), c


def test_go_decode_matches_decode_rune():
    assert go_decode(b"a\xe2\x82\xac") == "a€"
    assert go_decode(b"\xe2\x82a") == "\ufffd\ufffda"  # per byte, not Python's maximal subpart
    assert go_decode(b"\xed\xa0\x80") == "\ufffd" * 3  # surrogates are invalid
    assert go_decode(b"\xf4\x90\x80\x80") == "\ufffd" * 4  # > U+10FFFF
    assert go_decode(b"\xc0\x80") == "\ufffd" * 2  # overlong
    assert go_decode(b"\xf0\x9f\x98") == "\ufffd" * 3  # truncated


GO_ATOMS = ["a", "k", "K", "s", "é", "É", "中", "ſ", "\u212a", ".", "\\pL", "\\p{Greek}", "\\PN", "\\p{^Lu}", "[[:alpha:]]",
            "[[:^digit:]]", "[^a]", "[a-zé]", "\\d", "\\w", "\\s", "\\D", "\\W", "\\S", "\\A", "\\z", "^", "$", "\\b",
            "\\B", "\\Q.*\\E", "\\x{e9}", "\\101", "{", "a{,3}", "(?i)", "(?s)", "(?m)", "(?U)", "(?-i)", "(?i:a|k)",
            "(?P<n>a)", "(a|é)", "(?:)", "[^\\n]", "\\n", "[]a]", "[^]a]", "[\\d-z]", "\\.", "\\-", "\\x41",
            "[[:word:]]", "\\pN", "\\p{Han}", "(?i)[^k]", "[k-m]", "\\C", "\\8", "(?<n>a)", "(?=a)", "\\1", "[a-",
            "(?P<>a)", "x{1001}", "\\p{Lu}", "(?i)\\p{Lu}", "[\\p{Greek}\\d]", "\\P{^Han}", "(?m:$)", "[^\\x{0}-\\x{7f}]"]
GO_QUANTS = ["", "", "", "*", "+", "?", "{2}", "{1,2}", "*?", "{0,}", "**", "{2}{3}"]
GO_INPUT = [b"a", b"k", b"K", "\u212a".encode(), "ſ".encode(), "é".encode(), "É".encode(), "中".encode(), b"\xff",
            b"\xe2\x82", b"\x80", b"\n", b" ", b"_", b"1", b"\xef\xbf\xbd", "α".encode(), b"S", b"s", b"\xf0\x90\x80",
            b"\xed\xa0\x80", b".", b"*", b"A", "٣".encode(), b"\x00", b"{"]


def go_random_case(rng):
    r = "".join(rng.choice(GO_ATOMS) + rng.choice(GO_QUANTS) for _ in range(rng.randint(1, 4)))
    if rng.random() < 0.2:
        r += "|" + rng.choice(GO_ATOMS)
    return r


@pytest.mark.parametrize("seed", range(4))
def test_go_random_vs_oracle(seed):
    """Random Go patterns: the same syntax verdict as the oracle, and the
    same MatchString result on inputs with non-ASCII runes, case-fold
    partners, invalid and truncated sequences and surrogate encodings."""
    rng = random.Random(4000 + seed)
    checked = valid = 0
    for _ in range(700):
        r = go_random_case(rng)
        g = go_oracle(r)
        e0 = engine(r, b"", True)
        if e0 == -N.CG_UNSUPPORTED:
            continue
        assert (e0 >= 0) == (g is not None), r
        if g is None:
            continue
        valid += 1
        for _ in range(20):
            s = b"".join(rng.choice(GO_INPUT) for _ in range(rng.randint(0, 6)))
            assert engine(r, s, True) == int(g.match_string(s)), (r, s)
            checked += 1
    assert valid > 200 and checked > 4000


def test_go_unicode_tables_vs_unicodedata():
    """The generated Unicode-10 category tables against Python's own
    unicodedata (13.0): every code point assigned in both keeps its general
    category except the handful Unicode changed after 10.0."""
    import json
    import os
    with open(os.path.join(os.path.dirname(oracle.__file__), "go_unicode10.json")) as f:
        cats = json.load(f)["categories"]
    leaf = [c for c in cats if len(c) == 2]
    n = diff = 0
    for c in leaf:
        for lo, hi in cats[c]:
            for cp in range(lo, hi + 1):
                n += 1
                if unicodedata.category(chr(cp)) != c:
                    diff += 1
    assert n > 270_000 and diff < 50, (n, diff)
    for big in "CLMNPSZ":  # an aggregate category is the union of its leaves
        agg = sum(hi - lo + 1 for lo, hi in cats[big])
        assert agg == sum(hi - lo + 1 for c in leaf if c[0] == big for lo, hi in cats[c])


# ----------------------------------------------------------- ECMAScript ---
ECMA_ATOMS = ["a", "b", "x", "_", "1", " ", "\\b", "\\B", "[[:alpha:]]", "[[:digit:]x]", "[[.a.]-c]", "[[=a=]]",
              "[[.hyphen.]]", "\\cJ", "\\c1", "\\u0141", "\\0", "\\01", "[\\b]", "[^[:space:]]", "[[:ALPHA:]]",
              "[[:w:]]", "[[:punct:]]", "[[:cntrl:]]", "[[:xdigit:]]", "[[:print:]]", "[[:graph:]]", "[[:blank:]]",
              "[[:upper:][:lower:]]", "[[.NUL.]]", "[[.space.]a]", "[[=A=]]", "[[:alpha:]-]", "[a-[:digit:]]",
              "[[:foo:]]", "[[.ab.]]", "[[.-.]]", "[[", "[\\1]", "\\1", "\\x4", "[[.a.]-[.c.]]", "(?:a|\\b)", "[--a]",
              "[a--]", "[\\d-]", ".", "\\w", "\\W", "$", "^", "\\c", "[]", "[^]", "\\s", "[\\s\\d]", "(?=a)"]
ECMA_QUANTS = ["", "", "", "*", "+", "?", "{2}", "{1,2}", "*?"]
ECMA_INPUT = ["a", "b", "x", "_", "1", " ", "\t", "\n", "-", "A", "c", "\x00", "\x80", "\xff", "\x0b", "\x01", ".", "[",
              "J", "\x7f"]


@pytest.mark.parametrize("seed", range(3))
def test_ecma_random_vs_std_regex(seed):
    """Full match against std::regex_match: \\b \\B, [:class:] [.coll.]
    [=equiv=] brackets and libstdc++'s escapes; the same syntax verdict
    (UNSUPPORTED only for backreferences and lookahead)."""
    rng = random.Random(5000 + seed)
    checked = 0
    for _ in range(700):
        r = "".join(rng.choice(ECMA_ATOMS) + rng.choice(ECMA_QUANTS) for _ in range(rng.randint(1, 4)))
        if rng.random() < 0.2:
            r += "|" + rng.choice(ECMA_ATOMS)
        p = r.encode("latin-1")
        ov = oracle.regex_match(p, b"") != -1
        e0 = engine(p, b"", False)
        if e0 == -N.CG_UNSUPPORTED:
            assert ov and ("\\1" in r or "(?=" in r), r
            continue
        assert (e0 >= 0) == ov, r
        if not ov:
            continue
        for _ in range(20):
            s = "".join(rng.choice(ECMA_INPUT) for _ in range(rng.randint(0, 6))).encode("latin-1")
            assert engine(p, s, False) == oracle.regex_match(p, s), (r, s)
            checked += 1
    assert checked > 3000


def test_sanitize_is_go_syntax_and_envoy_compiles_ecmascript(host):
    """PortRuleHTTP.Sanitize accepts what Go's regexp.Compile accepts
    (http.go:66-84); Envoy then compiles the same string with std::regex, which
    rejects Go-only syntax: the NPDS update fails as a whole."""
    for ok in ["(?i)^/api", "\\pL+", "/v1/\\z", "\\Qa.b\\E", "[[:alpha:]]+", "GET|HEAD"]:
        PortRuleHTTP(Path=ok, Method="GET").sanitize()
    for bad in ["a**", "(?=x)", "\\1", "*", "(?<n>x)", "\\C"]:
        with pytest.raises(PolicyValidationError):
            PortRuleHTTP(Path=bad).sanitize()
    for go_only, envoy_ok in [("(?i)^/api", False), ("\\pL+", True), ("[[:alpha:]]+", True), ("\\Qa\\E", True),
                              ("\\bapi\\b", True)]:
        pol = [{"name": "p", "ingress_per_port_policies": [{"port": 80, "rules": [
            {"http_rules": {"http_rules": [{"headers": [{"name": ":path", "regex_match": go_only}]}]}}]}]}]
        assert (oracle.regex_match(go_only.encode(), b"") != -1) == envoy_ok, go_only
        if envoy_ok:
            host.update_http_policy(pol)
        else:
            with pytest.raises(N.CiliumGPUError) as ei:
                host.update_http_policy(pol)
            assert ei.value.code == N.CG_POLICY_REJECTED


# --------------------------------------------- through the verdict tables ---
# One r2d2 rule per Go construct; files with non-ASCII, case-fold partners and
# invalid UTF-8 (r2d2parser.go:80 MatchString on the file field)
GO_CONSTRUCTS = ["(?i)^readme", "(?s)a.b", "(?m)^x$", "(?U)a+b", "(?P<f>[a-z]+)\\.txt\\z", "\\Aetc/", "\\.conf\\z",
                 "\\Q*.log\\E", "[[:upper:]]{2}", "[[:^alpha:]]", "\\p{Lu}{2}", "\\p{Greek}", "\\p{Han}+", "\\PN\\z",
                 "\\bkey\\b", "\\Bey", "^.{2}$", "^[^/]{3}$", "(?i)straße", "(?i)k", "(?i)\\w+\\d", "\\x{e9}t\\x{e9}",
                 "[é-ú]", "^\\p{Lu}", "\\101B"]
FILES = [b"README", b"readme.md", b"ReadMe", b"a\nb", b"a-b", b"x\ny", b"y\nx\n", b"aab", b"ab", b"notes.txt",
         b"notes.txt\n", b"etc/passwd", b"/etc/x", b"app.conf", b"app.conf.bak", b"*.log", b"x.log", b"ABc", b"aBC",
         b"a1", "été".encode(), "中文".encode(), "αβγ".encode(), b"\xff", b"\xe2\x82", "é".encode(), b"\xc3",
         b"key", b"a key.", b"monkey", b"keys", "STRASSE".encode(), "straße".encode(), "\u212a".encode(), b"K",
         b"ab1", "ó".encode(), "Élan".encode(), b"AB", b"ABC", b"\xef\xbf\xbd", b"\xed\xa0\x80", b"", b"1"]


def _r2d2_construct_policy():
    rules = [{"remote_policies": [1], "l7_proto": "r2d2",
              "l7_rules": {"l7_rules": [{"rule": {"cmd": "READ", "file": rx}}]}}
             for rx in GO_CONSTRUCTS]
    # one port per construct, so each request sees exactly one regex
    return [{"name": "go", "ingress_per_port_policies": [
        {"port": 1000 + i, "rules": [r]} for i, r in enumerate(rules)]}]


def _r2d2_construct_check(cl, gpu: bool):
    pols = _r2d2_construct_policy()
    o = ProxylibOracle(pols)
    pl = P.ProxylibPolicy(cl)
    pl.update(pols)
    reqs = [(1000 + i, f) for i in range(len(GO_CONSTRUCTS)) for f in FILES]
    n = len(reqs)
    args = ([pl.index("go")] * n, [1] * n, [p for p, _ in reqs], [1] * n, [b"READ"] * n, [f for _, f in reqs])
    got = (pl.matches if gpu else pl.matches_host_diag)(*args)
    exp = [int(o.matches("go", True, p, 1, b"READ", f)) for p, f in reqs]
    bad = [(GO_CONSTRUCTS[reqs[i][0] - 1000], reqs[i][1], exp[i]) for i in range(n) if got[i] != exp[i]]
    assert not bad, bad[:10]
    per = [sum(exp[i * len(FILES):(i + 1) * len(FILES)]) for i in range(len(GO_CONSTRUCTS))]
    assert all(0 < k < len(FILES) for k in per), dict(zip(GO_CONSTRUCTS, per))  # every construct discriminates


def test_r2d2_go_constructs_tables(host):
    _r2d2_construct_check(host, gpu=False)


@pytest.mark.gpu
def test_gpu_r2d2_go_constructs(gpu):
    _r2d2_construct_check(gpu, gpu=True)


def _r2d2_rule(rx, remotes):
    return {"remote_policies": remotes, "l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"file": rx}}]}}


def _rand_go_policy(cl, rng):
    """12 random valid Go rules; a rule whose automaton does not fit one
    program part (CG_UNSUPPORTED, e.g. \\pL: its UTF-8 pending states have
    no self/dead default) is redrawn."""
    rules = []
    for k in range(12):
        while True:
            rx = go_random_case(rng)
            if go_oracle(rx) is None or engine(rx, b"", True) < 0:
                continue
            try:
                P.ProxylibPolicy(cl).update([{"name": "t", "ingress_per_port_policies": [
                    {"port": 80, "rules": [_r2d2_rule(rx, [1])]}]}])
            except N.CiliumGPUError as e:
                assert e.code == N.CG_UNSUPPORTED, (rx, e)
                continue
            break
        rules.append(_r2d2_rule(rx, [1 + k % 3]))
    return [{"name": "rg", "ingress_per_port_policies": [{"port": 80, "rules": rules}]}]


def _rand_go_check(cl, seed, n, gpu):
    rng = random.Random(seed)
    pols = _rand_go_policy(cl, rng)
    o = ProxylibOracle(pols)
    pl = P.ProxylibPolicy(cl)
    pl.update(pols)
    files = [b"".join(rng.choice(GO_INPUT) for _ in range(rng.randint(0, 8))) for _ in range(n)]
    rem = [rng.randint(1, 4) for _ in range(n)]
    got = (pl.matches if gpu else pl.matches_host_diag)([pl.index("rg")] * n, [1] * n, [80] * n, rem,
                                                        [b"READ"] * n, files)
    exp = [int(o.matches("rg", True, 80, r, b"READ", f)) for r, f in zip(rem, files)]
    assert got.tolist() == exp
    assert 0 < sum(exp) < n


@pytest.mark.parametrize("seed", range(2))
def test_r2d2_random_go_policies_tables(host, seed):
    _rand_go_check(host, 600 + seed, 1500, gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_r2d2_random_go_policies(gpu, seed):
    _rand_go_check(gpu, 700 + seed, 20000, gpu=True)


# cassandra table regexes (cassandraparser.go:89,113) on non-ASCII table names
CASS_RX = ["(?i)^ks\\.USERS$", "\\p{Greek}", "^ks\\.\\pL+$", "[[:digit:]]\\z", "\\bt\\b", "(?i)ü", "^.{4}$"]
CASS_TABLES = ["ks.users", "ks.Users", "ks.üsers", "ks.ÜSERS", "ks.αβ", "ks.t", "ks.t2", "ks.tt", "a.t b", "ks.x",
               "ks.中", "k.é"]


def _cass_check(cl, gpu):
    pols = [{"name": "c", "ingress_per_port_policies": [
        {"port": 2000 + i, "rules": [{"l7_proto": "cassandra", "l7_rules": {"l7_rules": [
            {"rule": {"query_action": "select", "query_table": rx}}]}}]} for i, rx in enumerate(CASS_RX)]}]
    o = ProxylibOracle(pols)
    pl = P.ProxylibPolicy(cl)
    pl.update(pols)
    cases = [(2000 + i, ("/query/select/" + t).encode()) for i in range(len(CASS_RX)) for t in CASS_TABLES]
    cases += [(2000, b"/query/select/ks.\xffx"), (2001, b"/query/select/\xce\xb1\xff")]
    n = len(cases)
    got = pl.matches_fields([pl.index("c")] * n, [1] * n, [p for p, _ in cases], [1] * n,
                            [P.cassandra_request(path) for _, path in cases], host_diag=not gpu)
    exp = [int(o.matches_path("c", True, p, 1, path)) for p, path in cases]
    assert got.tolist() == exp
    assert 0 < sum(exp) < n


def test_cassandra_go_tables(host):
    _cass_check(host, gpu=False)


@pytest.mark.gpu
def test_gpu_cassandra_go_constructs(gpu):
    _cass_check(gpu, gpu=True)


# memcache keyRegex (memcached/parser.go:91,132): every key must match
def _memcache_check(cl, gpu):
    from oracle import memcache_ref as MR
    from test_proxylib_memcache import _oracle_matches, _policy
    rules = [{"command": "get", "keyRegex": rx} for rx in ["^\\pL+$", "(?i)^user:", "\\d\\z", "[[:^ascii:]]"]]
    pols = [_policy(f"k{i}", [r]) for i, r in enumerate(rules)]
    pl = P.ProxylibPolicy(cl)
    pl.update(pols)
    keys = [b"user:1", b"USER:2", "ключ".encode(), b"key", "ÉTÉ".encode(), b"\xff", b"abc1", b"x:\xe2\x82"]
    metas = [(b"get", 0, [k]) for k in keys] + [(b"get", 0, [keys[0], keys[2]]), (b"get", 0, keys[1:3])]
    cases = [(i, m) for i in range(len(rules)) for m in metas]
    n = len(cases)
    got = pl.matches_fields([pl.index(f"k{i}") for i, _ in cases], [1] * n, [80] * n, [1] * n,
                            [P.memcache_request(*m) for _, m in cases], host_diag=not gpu)
    exp = [int(_oracle_matches([rules[i]], (1, 3, 4), 1)(MR.Meta(*m))) for i, m in cases]
    assert got.tolist() == exp
    assert 0 < sum(exp) < n


def test_memcache_go_tables(host):
    _memcache_check(host, gpu=False)


@pytest.mark.gpu
def test_gpu_memcache_go_constructs(gpu):
    _memcache_check(gpu, gpu=True)


# Envoy: the ECMAScript additions through the NPDS → http_kernel path
ENVOY_RX = ["\\bv1\\b.*", ".*\\Bing", "[[:alpha:]]+", "/[[:digit:][:upper:]]{2}/?", "[[.slash.]][[=a=]]b.*",
            "[^[:space:]]+", "/\\cz\\u0141", "/[[:punct:]]+"]
PATHS = ["/v1/x", "v1", "/v12", "/sing", "/ing", "abc", "ABC", "/9Z", "/9Z/", "/ab", "/Ab", "/a b", "/zA", "/!?", "/a!",
         "/", "x"]


def _envoy_check(cl, gpu):
    pols = [{"name": "e", "ingress_per_port_policies": [
        {"port": 3000 + i, "rules": [{"http_rules": {"http_rules": [
            {"headers": [{"name": ":path", "regex_match": rx}]}]}}]} for i, rx in enumerate(ENVOY_RX)]}]
    cl.update_http_policy(pols)
    cases = [(3000 + i, p) for i in range(len(ENVOY_RX)) for p in PATHS]
    parts, off = [], [0]
    for _, path in cases:
        b = b":method\0GET\0:path\0" + path.encode() + b"\0"
        parts.append(b)
        off.append(off[-1] + len(b))
    n = len(cases)
    rq = dict(policy=np.zeros(n, np.uint32), ingress=np.ones(n, np.uint8),
              port=np.array([p for p, _ in cases], np.uint16), remote=np.ones(n, np.uint32),
              hdr_blob=np.frombuffer(b"".join(parts), np.uint8).copy(), hdr_off=np.array(off, np.uint64))
    b = cl.pack_http(**rq)
    got = cl.http_verdicts(b) if gpu else cl.http_eval_host_diag(b)
    exp = oracle.HttpOracle(pols).eval(**rq)
    assert np.array_equal(got, exp)
    per = exp.reshape(len(ENVOY_RX), len(PATHS)).sum(1)
    assert (per > 0).all() and (per < len(PATHS)).all(), per


def test_envoy_constructs_tables(host):
    _envoy_check(host, gpu=False)


@pytest.mark.gpu
def test_gpu_envoy_constructs(gpu):
    _envoy_check(gpu, gpu=True)
