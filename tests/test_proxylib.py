"""proxylib generic-L7 rules (r2d2, cassandra) on the verdict engine.

KATs are the reference's own r2d2 tests (proxylib/r2d2/r2d2parser_test.go:
70-190: TestR2d2OnDataBasicPass, ...AllowDenyCmd, ...AllowDenyRegex); the
oracle is oracle/proxylib_ref.py (policymap.go + r2d2parser.go + cassandraparser.go
restated).  Cassandra KATs: cassandraparser_test.go:86-280 at the path level.
"""
import numpy as np
import pytest

from cilium_amd import proxylib as P
from oracle.proxylib_ref import ProxylibOracle

CP1 = {"name": "cp1", "policy": 2, "ingress_per_port_policies": [
    {"port": 80, "rules": [{"l7_proto": "r2d2"}]}]}
CP2 = {"name": "cp2", "policy": 2, "ingress_per_port_policies": [
    {"port": 80, "rules": [{"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"cmd": "READ"}}]}}]}]}
CP3 = {"name": "cp3", "policy": 2, "ingress_per_port_policies": [
    {"port": 80, "rules": [{"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"file": "s.*"}}]}}]}]}
# (policy, request line, expected) — ingress connection srcId 1 → port 80
KAT = [
    ("cp1", b"READ sssss", True), ("cp1", b"WRITE sssss", True), ("cp1", b"HALT", True), ("cp1", b"RESET", True),
    ("cp2", b"READ xssss", True), ("cp2", b"WRITE xssss", False),
    ("cp3", b"READ ssss", True), ("cp3", b"WRITE yyyyy", False),
]
# engine-contract cases beyond the reference tests: unlisted port → deny
EXTRA = [("cp1", 81, b"READ sssss", False), ("cp2", 81, b"READ x", False), ("nosuch", 80, b"READ x", False)]


def _eval(pl, cases, fn):
    pols = [pl.index(c[0]) for c in cases]
    ports = [c[1] for c in cases]
    lines = [c[2] for c in cases]
    cf = [P.r2d2_request(x) for x in lines]
    return fn(pols, [1] * len(cases), ports, [1] * len(cases), [c for c, _ in cf], [f for _, f in cf])


def _kat_cases():
    return [(p, 80, line, exp) for p, line, exp in KAT] + EXTRA


def test_oracle_kat():
    o = ProxylibOracle([CP1, CP2, CP3])
    for name, port, line, exp in _kat_cases():
        c, f = P.r2d2_request(line)
        assert o.matches(name, True, port, 1, c, f) == exp, (name, line)


def test_engine_tables_kat(host):
    pl = P.ProxylibPolicy(host)
    pl.update([CP1, CP2, CP3])
    cases = _kat_cases()
    got = _eval(pl, cases, pl.matches_host_diag)
    assert got.tolist() == [int(c[3]) for c in cases]


@pytest.mark.parametrize("rule,msg", [
    ({"cmd": "JUMP"}, "invalid cmd"),
    ({"cmd": "HALT", "file": "x"}, "not compatible"),
    ({"path": "x"}, "Unsupported key"),
])
def test_parse_errors(rule, msg):
    pol = {"name": "e", "ingress_per_port_policies": [
        {"port": 80, "rules": [{"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": rule}]}}]}]}
    with pytest.raises(P.ParseError, match=msg):
        P.translate_policies([pol])


def test_port_structure_errors_and_skips():
    dup = {"name": "d", "ingress_per_port_policies": [{"port": 80}, {"port": 80}]}
    with pytest.raises(P.ParseError, match="Duplicate port"):
        P.translate_policies([dup])
    mix = {"name": "m", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "r2d2"}, {"l7_proto": "other", "l7_rules": {"l7_rules": []}}]}]}
    # "other" is not registered: the port is dropped before the type check
    assert P.translate_policies([mix])[0]["ingress_per_port_policies"] == []
    P.register_l7_rule_parser("other", lambda l7: [])
    try:
        with pytest.raises(P.ParseError, match="Mismatching"):
            P.translate_policies([mix])
    finally:
        P._L7_RULE_PARSERS.pop("other")
    udp = {"name": "u", "ingress_per_port_policies": [{"port": 80, "protocol": "UDP"}]}
    assert P.translate_policies([udp])[0]["ingress_per_port_policies"] == []


FILE_RES = ["s.*", "^/public/", r"\.txt$", "[a-c]+x", "secret", "^a+$", "(foo|bar)[0-9]", "o{2,3}", "^$", "x?y"]
ALPHA = np.frombuffer(b"abcsxy/.0123txfoobarpublicsecret", np.uint8)


def _rand_policies(rng, n_pol=3):
    pols = []
    for pi in range(n_pol):
        pol = {"name": f"p{pi}", "ingress_per_port_policies": [], "egress_per_port_policies": []}
        for key in ("ingress_per_port_policies", "egress_per_port_policies"):
            for port in rng.choice([0, 80, 8080, 443], size=int(rng.integers(0, 4)), replace=False):
                rules = []
                for _ in range(int(rng.integers(0, 4))):
                    r = {}
                    if rng.random() < 0.4:
                        r["remote_policies"] = [int(x) for x in rng.choice(8, size=int(rng.integers(1, 4)),
                                                                           replace=False)]
                    u = rng.random()
                    if u < 0.85:
                        r["l7_proto"] = "r2d2"
                        l7 = []
                        for _ in range(int(rng.integers(0, 4))):
                            rule = {}
                            cmd = str(rng.choice(["", "READ", "WRITE", "HALT", "RESET"]))
                            if cmd:
                                rule["cmd"] = cmd
                            if cmd in ("", "READ", "WRITE") and rng.random() < 0.6:
                                rule["file"] = str(rng.choice(FILE_RES))
                            l7.append({"rule": rule})
                        if l7 or rng.random() < 0.5:
                            r["l7_rules"] = {"l7_rules": l7}
                    elif u < 0.92:
                        r["l7_proto"] = "unknownproto"
                    rules.append(r)
                protocol = "UDP" if rng.random() < 0.05 else "TCP"
                pol[key].append({"port": int(port), "protocol": protocol, "rules": rules})
        pols.append(pol)
    return pols


def _rand_requests(rng, n, n_pol):
    names = [f"p{i}" for i in range(n_pol)] + ["missing"]
    out = []
    for _ in range(n):
        cmd = bytes(rng.choice([b"READ", b"WRITE", b"HALT", b"RESET", b"JUMP"]))
        L = int(rng.integers(0, 14))
        f = ALPHA[rng.integers(0, len(ALPHA), L)].tobytes()
        if rng.random() < 0.2:
            f = bytes(rng.choice([b"/public/a", b"a.txt", b"secret", b"aaa", b"foo7", b"ssss", b""]))
        line = cmd if (not f and rng.random() < 0.5) else cmd + b" " + f
        if rng.random() < 0.05:
            line += b" extra"  # three fields: file stays ""
        out.append((str(rng.choice(names)), bool(rng.random() < 0.5), int(rng.choice([80, 8080, 443, 22])),
                    int(rng.integers(0, 9)), line))
    return out


def _check_random(cl, seed, n, gpu):
    rng = np.random.default_rng(seed)
    pols = _rand_policies(rng)
    reqs = _rand_requests(rng, n, len(pols))
    o = ProxylibOracle(pols)
    pl = P.ProxylibPolicy(cl)
    pl.update(pols)
    cf = [P.r2d2_request(r[4]) for r in reqs]
    args = ([pl.index(r[0]) for r in reqs], [int(r[1]) for r in reqs], [r[2] for r in reqs], [r[3] for r in reqs],
            [c for c, _ in cf], [f for _, f in cf])
    got = (pl.matches if gpu else pl.matches_host_diag)(*args)
    exp = [int(o.matches(r[0], r[1], r[2], r[3], c, f)) for r, (c, f) in zip(reqs, cf)]
    assert got.tolist() == exp


@pytest.mark.parametrize("seed", range(6))
def test_random_tables_vs_oracle(host, seed):
    _check_random(host, seed, 3000, gpu=False)


@pytest.mark.gpu
def test_gpu_kat(gpu):
    pl = P.ProxylibPolicy(gpu)
    pl.update([CP1, CP2, CP3])
    cases = _kat_cases()
    got = _eval(pl, cases, pl.matches)
    assert got.tolist() == [int(c[3]) for c in cases]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_random_vs_oracle(gpu, seed):
    _check_random(gpu, 100 + seed, 20000, gpu=True)


# ------------------------------------------------------------- cassandra ----
# proxylib/cassandra/cassandraparser_test.go: cp6 (query_action select, remotes
# 1,3,4) passes an OPTIONS frame ("/options", :86-115); cp4 (query_table ".*")
# passes and cp1 (query_table "no-match") drops "SELECT ... FROM system.local"
# ("/query/select/system.local", :145-172, :236-280).
def _cass(name, rule):
    return {"name": name, "policy": 2, "ingress_per_port_policies": [{"port": 80, "rules": [
        {"remote_policies": [1, 3, 4], "l7_proto": "cassandra", "l7_rules": {"l7_rules": [{"rule": rule}]}}]}]}


CASS_POLS = [_cass("cp6", {"query_action": "select"}), _cass("cp4", {"query_table": ".*"}),
             _cass("cp1", {"query_table": "no-match"})]
CASS_KAT = [("cp6", b"/options", True), ("cp4", b"/query/select/system.local", True),
            ("cp1", b"/query/select/system.local", False), ("cp1", b"/options", True),
            ("cp6", b"/query/insert/system.local", False), ("cp6", b"/query/select", False)]


def _cass_eval(pl, cases, host_diag):
    n = len(cases)
    return pl.matches_fields([pl.index(c[0]) for c in cases], [1] * n, [c[1] for c in cases], [c[2] for c in cases],
                             [P.cassandra_request(c[3]) for c in cases], host_diag=host_diag)


def test_cassandra_oracle_kat():
    o = ProxylibOracle(CASS_POLS)
    for name, path, exp in CASS_KAT:
        assert o.matches_path(name, True, 80, 1, path) == exp, (name, path)
    assert not o.matches_path("cp6", True, 80, 2, b"/options")  # remote 2 not in {1,3,4}


def test_cassandra_tables_kat(host):
    pl = P.ProxylibPolicy(host)
    pl.update(CASS_POLS)
    cases = [(n, 80, 1, p) for n, p, _ in CASS_KAT] + [("cp6", 80, 2, b"/options")]
    assert _cass_eval(pl, cases, True).tolist() == [int(e) for _, _, e in CASS_KAT] + [0]


@pytest.mark.parametrize("rule,msg", [
    ({"query_action": "explode"}, "invalid query_action"),
    ({"query_action": "create-role", "query_table": "t"}, "not compatible"),
    ({"table": "x"}, "Unsupported key"),
])
def test_cassandra_parse_errors(rule, msg):
    with pytest.raises(P.ParseError, match=msg):
        P.translate_policies([_cass("e", rule)])


CASS_TABLE_RES = ["^system\\.", "local$", "users", "db[0-9]", ".*", "^$", "a|b"]
CASS_ACTIONS = ["select", "insert", "update", "delete", "use", "create-role", "drop-index"]


def _cass_random(rng, n):
    pols = []
    for pi in range(3):
        ports = []
        for port in rng.choice([0, 9042, 80], size=int(rng.integers(1, 3)), replace=False):
            rules = []
            for _ in range(int(rng.integers(0, 3))):
                r = {"l7_proto": "cassandra"}
                if rng.random() < 0.4:
                    r["remote_policies"] = [int(x) for x in rng.choice(6, size=2, replace=False)]
                l7 = []
                for _ in range(int(rng.integers(0, 3))):
                    rule = {}
                    a = str(rng.choice(CASS_ACTIONS + [""]))
                    if a:
                        rule["query_action"] = a
                    if CASS_ACTIONS.index(a) < 5 if a else True:
                        if rng.random() < 0.6:
                            rule["query_table"] = str(rng.choice(CASS_TABLE_RES))
                    l7.append({"rule": rule})
                r["l7_rules"] = {"l7_rules": l7}
                rules.append(r)
            ports.append({"port": int(port), "rules": rules})
        pols.append({"name": f"c{pi}", "ingress_per_port_policies": ports})
    tables = ["system.local", "db1.users", "db2.t", "", "x.local", "ab", "users"]
    reqs = []
    for _ in range(n):
        u = rng.random()
        if u < 0.2:
            path = b"/" + bytes(rng.choice([b"options", b"startup", b"register"]))
        elif u < 0.3:
            path = b"/query/" + bytes(rng.choice([b"select", b"use"]))
        else:
            path = b"/" + bytes(rng.choice([b"query", b"execute", b"batch"])) + b"/" + \
                str(rng.choice(CASS_ACTIONS)).encode() + b"/" + str(rng.choice(tables)).encode()
            if rng.random() < 0.1:
                path += b"/extra"
        reqs.append((f"c{int(rng.integers(0, 4))}", int(rng.choice([9042, 80, 7000])), int(rng.integers(0, 7)),
                     path))
    return pols, reqs


def _check_cass(cl, seed, n, host_diag):
    rng = np.random.default_rng(seed)
    pols, reqs = _cass_random(rng, n)
    o = ProxylibOracle(pols)
    pl = P.ProxylibPolicy(cl)
    pl.update(pols)
    got = _cass_eval(pl, reqs, host_diag)
    assert got.tolist() == [int(o.matches_path(r[0], True, r[1], r[2], r[3])) for r in reqs]


@pytest.mark.parametrize("seed", range(4))
def test_cassandra_random_tables_vs_oracle(host, seed):
    _check_cass(host, seed, 3000, True)


@pytest.mark.gpu
def test_gpu_cassandra_kat_and_random(gpu):
    pl = P.ProxylibPolicy(gpu)
    pl.update(CASS_POLS)
    cases = [(n, 80, 1, p) for n, p, _ in CASS_KAT]
    assert _cass_eval(pl, cases, False).tolist() == [int(e) for _, _, e in CASS_KAT]
    for seed in range(3):
        _check_cass(gpu, 200 + seed, 20000, False)


# ------------------------------------------ golden: reference policy texts ----
def _golden():
    import json
    import os
    return json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "proxylib_kat.json")))


def _golden_eval(cl, matches_fn_name):
    g = _golden()
    pols, cases = [], []
    for kind in ("r2d2", "cassandra"):
        for c in g[kind]:
            pol = P.parse_policy_text(c["policy"])
            pol["name"] = f"{kind}-{pol['name']}"
            pols.append(pol)
            cases += [(kind, pol["name"], req.encode(), exp) for req, exp in c["requests"]]
    o = ProxylibOracle(pols)
    for kind, name, req, exp in cases:  # the oracle against the reference's assertions
        if kind == "r2d2":
            assert o.matches(name, True, g["port"], g["remote"], *P.r2d2_request(req)) == exp, (name, req)
        else:
            assert o.matches_path(name, True, g["port"], g["remote"], req) == exp, (name, req)
    pl = P.ProxylibPolicy(cl)
    pl.update(pols)
    fields = [[(b"cmd", c), (b"file", f)] for c, f in [P.r2d2_request(r) for k, _, r, _ in cases if k == "r2d2"]]
    fields += [P.cassandra_request(r) for k, _, r, _ in cases if k == "cassandra"]
    ordered = [c for c in cases if c[0] == "r2d2"] + [c for c in cases if c[0] == "cassandra"]
    n = len(ordered)
    got = pl.matches_fields([pl.index(c[1]) for c in ordered], [1] * n, [g["port"]] * n, [g["remote"]] * n, fields,
                            host_diag=(matches_fn_name == "host"))
    assert got.tolist() == [int(c[3]) for c in ordered]


def test_golden_policy_texts(host):
    """The reference tests' protobuf-text policies (tests/golden/proxylib_kat.json)."""
    _golden_eval(host, "host")


@pytest.mark.gpu
def test_gpu_golden_policy_texts(gpu):
    _golden_eval(gpu, "gpu")


def test_policy_text_forms():
    """Brace and angle-bracket message forms, comments, repeated fields."""
    t = '''
    # comment
    name: "x" policy: 7
    egress_per_port_policies { port: 9042 protocol: TCP rules {
        remote_policies: 5 remote_policies: 6
        l7_proto: "cassandra"
        l7_rules { l7_rules { rule { key: "query_action" value: "select" }
                              rule { key: "query_table" value: "^db\\\\." } } }
    } }
    egress_per_port_policies < port: 53 protocol: UDP >
    '''
    p = P.parse_policy_text(t)
    assert p["name"] == "x" and p["policy"] == 7
    pp = p["egress_per_port_policies"]
    assert [x["port"] for x in pp] == [9042, 53] and pp[1]["protocol"] == "UDP"
    r = pp[0]["rules"][0]
    assert r["remote_policies"] == [5, 6]
    assert r["l7_rules"] == {"l7_rules": [{"rule": {"query_action": "select", "query_table": "^db\\."}}]}


# ----------------------------------------- arbitrary bytes in r2d2 fields --
# r2d2 compares the whole cmd and runs Go's regexp on the whole file
# (r2d2parser.go:61-85, :157-183): a NUL or control byte inside either is
# part of the string, not a separator, and there is no HTTP codec to reject
# it.  The engine escapes such bytes (proxylib.escape_value) instead of
# cutting or denying the request.
CTRL_POLS = [
    {"name": "c1", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"cmd": "READ"}}]}}]}]},
    {"name": "c2", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"file": "^pub$"}}, {"rule": {"file": "a.b"}},
                                                       {"rule": {"cmd": "WRITE", "file": "x\\sy"}}]}}]}]},
]
CTRL_LINES = [b"READ\0x foo", b"READ a\x01b", b"READ pub\0secret", b"READ pub", b"WRITE a\rb", b"WRITE a\nb",
              b"WRITE x\x0by", b"WRITE x\ty", b"READ \x03\x10", b"READ a\x7fb", b"READ\x02 pub", b"HALT",
              b"READ a\x00b", b"\0\0\0\0 \x01\x02\x03"]


def _ctrl_cases():
    return [(n, line) for n in ("c1", "c2") for line in CTRL_LINES]


def _ctrl_check(cl, gpu: bool):
    pl = P.ProxylibPolicy(cl)
    pl.update(CTRL_POLS)
    o = ProxylibOracle(CTRL_POLS)
    cases = _ctrl_cases()
    cmds, files = zip(*[P.r2d2_request(line) for _, line in cases])
    pol = [pl.index(n) for n, _ in cases]
    one = [1] * len(cases)
    got = (pl.matches if gpu else pl.matches_host_diag)(pol, one, [80] * len(cases), one, cmds, files)
    exp = [o.matches(n, True, 80, 1, c, f) for (n, _), c, f in zip(cases, cmds, files)]
    assert got.tolist() == [int(x) for x in exp], [(c, g, e) for c, g, e in zip(cases, got, exp) if g != e]
    # the cases the review named: cmd "READ\0x" is not READ; "pub\0secret" is not ^pub$;
    # control bytes are compared, not rejected
    d = dict(zip(cases, got.tolist()))
    assert d[("c1", b"READ\0x foo")] == 0 and d[("c1", b"READ a\x01b")] == 1
    assert d[("c2", b"READ pub\0secret")] == 0 and d[("c2", b"READ pub")] == 1


def test_control_bytes_tables_vs_oracle(host):
    _ctrl_check(host, gpu=False)


@pytest.mark.gpu
def test_gpu_control_bytes_vs_oracle(gpu):
    _ctrl_check(gpu, gpu=True)


def test_escape_value():
    assert P.escape_value(b"abc") == b"abc"
    assert P.escape_value(b"a\0b\x03") == b"a\x03\x10b\x03\x13"
