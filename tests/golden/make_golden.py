"""Writes the golden fixtures of tests/golden/.

Two kinds of fixture:

* ``*_kat.json`` — known-answer tests transcribed by hand from the
  reference's own tests and documentation (each case cites the file:line of
  the assertion it restates).  Expected values come from those assertions,
  not from running anything.
* ``*_vectors.json`` — seeded input/output vectors produced by the CPU
  oracle (oracle/liboracle.so, std::regex = Envoy's engine) and cross-checked
  here against an independent pure-Python restatement (Python ``re`` for the
  printable-ASCII regex subset where ECMAScript and Python agree) before
  being written.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import random
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from cilium_amd.policy import PortRuleHTTP, get_http_rule  # noqa: E402

# --------------------------------------------------------------- HTTP KATs --
BASIC_RULES = [  # envoy/cilium_integration_test.cc:163-198 (BASIC_POLICY)
    {"remote_policies": [1], "http_rules": {"http_rules": [
        {"headers": [{"name": ":path", "exact_match": "/allowed"}]},
        {"headers": [{"name": ":path", "regex_match": ".*public$"}]},
        {"headers": [{"name": ":authority", "exact_match": "allowedHOST"}]},
        {"headers": [{"name": ":authority", "regex_match": ".*REGEX.*"}]},
        {"headers": [{"name": ":method", "exact_match": "PUT"}, {"name": ":path", "exact_match": "/public/opinions"}]},
    ]}},
    {"remote_policies": [2], "http_rules": {"http_rules": [
        {"headers": [{"name": ":path", "exact_match": "/only-2-allowed"}]},
    ]}},
]
BASIC_POLICY = [{"name": "173", "policy": 3,
                 "ingress_per_port_policies": [{"port": 80, "rules": BASIC_RULES}],
                 "egress_per_port_policies": [{"port": 80, "rules": BASIC_RULES}]}]


def _h(method, path, host, extra=()):
    return [[":method", method], [":path", path], [":authority", host]] + [list(x) for x in extra]


# (name, headers, expect, line) — ingress tests :738-776, egress :821-854.
# The test's SocketOption gives remote identity 1 and port 80 (:217-219).
BASIC_CASES = [
    ("DeniedPathPrefix", _h("GET", "/prefix", "host"), 0, 738),
    ("AllowedPathPrefix", _h("GET", "/allowed", "host"), 1, 742),
    ("AllowedPathPrefixStrippedHeader", _h("GET", "/allowed", "host", [("x-envoy-original-dst-host", "1.1.1.1:9999")]),
     1, 746),
    ("AllowedPathRegex", _h("GET", "/maybe/public", "host"), 1, 751),
    ("DeniedPath", _h("GET", "/maybe/private", "host"), 0, 755),
    ("AllowedHostString", _h("GET", "/maybe/private", "allowedHOST"), 1, 759),
    ("AllowedHostRegex", _h("GET", "/maybe/private", "hostREGEXname"), 1, 763),
    ("DeniedMethod", _h("POST", "/maybe/private", "host"), 0, 767),
    ("AcceptedMethod", _h("PUT", "/public/opinions", "host"), 1, 771),
    ("L3DeniedPath", _h("GET", "/only-2-allowed", "host"), 0, 775),
]


def http_kats() -> dict:
    suites = []
    reqs = []
    for ingress in (1, 0):
        for name, hs, exp, line in BASIC_CASES:
            if not ingress and name == "AllowedPathPrefixStrippedHeader":
                continue  # only an ingress case in the reference
            reqs.append({"name": ("" if ingress else "Egress") + name, "policy": "173", "ingress": ingress,
                         "port": 80, "remote": 1, "headers": hs, "expect": exp,
                         "source": f"envoy/cilium_integration_test.cc:{line if ingress else line + 83}"})
    suites.append({"name": "envoy BASIC_POLICY", "policy": BASIC_POLICY, "requests": reqs})

    # test/runtime/Policies.go:1015-1085 "Extended HTTP Methods tests":
    # httpd1 ingress from app1: {method, /public}; from app2: {method, /public, X-Test: True}
    APP1, APP2, APP3 = 1001, 1002, 1003
    for method in ("GET", "POST"):
        r1 = PortRuleHTTP(Method=method, Path="/public")
        r2 = PortRuleHTTP(Method=method, Path="/public", Headers=["X-Test: True"])
        pol = [{"name": "httpd1", "policy": 2000, "ingress_per_port_policies": [{"port": 80, "rules": [
            {"remote_policies": [APP1], "http_rules": {"http_rules": [{"headers": get_http_rule(r1)[0]}]}},
            {"remote_policies": [APP2], "http_rules": {"http_rules": [{"headers": get_http_rule(r2)[0]}]}},
        ]}]}]
        dest = _h(method, "/public", "httpd1")
        dest_hdr = _h(method, "/public", "httpd1", [("X-Test", "True")])
        cases = [(APP1, dest, 1, 1071), (APP2, dest, 0, 1074), (APP2, dest_hdr, 1, 1077), (APP1, dest_hdr, 1, 1080),
                 (APP3, dest_hdr, 0, 1083), (APP3, dest, 0, 1086)]
        suites.append({"name": f"runtime Extended HTTP Methods {method}", "policy": pol, "requests": [
            {"name": f"{method}-{rid}-{'hdr' if len(h) > 3 else 'plain'}", "policy": "httpd1", "ingress": 1,
             "port": 80, "remote": rid, "headers": h, "expect": e, "source": f"test/runtime/Policies.go:{ln}"}
            for rid, h, e, ln in cases]})

    # Star wars demo policy (examples/demo/sw_policy_http.real.json:13-31) with
    # the outcomes of the demo (test/k8sT/demos.go:137-159 and
    # Documentation/gettingstarted): GET /v1/ allowed, PUT /v1/exhaust-port
    # without the force header → 403, with "X-Has-Force: true" allowed.
    rules = [PortRuleHTTP(Method="GET", Path="/v1/"), PortRuleHTTP(Method="POST", Path="/v1/request-landing/"),
             PortRuleHTTP(Method="PUT", Path="/v1/exhaust-port/", Headers=["X-Has-Force: true"])]
    pol = [{"name": "spaceship", "policy": 257, "egress_per_port_policies": [{"port": 80, "rules": [
        {"remote_policies": [], "http_rules": {"http_rules": [{"headers": get_http_rule(r)[0]} for r in rules]}}]}]}]
    sw = [("GET /v1/", _h("GET", "/v1/", "deathstar"), 1), ("GET /v1", _h("GET", "/v1", "deathstar"), 0),
          ("POST landing", _h("POST", "/v1/request-landing/", "deathstar"), 1),
          ("PUT exhaust-port", _h("PUT", "/v1/exhaust-port/", "deathstar"), 0),
          ("PUT exhaust-port force", _h("PUT", "/v1/exhaust-port/", "deathstar", [("X-Has-Force", "true")]), 1),
          ("PUT exhaust-port Force", _h("PUT", "/v1/exhaust-port/", "deathstar", [("X-Has-Force", "True")]), 0),
          ("other port", [[":method", "DELETE"], [":path", "/"]], 1)]
    suites.append({"name": "star wars demo", "policy": pol, "requests": [
        {"name": n, "policy": "spaceship", "ingress": 0, "port": 80 if n != "other port" else 8080, "remote": 258,
         "headers": h, "expect": e, "source": "examples/demo/sw_policy_http.real.json + test/k8sT/demos.go:150-159"}
        for n, h, e in sw]})
    return {"suites": suites,
            "rejected_policies": [
                {"name": "DuplicatePort", "source": "envoy/cilium_integration_test.cc:779-798",
                 "policy": [{"name": "173", "policy": 3, "ingress_per_port_policies": [
                     {"port": 80, "rules": BASIC_RULES},
                     {"port": 80, "rules": [{"remote_policies": [2], "http_rules": {"http_rules": [
                         {"headers": [{"name": ":path", "value": "/only-2-allowed", "regex": False}]}]}}]}]}]}]}


def translation_kats() -> dict:
    """pkg/envoy/server_test.go:38-93 PortRuleHTTP1..3 → ExpectedHeaders1..3 and
    pkg/policy/api/rule_validation_test.go:155-200 (TestHTTPRuleRegexes)."""
    return {"get_http_rule": [
        {"rule": {"Path": "/foo", "Method": "GET", "Host": "foo.cilium.io", "Headers": ["header2 value", "header1"]},
         "expected": [{"name": ":authority", "regex_match": "foo.cilium.io"},
                      {"name": ":method", "regex_match": "GET"},
                      {"name": ":path", "regex_match": "/foo"},
                      {"name": "header1", "present_match": True},
                      {"name": "header2", "exact_match": "value"}],
         "source": "pkg/envoy/server_test.go:38-43,54-75,326-329"},
        {"rule": {"Path": "/bar", "Method": "PUT"},
         "expected": [{"name": ":method", "regex_match": "PUT"}, {"name": ":path", "regex_match": "/bar"}],
         "source": "pkg/envoy/server_test.go:45-48,77-85"},
        {"rule": {"Path": "/bar", "Method": "GET"},
         "expected": [{"name": ":method", "regex_match": "GET"}, {"name": ":path", "regex_match": "/bar"}],
         "source": "pkg/envoy/server_test.go:50-53,87-93"}],
        "sanitize_rejects": [
            {"rule": {"Method": "GET", "Path": "*"}, "source": "pkg/policy/api/rule_validation_test.go:157-178"},
            {"rule": {"Method": "*", "Path": "/"}, "source": "pkg/policy/api/rule_validation_test.go:180-200"}]}


# -------------------------------------------------------------- Kafka KATs --
def kafka_kats() -> dict:
    """pkg/kafka/policy_test.go:52-127 and pkg/proxy/kafka_test.go:184-258."""
    produce = {"api_key": 0, "api_version": 0, "kind": 1, "client_id": "test", "topics": ["foo", "bar"]}
    cases = [
        ([], produce, 0, 86), ([{}], produce, 1, 89), ([{"topic": "foo"}], produce, 0, 91),
        ([{"topic": "foo"}, {"topic": "bar"}], produce, 1, 94), ([{"topic": "foo"}, {"topic": "baz"}], produce, 0, 97),
        ([{"topic": "baz"}, {"topic": "foo2"}], produce, 0, 100), ([{"topic": "bar"}, {"topic": "foo"}], produce, 1, 103),
        ([{"topic": "bar"}, {"topic": "foo"}, {"topic": "baz"}], produce, 1, 107),
    ]
    apiv = {"api_key": 18, "api_version": 0, "kind": 0, "client_id": "", "topics": []}
    r12 = [{"apiKey": "metadata"}, {"apiKey": "apiversions"}]
    cases += [([], apiv, 0, 116), (r12, apiv, 1, 123),
              (r12, {"api_key": 19, "api_version": 0, "kind": 0, "client_id": "", "topics": []}, 0, 126)]
    out = [{"rules": r, "request": q, "expect": e, "source": f"pkg/kafka/policy_test.go:{ln}"} for r, q, e, ln in cases]
    proxy_rules = [{"apiKey": "metadata", "apiVersion": "0"},
                   {"apiKey": "produce", "apiVersion": "0", "topic": "allowedTopic"}]
    out += [
        {"rules": proxy_rules, "request": {"api_key": 0, "api_version": 0, "kind": 1, "client_id": "tester",
                                           "topics": ["allowedTopic"]}, "expect": 1,
         "source": "pkg/proxy/kafka_test.go:246-249"},
        {"rules": proxy_rules, "request": {"api_key": 0, "api_version": 0, "kind": 1, "client_id": "tester",
                                           "topics": ["disallowedTopic"]}, "expect": 0,
         "source": "pkg/proxy/kafka_test.go:251-253"},
        {"rules": proxy_rules, "request": {"api_key": 3, "api_version": 0, "kind": 1, "client_id": "tester",
                                           "topics": ["allowedTopic"]}, "expect": 1,
         "source": "pkg/proxy/kafka_test.go:184-196 (metadata v0 by the client)"},
    ]
    sanitize = [({"role": "produce", "apiKey": "produce"}, False), ({"apiKey": "Metadata"}, True),
                ({"apiKey": "nosuchkey"}, False), ({"role": "CONSUME"}, True), ({"role": "admin"}, False),
                ({"apiVersion": "70000"}, False), ({"apiVersion": "-1"}, True), ({"apiVersion": "1.0"}, False),
                ({"topic": "a" * 256}, False), ({"topic": "a" * 255}, True), ({"topic": "bad topic"}, False),
                ({"topic": "ok.topic_name-1"}, True), ({"topic": "back\\slash"}, True)]
    return {"matches_rule": out, "sanitize": [{"rule": r, "valid": v,
                                               "source": "pkg/policy/api/rule_validation.go:232-275"}
                                              for r, v in sanitize]}


# ---------------------------------------------------------------- LPM KATs --
def kafka_wire_kats() -> dict:
    """Wire bytes of the requests pkg/proxy/kafka_test.go:184-258 sends
    through the proxy (optiopay client: broker.go:296 metadata with the
    broker's clientID, broker.go:818 ProduceReq with NewProducerConf's
    RequiredAcks -1 / 5 s timeout, messages "first" and "second"), encoded
    per the vendored proto encoders (cilium_amd.kafka_requests), with the
    verdicts that test asserts and the decode ReadRequest yields; plus the
    ReadReq / ReadRequest error cases (messages.go:131, request.go:195-198)."""
    from cilium_amd import kafka_requests as K
    rules = [{"apiKey": "metadata", "apiVersion": "0"},
             {"apiKey": "produce", "apiVersion": "0", "topic": "allowedTopic"}]
    msgs = [(None, b"first"), (None, b"second")]

    def prod(topic):
        return K.produce(0, b"tester", [(topic, [(0, msgs)])], acks=-1, timeout_ms=5000)
    cases = [
        ("pkg/proxy/kafka_test.go:215 (Dial: metadata, all topics)", K.metadata(0, b"tester", None), 1,
         [3, 0, "typed", "tester", []]),
        ("pkg/proxy/kafka_test.go:246 (leader lookup: metadata for allowedTopic)",
         K.metadata(0, b"tester", [b"allowedTopic"]), 1, [3, 0, "typed", "tester", ["allowedTopic"]]),
        ("pkg/proxy/kafka_test.go:246-249", prod(b"allowedTopic"), 1, [0, 0, "typed", "tester", ["allowedTopic"]]),
        ("pkg/proxy/kafka_test.go:251-253", prod(b"disallowedTopic"), 0,
         [0, 0, "typed", "tester", ["disallowedTopic"]]),
        ("pkg/kafka/request.go:195-198 (length < 12)", bytes([0, 0, 0, 6, 0, 3, 0, 0, 0, 1]), 2, None),
        ("vendor/github.com/optiopay/kafka/proto/messages.go:131 (size <= 0)", bytes([0, 0, 0, 0, 0, 3]), 2, None),
        ("vendor/github.com/optiopay/kafka/proto/messages.go:141-147 (size > maxParseBufSize)",
         bytes([0, 0x64, 0, 0, 0, 3]) + bytes(8), 2, None),
    ]
    return {"rules": rules, "cases": [{"source": src, "hex": raw.hex(), "expect": v, "decoded": d}
                                      for src, raw, v, d in cases]}


def lpm_kats() -> dict:
    """test/bpf/unit-test.c:77-102 (prefix p/len covers a iff a & mask == p)."""
    c = [("255.255.255.255/32", "255.255.255.255", 1), ("255.255.255.255/32", "255.240.0.0", 0),
         ("255.255.255.254/31", "255.255.255.254", 1), ("255.255.255.254/31", "255.255.255.255", 1),
         ("255.255.255.254/31", "255.240.0.0", 0), ("255.255.252.0/22", "255.255.252.0", 1),
         ("255.255.252.0/22", "255.255.255.255", 1), ("255.255.252.0/22", "255.240.0.0", 0),
         ("255.224.0.0/11", "255.224.0.0", 1), ("255.224.0.0/11", "255.255.255.255", 1),
         ("255.224.0.0/11", "255.240.0.0", 1), ("240.0.0.0/11", "240.0.0.0", 1), ("0.0.0.0/0", "0.0.0.0", 1),
         ("0.0.0.0/0", "255.255.255.255", 1)]
    return {"covers": [{"prefix": p, "addr": a, "covered": v, "source": "test/bpf/unit-test.c:77-102"}
                       for p, a, v in c]}


# ------------------------------------------------------------ regex vectors --
def regex_vectors(seed: int = 7, n_patterns: int = 160, n_strings: int = 24) -> dict:
    """Random patterns from the supported subset over printable ASCII, with
    std::regex_match results from the oracle, cross-checked with Python re."""
    import oracle
    rng = random.Random(seed)
    atoms = ["a", "b", "c", "/", ".", "[a-c]", "[^a]", "\\d", "\\w", "x", "(a|b)", "(?:ab|c)", "[0-9]", "\\."]
    quants = ["", "", "", "*", "+", "?", "{1,2}", "{2}"]
    pats = []
    for _ in range(n_patterns):
        k = rng.randint(1, 5)
        p = "".join(rng.choice(atoms) + rng.choice(quants) for _ in range(k))
        if rng.random() < 0.2:
            p = p + "|" + rng.choice(atoms)
        if rng.random() < 0.15:
            p = "^" + p + "$"
        pats.append(p)
    alpha = "abcx/.1 9_-A"
    out = []
    for p in pats:
        strs = ["".join(rng.choice(alpha) for _ in range(rng.randint(0, 7))) for _ in range(n_strings)]
        res = []
        for s in strs:
            o = oracle.regex_match(p.encode(), s.encode())
            py = 1 if re.fullmatch(p, s) else 0
            if o != py:
                raise SystemExit(f"oracle and Python re disagree on {p!r} {s!r}: {o} vs {py}")
            res.append(o)
        out.append({"pattern": p, "strings": strs, "full_match": res})
    return {"generator": "tests/golden/make_golden.py regex_vectors(seed=7)", "cases": out}


def _r2d2_policy(name: str, rule: str) -> str:
    """The protobuf-text policy shape of r2d2parser_test.go (one ingress port 80
    rule; `rule` is the l7_rules body, "" for the allow-all rule)."""
    l7 = ("\n    l7_rules: <\n      l7_rules: <\n" + rule + "      >\n    >") if rule else ""
    return (f'name: "{name}"\npolicy: 2\ningress_per_port_policies: <\n  port: 80\n  rules: <\n'
            f'    l7_proto: "r2d2"{l7}\n  >\n>\n')


def _cassandra_policy(name: str, key: str, value: str) -> str:
    """cassandraparser_test.go's shape: remotes 1, 3, 4 and one l7 rule."""
    return (f'name: "{name}"\npolicy: 2\ningress_per_port_policies: <\n  port: 80\n  rules: <\n'
            '    remote_policies: 1\n    remote_policies: 3\n    remote_policies: 4\n'
            '    l7_proto: "cassandra"\n    l7_rules: <\n      l7_rules: <\n'
            f'        rule: <\n          key: "{key}"\n          value: "{value}"\n        >\n'
            '      >\n    >\n  >\n>\n')


def proxylib_kats() -> dict:
    """proxylib policies in NPDS protobuf text (as the reference's tests insert
    them) with the verdicts those tests assert, per request frame."""
    r2d2 = [
        {"src": "proxylib/r2d2/r2d2parser_test.go:70-95 TestR2d2OnDataBasicPass",
         "policy": _r2d2_policy("cp1", ""),
         "requests": [["READ sssss", True], ["WRITE sssss", True], ["HALT", True], ["RESET", True]]},
        {"src": "proxylib/r2d2/r2d2parser_test.go:119-146 TestR2d2OnDataAllowDenyCmd",
         "policy": _r2d2_policy("cp2", '        rule: <\n          key: "cmd"\n          value: "READ"\n        >\n'),
         "requests": [["READ xssss", True], ["WRITE xssss", False]]},
        {"src": "proxylib/r2d2/r2d2parser_test.go:148-176 TestR2d2OnDataAllowDenyRegex",
         "policy": _r2d2_policy("cp3", '        rule: <\n          key: "file"\n          value: "s.*"\n        >\n'),
         "requests": [["READ ssss", True], ["WRITE yyyyy", False]]},
    ]
    cass = [
        {"src": "proxylib/cassandra/cassandraparser_test.go:86-115 TestCassandraOnDataOptionsReq (OPTIONS frame)",
         "policy": _cassandra_policy("cp6", "query_action", "select"), "requests": [["/options", True]]},
        {"src": "proxylib/cassandra/cassandraparser_test.go:145-172 TestCassandraOnDataQueryReq "
                "(SELECT ... FROM system.local)",
         "policy": _cassandra_policy("cp4", "query_table", ".*"),
         "requests": [["/query/select/system.local", True]]},
        {"src": "proxylib/cassandra/cassandraparser_test.go:236-280 TestSimpleCassandraPolicy",
         "policy": _cassandra_policy("cp1", "query_table", "no-match"),
         "requests": [["/options", True], ["/query/select/system.local", False]]},
    ]
    return {"generator": "tests/golden/make_golden.py proxylib_kats()", "remote": 1, "port": 80,
            "r2d2": r2d2, "cassandra": cass}


def main():
    files = {"proxylib_kat.json": proxylib_kats(), "http_kat.json": http_kats(), "translation_kat.json": translation_kats(),
             "kafka_kat.json": kafka_kats(), "kafka_wire_kat.json": kafka_wire_kats(), "lpm_kat.json": lpm_kats(), "regex_vectors.json": regex_vectors()}
    for name, data in files.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, indent=1, sort_keys=False)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
