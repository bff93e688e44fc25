"""proxylib generic-L7 policy on the verdict engine.

Mirrors the reference's proxylib policy layer:

* ``RegisterL7RuleParser`` / the per-parser rule parsers
  (proxylib/proxylib/policymap.go:28-45) — here a parser translates one NPDS
  ``PortNetworkPolicyRule`` with ``l7_proto`` and ``l7_rules`` into header
  matchers of the engine's HTTP union-DFA compiler;
* ``newPortNetworkPolicies`` / ``newPortNetworkPolicyRules``
  (policymap.go:118-206): UDP ports skipped, a duplicate port or a transport
  other than TCP is a ParseError, a rule whose L7 parser is unknown drops the
  whole port (the port is not installed), mismatching L7 types on one port
  are a ParseError;
* the verdict contract ``PolicyInstance.Matches`` (policymap.go:254-260,
  :208-236): exact port, then port 0, and **no policy for the port → deny**
  (the engine's ``"proxylib": true`` policy flag; Envoy would allow).

The cassandra parser (proxylib/cassandra/cassandraparser.go:58-131) works on
the request path "/opcode/action/table"; each rule becomes an OR of engine
rules over the path's shape, action and table (see cassandra_rule_parser).

The r2d2 parser (proxylib/r2d2/r2d2parser.go:61-123): a rule is an AND of
``cmd`` exact equality (if non-empty) and an **unanchored** Go
``regexp.MatchString`` on ``file`` (if non-empty), compiled by the engine in
its search mode (``regex_search`` matcher).  A request is ``{cmd, file}`` as
r2d2's OnData splits it (file is "" unless the line has exactly two fields).

Verdicts run in the HIP ``http_kernel``: no CPU path.  Field bytes must be
printable ASCII (0x21-0x7E: r2d2 splits on spaces) — the subset where Go
RE2, ECMAScript and the engine agree; the packer flags control bytes as
malformed, so such a request is denied (documented divergence).
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import numpy as np

from . import _native as N


class ParseError(ValueError):
    """proxylib.ParseError (policymap.go): the policy update is rejected."""


# L7 rule parsers: name -> f(l7_rules list of {"rule": {k: v}}) -> list of matcher lists
_L7_RULE_PARSERS: dict[str, Callable[[list], list[list[dict]]]] = {}


def register_l7_rule_parser(name: str, fn: Callable[[list], list[list[dict]]]) -> None:
    """RegisterL7RuleParser (policymap.go:42-45)."""
    _L7_RULE_PARSERS[name] = fn


R2D2_CMDS = ("READ", "WRITE", "HALT", "RESET")


def r2d2_rule_parser(l7_rules: list) -> list[list[dict]]:
    """ruleParser (r2d2parser.go:91-123): each L7 rule → an AND of matchers."""
    out = []
    for l7 in l7_rules:
        rule = l7.get("rule") or {}
        cmd, file_re = "", None
        for k, v in rule.items():
            if k == "cmd":
                cmd = v
            elif k == "file":
                if v != "":
                    file_re = v
            else:
                raise ParseError(f"Unsupported key: {k}")
        if cmd and cmd not in R2D2_CMDS:
            raise ParseError(f"Unable to parse L7 r2d2 rule with invalid cmd: '{cmd}'")
        if file_re is not None and cmd not in ("", "READ", "WRITE"):
            raise ParseError(f"Unable to parse L7 r2d2 rule, cmd '{cmd}' is not compatible with 'file'")
        ms = []
        if cmd:
            ms.append({"name": "cmd", "exact_match": cmd})
        if file_re is not None:
            ms.append({"name": "file", "regex_search": file_re})
        out.append(ms)
    return out


register_l7_rule_parser("r2d2", r2d2_rule_parser)

# queryActionMap (proxylib/cassandra/cassandraparser.go:315-366): 1 = takes a
# table (query_table allowed), 2 = no table
CASSANDRA_ACTIONS = dict(
    [(a, 1) for a in ("select", "delete", "insert", "update", "create-table", "drop-table", "alter-table",
                      "truncate-table", "use", "create-keyspace", "alter-keyspace", "drop-keyspace")] +
    [(a, 2) for a in ("drop-index", "create-index", "create-materialized-view", "drop-materialized-view",
                      "create-role", "alter-role", "drop-role", "grant-role", "revoke-role", "list-roles",
                      "grant-permission", "revoke-permission", "list-permissions", "create-user", "alter-user",
                      "drop-user", "list-users", "create-function", "drop-function", "create-aggregate",
                      "drop-aggregate", "create-type", "alter-type", "drop-type", "create-trigger",
                      "drop-trigger")])


def cassandra_rule_parser(l7_rules: list) -> list[list[dict]]:
    """CassandraRuleParser (cassandraparser.go:97-131).  A rule's Matches
    (:58-90) is an OR of request shapes, split into engine rules (the L7
    rules of a PNPR are OR-ed): a path of <= 2 parts matches any rule; one of
    >= 4 parts needs the action and, if the table part is non-empty, the
    unanchored table regex; a 3-part path matches none."""
    out = []
    for l7 in l7_rules:
        rule = l7.get("rule") or {}
        action, table_re = "", None
        for k, v in rule.items():
            if k == "query_action":
                action = v
            elif k == "query_table":
                if v != "":
                    table_re = v
            else:
                raise ParseError(f"Unsupported key: {k}")
        if action:
            kind = CASSANDRA_ACTIONS.get(action, 0)
            if kind == 0:
                raise ParseError(f"Unable to parse L7 cassandra rule with invalid query_action: '{action}'")
            if kind == 2 and table_re is not None:
                raise ParseError(f"query_action '{action}' is not compatible with a query_table match")
        out.append([{"name": "cshape", "exact_match": "S"}])
        long = [{"name": "cshape", "exact_match": "L"}]
        if action:
            long.append({"name": "action", "exact_match": action})
        if table_re is None:
            out.append(long)
        else:
            out.append(long + [{"name": "table", "exact_match": ""}])
            out.append(long + [{"name": "table", "regex_search": table_re}])
    return out


register_l7_rule_parser("cassandra", cassandra_rule_parser)

# MemcacheOpCodeMap (proxylib/memcached/parser.go:212-474): rule command →
# (text commands, binary opcodes)
_MC_STORE = ("add", "set", "replace", "append", "prepend", "cas", "incr", "decr")
MEMCACHE_COMMANDS: dict[str, tuple[tuple[str, ...], tuple[int, ...]]] = {
    "add": (("add",), (2, 18)), "set": (("set",), (1, 17)), "replace": (("replace",), (3, 19)),
    "append": (("append",), (14, 25)), "prepend": (("prepend",), (15, 26)), "cas": (("cas",), ()),
    "incr": (("incr",), (5, 21)), "decr": (("decr",), (6, 22)),
    "storage": (_MC_STORE, (1, 2, 3, 5, 6, 17, 18, 19, 21, 22, 25, 26)),
    "get": (("get", "gets"), (0, 9, 12, 13)), "delete": (("delete",), (4, 20)), "touch": (("touch",), (28,)),
    "gat": (("gat", "gats"), (29, 30)),
    "writeGroup": (_MC_STORE + ("delete", "touch"), (1, 2, 3, 4, 5, 6, 17, 18, 19, 20, 21, 22, 25, 26, 28)),
    "slabs": (("slabs",), ()), "lru": (("lru",), ()), "lru_crawler": (("lru_crawler",), ()),
    "watch": (("watch",), ()), "stats": (("stats",), (16,)), "flush_all": (("flush_all",), (8, 24)),
    "cache_memlimit": (("cache_memlimit",), ()), "version": (("version",), (11,)),
    "misbehave": (("misbehave",), ()), "quit": (("quit",), (7, 23)), "noop": ((), (10,)),
    "verbosity": ((), (27,)), "sasl-list-mechs": ((), (32,)), "sasl-auth": ((), (33,)), "sasl-step": ((), (34,)),
}
MEMCACHE_COMMANDS.update({n: ((), (48 + i,)) for i, n in enumerate(
    ("rget", "rset", "rsetq", "rappend", "rappendq", "rprepend", "rprependq", "rdelete", "rdeleteq", "rincr",
     "rincrq", "rdecr", "rdecrq", "set-vbucket", "get-vbucket", "del-vbucket", "tap-connect", "tap-mutation",
     "tap-delete", "tap-flush", "tap-opaque", "tap-vbucket-set", "tap-checkpoint-start", "tap-checkpoint-end"))})


def memcache_rule_parser(l7_rules: list) -> list[list[dict]]:
    """L7RuleParser (proxylib/memcached/parser.go:114-148).  Rule.Matches
    (:46-100) is the command (a text command or binary opcode in the rule's
    set) AND, for the first non-empty of keyExact / keyPrefix / keyRegex, a
    test that EVERY key of the request passes.  A request is packed as the
    fields ``mccmd`` ("t" + command, or "b" + two hex digits of the opcode)
    and ``mckeys`` (each key, escaped, then the separator pair 0x03 0x14), so
    the key test is a list matcher over the separated keys; one engine rule
    per allowed command token.  No command: an empty rule (matches
    everything) unless a key is given, which is a ParseError."""
    out = []
    for l7 in l7_rules:
        rule = l7.get("rule") or {}
        cmds, exact, prefix, regex = None, "", "", None
        for k, v in rule.items():
            if k == "command":
                cmds = MEMCACHE_COMMANDS.get(v)
            elif k == "keyExact":
                exact = v
            elif k == "keyPrefix":
                prefix = v
            elif k == "keyRegex":
                regex = v
            else:
                raise ParseError(f"Unsupported key: {k}")
        if cmds is None:
            if exact or prefix or regex is not None:
                raise ParseError("command not specified but key was provided")
            out.append([])
            continue
        key = ([{"name": "mckeys", "list_exact": exact}] if exact else
               [{"name": "mckeys", "list_prefix": prefix}] if prefix else
               [{"name": "mckeys", "list_search": regex}] if regex is not None else [])
        toks = ["t" + t for t in cmds[0]] + ["b%02x" % b for b in cmds[1]]
        out.extend([{"name": "mccmd", "exact_match": t}] + key for t in toks)
    return out


register_l7_rule_parser("memcache", memcache_rule_parser)


def memcache_request(command: bytes, opcode: int, keys: Sequence[bytes]) -> list[tuple[bytes, bytes]]:
    """A memcache request's fields (MemcacheMeta, memcached/meta/meta.go):
    a text command (``command`` non-empty) or a binary opcode, and its keys.
    The separators are appended after escaping (pack_fields escapes values),
    so they are passed pre-escaped via the raw form of ``mckeys``."""
    cmd = b"t" + command if command else b"b%02x" % opcode
    return [(b"mccmd", cmd), (b"mckeys", _RawField(b"".join(escape_value(k) + b"\x03\x14" for k in keys)))]


class _RawField(bytes):
    """A field value already in the engine's escaped form."""


def _translate_port(pp: dict) -> Optional[dict]:
    """newPortNetworkPolicyRules (policymap.go:118-148) for one port; None =
    the port is not installed (a rule with an unknown parser)."""
    rules_out = []
    first_type = ""
    for r in pp.get("rules") or []:
        l7_proto = r.get("l7_proto", "")
        l7 = (r.get("l7_rules") or {}).get("l7_rules") or []
        if l7_proto and l7_proto not in _L7_RULE_PARSERS:
            return None  # newPortNetworkPolicyRule !ok → port skipped (:186-204)
        if l7_proto:
            if first_type == "":
                first_type = l7_proto
            elif l7_proto != first_type:
                raise ParseError("Mismatching L7 types on the same port")
        ms = _L7_RULE_PARSERS[l7_proto](l7) if l7_proto else []
        out = {}
        if r.get("remote_policies"):
            out["remote_policies"] = [int(x) for x in r["remote_policies"]]
        # a rule contributes L7 rules only when its parser produced some
        # (HaveL7Rules, :132-134); otherwise it matches any payload
        if ms:
            out["http_rules"] = {"http_rules": [{"headers": m} for m in ms]}
        rules_out.append(out)
    return {"port": int(pp.get("port", 0)), "protocol": "TCP", "rules": rules_out}


def translate_policies(policies: Sequence[dict]) -> list[dict]:
    """NPDS NetworkPolicy dicts with proxylib L7 rules → the engine's NPDS form
    (newPolicyInstance / newPortNetworkPolicies, policymap.go:177-252)."""
    out = []
    for p in policies:
        q = {"name": p["name"], "proxylib": True}
        if "policy" in p:
            q["policy"] = p["policy"]
        for key in ("ingress_per_port_policies", "egress_per_port_policies"):
            ports, seen = [], set()
            for pp in p.get(key) or []:
                proto = pp.get("protocol", "TCP")
                if proto in ("UDP", 1):
                    continue
                port = int(pp.get("port", 0))
                if port in seen:
                    raise ParseError(f"Duplicate port number {port}")
                seen.add(port)
                if proto not in ("TCP", 0):
                    raise ParseError(f"Invalid transport protocol {proto}")
                t = _translate_port(pp)
                if t is not None:
                    ports.append(t)
            q[key] = ports
        out.append(q)
    return out


def cassandra_request(path: bytes) -> list[tuple[bytes, bytes]]:
    """The fields of a cassandra request path ("/opcode[/action/table]",
    cassandraparser.go:486-578) as CassandraRule.Matches splits it (:73-89)."""
    parts = path.split(b"/")
    if len(parts) <= 2:
        return [(b"cshape", b"S")]
    if len(parts) < 4:
        return [(b"cshape", b"X")]
    return [(b"cshape", b"L"), (b"action", parts[2]), (b"table", parts[3])]


# NPDS protobuf text format (the form the reference's proxylib tests insert
# policies in, CheckInsertPolicyText): repeated fields of
# envoy/cilium/npds.proto:31-182 become lists, the L7 rule map entries
# ("rule: < key: .. value: .. >") a dict.
_REPEATED = {"ingress_per_port_policies", "egress_per_port_policies", "rules", "remote_policies", "l7_rules",
             "http_rules", "headers", "kafka_rules"}
_TOKEN_RE = None


def parse_policy_text(text: str) -> dict:
    """One NetworkPolicy in protobuf text format → the dict form used here."""
    import re
    global _TOKEN_RE
    if _TOKEN_RE is None:
        _TOKEN_RE = re.compile(r'\s*(?:(#[^\n]*)|([A-Za-z_][A-Za-z0-9_]*)|("(?:[^"\\]|\\.)*")|'
                               r"('(?:[^'\\]|\\.)*')|(-?[0-9]+)|([:<>{}]))")
    toks, pos = [], 0
    while pos < len(text):
        m = _TOKEN_RE.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise ParseError(f"bad policy text at {pos}")
        pos = m.end()
        if m.group(1):
            continue
        toks.append(next(g for g in m.groups()[1:] if g is not None))
    i = 0

    def value(tok):
        if tok[0] in "\"'":
            return bytes(tok[1:-1], "utf-8").decode("unicode_escape")
        if tok.lstrip("-").isdigit():
            return int(tok)
        return {"true": True, "false": False}.get(tok, tok)

    def message(end):
        nonlocal i
        out: dict = {}
        while i < len(toks) and toks[i] != end:
            name = toks[i]
            i += 1
            if toks[i] == ":":
                i += 1
            if toks[i] in ("<", "{"):
                close = ">" if toks[i] == "<" else "}"
                i += 1
                v = message(close)
                i += 1
                if name == "rule" and set(v) <= {"key", "value"}:  # map<string,string> entry
                    out.setdefault("rule", {})[v.get("key", "")] = v.get("value", "")
                    continue
            else:
                v = value(toks[i])
                i += 1
            if name in _REPEATED:
                out.setdefault(name, []).append(v)
            else:
                out[name] = v
        return out

    pol = message(None)
    # l7_rules is a message holding a repeated l7_rules: lift the inner list
    for key in ("ingress_per_port_policies", "egress_per_port_policies"):
        for pp in pol.get(key, []):
            for r in pp.get("rules", []):
                if "l7_rules" in r:
                    inner = [x for wrapper in r["l7_rules"] for x in wrapper.get("l7_rules", [])]
                    r["l7_rules"] = {"l7_rules": inner}
    return pol


def r2d2_request(line: bytes) -> tuple[bytes, bytes]:
    """r2d2 OnData request split (r2d2parser.go:157-167): cmd, and the file
    only when the line has exactly two space-separated fields."""
    fields = line.split(b" ")
    return fields[0], (fields[1] if len(fields) == 2 else b"")


def escape_value(v: bytes) -> bytes:
    """A proxylib field value in the engine's escaped form: bytes 0x00-0x03
    become 0x03, 0x10 + b (regex.h kEscByte), so values may hold any byte
    (a NUL inside an r2d2 cmd or file stays part of the string the rules
    compare, r2d2parser.go:157-183)."""
    if not any(b <= 3 for b in v):
        return v
    return b"".join(bytes([3, 0x10 + b]) if b <= 3 else bytes([b]) for b in v)


class ProxylibPolicy:
    """A proxylib policy snapshot on a Classifier: ``update`` then batched
    ``matches`` for r2d2 requests (Instance.PolicyMatches, instance.go:157-165)."""

    def __init__(self, cl):
        self.cl = cl
        self.names: list[str] = []

    def update(self, policies: Sequence[dict]) -> None:
        eng = translate_policies(policies)
        self.cl.update_http_policy(eng)
        self.names = [p["name"] for p in eng]

    def index(self, name: str) -> int:
        try:
            return self.cl.http_policy_index(name)
        except N.CiliumGPUError:
            return 0xFFFFFFFF  # unknown policy → deny

    def pack_fields(self, policy, ingress, port, remote, fields: Sequence[Sequence[tuple[bytes, bytes]]]):
        """Requests given as their parser's (name, value) fields."""
        parts, off = [], [0]
        for fs in fields:
            b = b"".join(k + b"\0" + (v if isinstance(v, _RawField) else escape_value(v)) + b"\0" for k, v in fs)
            parts.append(b)
            off.append(off[-1] + len(b))
        blob = np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy()
        return self.cl.pack_http(np.asarray(policy, np.uint32), np.asarray(ingress, np.uint8),
                                 np.asarray(port, np.uint16), np.asarray(remote, np.uint32), blob,
                                 np.asarray(off, np.uint64))

    def pack(self, policy, ingress, port, remote, cmds: Sequence[bytes], files: Sequence[bytes]):
        """r2d2 requests: {cmd, file}."""
        return self.pack_fields(policy, ingress, port, remote,
                                [[(b"cmd", c), (b"file", f)] for c, f in zip(cmds, files)])

    def matches_fields(self, policy, ingress, port, remote, fields, host_diag: bool = False) -> np.ndarray:
        b = self.pack_fields(policy, ingress, port, remote, fields)
        return self.cl.http_eval_host_diag(b) if host_diag else self.cl.http_verdicts(b)

    def matches(self, policy, ingress, port, remote, cmds, files) -> np.ndarray:
        """One allow byte per request, from the GPU kernel."""
        return self.cl.http_verdicts(self.pack(policy, ingress, port, remote, cmds, files))

    def matches_host_diag(self, policy, ingress, port, remote, cmds, files) -> np.ndarray:
        """Table-compiler diagnostics only (CPU walk of the same tables)."""
        return self.cl.http_eval_host_diag(self.pack(policy, ingress, port, remote, cmds, files))
