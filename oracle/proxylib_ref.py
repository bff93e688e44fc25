"""CPU restatement of proxylib's generic-L7 policy evaluation with the r2d2
rule parser.  TEST INFRASTRUCTURE ONLY (checker for tests/ and smoke()); it
shares no code with cilium_amd and evaluates rules directly, rule by rule,
the way the Go code does:

  PolicyInstance.Matches         proxylib/proxylib/policymap.go:254-260
  PortNetworkPolicies.Matches    :208-236 (exact port, port 0, else false)
  newPortNetworkPolicies         :177-206 (UDP skipped, duplicate port error)
  PortNetworkPolicyRules.Matches :150-171 (!HaveL7Rules → true)
  newPortNetworkPolicyRules      :118-148 (unknown parser → port dropped)
  PortNetworkPolicyRule.Matches  :91-111  (remote set, OR over L7 rules)
  r2d2Rule.Matches / ruleParser  proxylib/r2d2/r2d2parser.go:61-123
  CassandraRule.Matches / parser proxylib/cassandra/cassandraparser.go:40-131

Go ``regexp.MustCompile`` + ``MatchString`` is oracle/go_regexp_ref.py
(Go 1.10 regexp/syntax restated; inputs stepped as utf8.DecodeRune steps,
an invalid byte being one U+FFFD).  Rule strings arrive as JSON text (Go
strings: UTF-8); request fields as bytes, passed here latin-1 decoded.
Pure-Python loops, so it is sized for small cases.
"""
from __future__ import annotations

from .go_regexp_ref import GoRegexp, GoSyntaxError


class ParseError(ValueError):
    pass


class _GoSearch:
    """regexp.MustCompile(pattern) (a syntax error panics: ParseError);
    search(s) = MatchString on the bytes s holds (latin-1 decoded)."""

    def __init__(self, pattern: str):
        try:
            self.re = GoRegexp(pattern.encode("utf-8", "surrogateescape"))
        except GoSyntaxError as e:
            raise ParseError("regexp: " + str(e)) from e

    def search(self, s: str) -> bool:
        return self.re.match_string(s.encode("latin-1"))


def go_regexp(pattern: str) -> _GoSearch:
    return _GoSearch(pattern)


def _b(s: str) -> str:
    """A rule string (UTF-8 in Go) as the latin-1 text of its bytes, so it
    compares byte for byte with request fields."""
    return s.encode("utf-8", "surrogateescape").decode("latin-1")


class _R2d2Rule:
    def __init__(self, rule: dict):
        self.cmd, self.file_re = "", None
        for k, v in rule.items():
            if k == "cmd":
                self.cmd = _b(v)
            elif k == "file":
                if v != "":
                    self.file_re = go_regexp(v)
            else:
                raise ParseError("Unsupported key: " + k)
        if self.cmd not in ("", "READ", "WRITE", "HALT", "RESET"):
            raise ParseError("invalid cmd")
        if self.file_re is not None and self.cmd not in ("", "READ", "WRITE"):
            raise ParseError("cmd not compatible with file")

    def matches(self, cmd: str, file: str) -> bool:
        if self.cmd and self.cmd != cmd:
            return False
        if self.file_re is not None and not self.file_re.search(file):
            return False
        return True


_CASS_NO_TABLE = {"drop-index", "create-index", "create-materialized-view", "drop-materialized-view",
                  "create-role", "alter-role", "drop-role", "grant-role", "revoke-role", "list-roles",
                  "grant-permission", "revoke-permission", "list-permissions", "create-user", "alter-user",
                  "drop-user", "list-users", "create-function", "drop-function", "create-aggregate",
                  "drop-aggregate", "create-type", "alter-type", "drop-type", "create-trigger", "drop-trigger"}
_CASS_TABLE = {"select", "delete", "insert", "update", "create-table", "drop-table", "alter-table",
               "truncate-table", "use", "create-keyspace", "alter-keyspace", "drop-keyspace"}


class _CassandraRule:
    """CassandraRule (proxylib/cassandra/cassandraparser.go:40-131); the
    request is the path string its OnData builds."""

    def __init__(self, rule: dict):
        self.action, self.table_re = "", None
        for k, v in rule.items():
            if k == "query_action":
                self.action = _b(v)
            elif k == "query_table":
                if v != "":
                    self.table_re = go_regexp(v)
            else:
                raise ParseError("Unsupported key: " + k)
        if self.action:
            if self.action not in _CASS_TABLE and self.action not in _CASS_NO_TABLE:
                raise ParseError("invalid query_action")
            if self.action in _CASS_NO_TABLE and self.table_re is not None:
                raise ParseError("not compatible with a query_table match")

    def matches(self, path: str, _unused: str = "") -> bool:
        parts = path.split("/")
        if len(parts) <= 2:
            return True
        if len(parts) < 4:
            return False
        if self.action and self.action != parts[2]:
            return False
        if len(parts[3]) > 0 and self.table_re is not None and not self.table_re.search(parts[3]):
            return False
        return True


_PARSERS = {"r2d2": lambda l7: [_R2d2Rule(x.get("rule") or {}) for x in l7],
            "cassandra": lambda l7: [_CassandraRule(x.get("rule") or {}) for x in l7]}


class _Rules:
    def __init__(self, rules_cfg: list):
        self.rules, self.have_l7, self.ok = [], False, True
        first = ""
        for r in rules_cfg:
            proto = r.get("l7_proto", "")
            if proto and proto not in _PARSERS:
                self.ok = False
                return
            if proto:
                if not first:
                    first = proto
                elif proto != first:
                    raise ParseError("Mismatching L7 types on the same port")
            l7 = _PARSERS[proto]((r.get("l7_rules") or {}).get("l7_rules") or []) if proto else []
            if l7:
                self.have_l7 = True
            self.rules.append((set(int(x) for x in r.get("remote_policies") or []), l7))

    def matches(self, remote: int, cmd: str, file: str) -> bool:
        if not self.have_l7 or not self.rules:
            return True
        for remotes, l7 in self.rules:
            if remotes and remote not in remotes:
                continue
            if not l7 or any(x.matches(cmd, file) for x in l7):
                return True
        return False


class _Ports:
    def __init__(self, cfg: list):
        self.by_port = {}
        for pp in cfg or []:
            proto = pp.get("protocol", "TCP")
            if proto in ("UDP", 1):
                continue
            port = int(pp.get("port", 0))
            if port in self.by_port:
                raise ParseError("Duplicate port number")
            if proto not in ("TCP", 0):
                raise ParseError("Invalid transport protocol")
            r = _Rules(pp.get("rules") or [])
            if r.ok:
                self.by_port[port] = r

    def matches(self, port: int, remote: int, cmd: str, file: str) -> bool:
        r = self.by_port.get(port)
        if r is not None and r.matches(remote, cmd, file):
            return True
        w = self.by_port.get(0)
        if w is not None and w.matches(remote, cmd, file):
            return True
        return False


class ProxylibOracle:
    def __init__(self, policies: list[dict]):
        self.pol = {}
        for p in policies:
            self.pol[p["name"]] = (_Ports(p.get("ingress_per_port_policies")),
                                   _Ports(p.get("egress_per_port_policies")))

    def matches_path(self, name: str, ingress: bool, port: int, remote: int, path: bytes) -> bool:
        """cassandra: the request is its path ("/opcode/action/table")."""
        p = self.pol.get(name)
        if p is None:
            return False
        return (p[0] if ingress else p[1]).matches(port, remote, path.decode("latin-1"), "")

    def matches(self, name: str, ingress: bool, port: int, remote: int, cmd: bytes, file: bytes) -> bool:
        p = self.pol.get(name)
        if p is None:
            return False
        return (p[0] if ingress else p[1]).matches(port, remote, cmd.decode("latin-1"), file.decode("latin-1"))
