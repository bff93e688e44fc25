"""proxylib Cassandra (proxylib/cassandra/) through the
proxylib C ABI: the reference's cassandraparser_test.go cases (transcribed as
data in tests/golden/cassandra_kat.json) and random frame streams against
oracle/cassandra_ref.py.  Framing, query parsing and prepared-statement
tracking run on the host (proxylib_cassandra.cc); every path's
PolicyMatches verdict comes from the GPU batch of its OnData call, so the ABI
tests with policies are GPU tests.  The oracle itself is pinned on the CPU
against the same fixtures, and the framing alone (a policy name that is not
installed: every request denied without a GPU batch) runs on the CPU."""
import json

import numpy as np
import pytest

from cilium_amd import _native as N
from cilium_amd import proxylib as P
from kat_util import load
from oracle import cassandra_ref as CR
from oracle.proxylib_ref import ProxylibOracle
from test_proxylib_abi import F_OK, Conn, _lib, open_module

KAT = load("cassandra_kat.json")


def _oracle_for(case):
    if case["policy"] is None:
        return lambda path: False
    pol = P.parse_policy_text(case["policy"])
    o = ProxylibOracle([pol])
    return lambda path: o.matches_path(pol["name"], True, KAT["port"], KAT["remote"], path)


def test_oracle_pinned_on_reference_cases():
    for case in KAT["cases"]:
        conn = CR.Connection(_oracle_for(case), KAT["buf_cap"])
        for c in case["calls"]:
            rc, ops = conn.on_data(c["reply"], [bytes.fromhex(x) for x in c["chunks"]], len(c["ops"]))
            assert rc == CR.F_OK and [list(o) for o in ops] == c["ops"], case["name"]
            assert bytes(conn.reply_buf) == bytes.fromhex(c["inject"]), case["name"]
            conn.reply_buf.clear()


def _q(conn, query: bytes):
    return conn._query(query)


def test_oracle_query_parsing():
    c = CR.Connection(lambda p: True)
    assert _q(c, b"SELECT a FROM Sys.Local WHERE k=1;;") == (b"select", b"sys.local")
    assert _q(c, b"select a from t") == (b"select", b".t")
    assert _q(c, b"USE 'Ks'") == (b"use", b"ks")
    assert _q(c, b"select a from t") == (b"select", b"ks.t")
    assert _q(c, b"insert into x (a) values (1)") == (b"insert", b"ks.x")
    assert _q(c, b"CREATE TABLE IF NOT EXISTS a.b (x int)") == (b"create-table", b"a.b")
    assert _q(c, b"drop keyspace if exists k2") == (b"drop-keyspace", b"ks.k2")
    assert _q(c, b"alter table if t") == (b"alter-table", b"ks.if")
    assert _q(c, b"create materialized view v as select") == (b"create-materialized-view", b"")
    assert _q(c, b"create custom index i on t(a)") == (b"create-index", b"")
    assert _q(c, b"select a from t -- x") == (b"", b"")
    assert _q(c, b"grant all on t") == (b"", b"")
    assert _q(c, b"select") == (b"", b"")
    with pytest.raises(CR._Panic):
        _q(c, b"select a from")
    # Go's Unicode rules (cassandraparser.go:373): NBSP / ideographic space
    # separate fields, U+0130 lowers to "i", the rest re-encoded after a change
    assert _q(c, "SELECT\u00a0a FROM\u3000ÜSERS".encode()) == (b"select", "ks.üsers".encode())
    assert _q(c, "UPDATE İ.T SET".encode()) == (b"update", b"i.t")
    assert _q(c, b"SELECT a FROM \xffX.\xc3\x9c") == (b"select", "\ufffdx.ü".encode())  # changed at 'S'
    assert _q(c, b"select a from \xffX.t") == (b"select", b"\xffx.t")  # \xff before the first change
    assert _q(c, b"select a from \xffx.t") == (b"select", b"\xffx.t")


# ---- random frame streams ------------------------------------------------
WORDS = [b"t", b"users", b"ks.t", b"system.local", b"Sys.Peers", b"a.b.c", b"'quoted'", b"x/y",
         "ÜSERS".encode(), "Ks.İtem".encode(), "ks.Σ\u00a0x".encode(), b"\xffKS.T", "ks.t\u3000".encode()]
QUERIES = [
    b"SELECT a FROM {t} WHERE k=1", b"select * from {t};", b"DELETE FROM {t} WHERE a=1", b"INSERT INTO {t} (a) VALUES (1)",
    b"UPDATE {t} SET a=1", b"USE {k}", b"use \"{k}\"", b"CREATE TABLE IF NOT EXISTS {t} (a int)", b"CREATE TABLE {t} (a int)",
    b"DROP TABLE IF EXISTS {t}", b"DROP TABLE {t}", b"CREATE KEYSPACE {k} WITH r", b"DROP KEYSPACE IF EXISTS {k}",
    b"ALTER TABLE {t} ADD x int", b"TRUNCATE {t}", b"truncate table {t}", b"CREATE INDEX ON {t}(a)",
    b"CREATE MATERIALIZED VIEW v AS SELECT", b"CREATE CUSTOM INDEX i ON {t}(a)", b"LIST ROLES", b"create role r",
    b"Select A From {t}\tWhere", b"CREATE TABLE IF {t}", "SELECT\u2003a FROM {t}".encode(),
    "UPDATE\u0085{t} SET".encode(),
]
BAD_QUERIES = [b"GRANT ALL ON {t}", b"select * from", b"select a from {t} -- c", b"select", b"insert {t}",
               b"drop table if exists"]
KEYSPACES = [b"ks", b"Sys", b"system", b"k2"]


def _frame(opcode: int, body: bytes, stream: int, version: int = 4, flags: int = 0) -> bytes:
    return bytes([version, flags]) + stream.to_bytes(2, "big") + bytes([opcode]) + len(body).to_bytes(4, "big") + body


def _query_body(rng, q: bytes) -> bytes:
    if rng.random() < 0.02:  # a query length past the frame
        return (len(q) + int(rng.integers(1, 40))).to_bytes(4, "big") + q
    return len(q).to_bytes(4, "big") + q + b"\x00\x01"


def _rand_query(rng) -> bytes:
    qs = BAD_QUERIES if rng.random() < 0.08 else QUERIES
    q = qs[int(rng.integers(len(qs)))]
    return q.replace(b"{t}", WORDS[int(rng.integers(len(WORDS)))]).replace(b"{k}", KEYSPACES[int(rng.integers(4))])


class _Stream:
    """Client frames for one connection; prepared ids the emulated server
    hands out are remembered for later EXECUTE frames."""

    def __init__(self, rng):
        self.rng = rng
        self.stream = 1
        self.pending_prepares: list[int] = []
        self.ids: list[bytes] = []

    def request(self) -> bytes:
        r, rng = self.rng.random(), self.rng
        self.stream = (self.stream + 1) & 0xFFFF
        if r < 0.12:
            return _frame(int(rng.choice([0x01, 0x05, 0x0B, 0x06, 0x20])), b"", self.stream)
        if r < 0.55:
            return _frame(0x07, _query_body(rng, _rand_query(rng)), self.stream)
        if r < 0.7:
            self.pending_prepares.append(self.stream)
            return _frame(0x09, _query_body(rng, _rand_query(rng)), self.stream)
        if r < 0.85:
            pid = self.ids[int(rng.integers(len(self.ids)))] if self.ids and rng.random() < 0.95 else b"nope%d" % int(
                rng.integers(9))
            return _frame(0x0A, len(pid).to_bytes(2, "big") + pid + b"\x00\x01", self.stream)
        if r < 0.96:
            return _frame(0x07, _query_body(rng, _rand_query(rng)), self.stream)
        if r < 0.97:
            return _frame(0x0D, b"\x00\x00\x01", self.stream)
        if r < 0.98:
            return _frame(0x07, _query_body(rng, b"select a from t"), self.stream, flags=1)
        if r < 0.99:
            return _frame(0x07, _query_body(rng, b"select a from t"), self.stream, version=0x84)
        if r < 0.995:
            return bytes([4, 0, 0, 1, 7]) + (1 << 29).to_bytes(4, "big")
        return _frame(0x07, b"\x00\x00", self.stream)  # query length runs past the input

    def reply(self) -> bytes:
        """A RESULT/prepared reply for a pending PREPARE (or a plain reply)."""
        rng = self.rng
        if self.pending_prepares and rng.random() < 0.8:
            s = self.pending_prepares.pop(0)
            pid = b"id%d" % int(rng.integers(1000))
            self.ids.append(pid)
            return _frame(0x08, (4).to_bytes(4, "big") + len(pid).to_bytes(2, "big") + pid, s, version=0x84)
        return _frame(0x08, (1).to_bytes(4, "big"), 0, version=0x84)


def _chunks(rng, data: bytes) -> list[bytes]:
    cuts = sorted(set(int(x) for x in rng.integers(0, len(data) + 1, int(rng.integers(0, 3)))))
    out, a = [], 0
    for c in cuts + [len(data)]:
        out.append(data[a:c])
        a = c
    return out


def _run_streams(inst, rng, pol_name: bytes, matches, n_conns=40, remote=1, port=80):
    """Random request/reply calls; each call compared op by op (and on the
    injected reply bytes) with the oracle; unconsumed input is presented
    again with the next call."""
    n_frames = n_denied = 0
    for _ in range(n_conns):
        c = Conn(inst, proto=b"cassandra", src=remote, dst_addr=b"2.2.2.2:%d" % port, policy=pol_name)
        assert c.rc == F_OK
        o = CR.Connection(matches, 1024)
        s = _Stream(rng)
        pend = {False: b"", True: b""}
        for _ in range(int(rng.integers(2, 10))):
            reply = bool(rng.random() < 0.3)
            new = b"".join(s.reply() if reply else s.request() for _ in range(int(rng.integers(1, 5))))
            if rng.random() < 0.3:
                new = new[:int(rng.integers(0, len(new) + 1))]
            data = pend[reply] + new
            chunks = _chunks(rng, data)
            cap = int(rng.integers(1, 17))
            rc, ops = c.on_data(chunks, reply=reply, cap=cap)
            orc, oops = o.on_data(reply, chunks, cap)
            assert (rc, ops) == (orc, [tuple(x) for x in oops]), (chunks, reply, cap)
            assert c.injected_reply() == bytes(o.reply_buf), chunks
            c.reply.len = 0
            o.reply_buf.clear()
            if rc != F_OK or any(op == CR.ERROR for op, _ in ops):
                break  # the datapath closes the connection
            used = sum(n for op, n in ops if op in (CR.PASS, CR.DROP))
            n_frames += sum(op in (CR.PASS, CR.DROP) for op, _ in ops) if not reply else 0
            n_denied += sum(op == CR.DROP for op, _ in ops)
            pend[reply] = data[used:]
        c.close()
    return n_frames, n_denied


def test_framing_random_streams_no_policy():
    inst = open_module([(b"node-id", b"cpu-cassandra-frames")], "-1")
    assert inst != 0
    rng = np.random.default_rng(11)
    n_frames, n_denied = _run_streams(inst, rng, b"not-installed", lambda p: False, n_conns=150)
    assert n_frames > 50 and n_denied > 50
    _lib.CloseModule(inst)


def _cass_policy(name, rules, remotes=(1, 3, 4), port=80):
    return {"name": name, "policy": 2, "ingress_per_port_policies": [{"port": port, "rules": [
        {"remote_policies": list(remotes), "l7_proto": "cassandra",
         "l7_rules": {"l7_rules": [{"rule": dict(r)} for r in rules]}}]}]}


def _rand_rules(rng):
    rules = []
    for _ in range(int(rng.integers(1, 4))):
        r = {}
        if rng.random() < 0.7:
            r["query_action"] = str(rng.choice(["select", "insert", "update", "delete", "use", "create-table",
                                                "drop-table", "drop-keyspace", "alter-table", "truncate-table"]))
        if rng.random() < 0.7:
            r["query_table"] = str(rng.choice(["^ks\\.", "t$", ".*", "system\\..*", "^\\.", "users", "a\\.b", "üsers", "ks\\.i"]))
        rules.append(r)
    return rules


@pytest.mark.gpu
def test_gpu_cassandra_reference_cases():
    inst = open_module([(b"node-id", b"gpu-cassandra-kat")], "0")
    assert inst != 0
    for case in KAT["cases"]:
        if case["policy"] is not None:
            t = json.dumps([P.parse_policy_text(case["policy"])]).encode()
            assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK, case["name"]
        c = Conn(inst, proto=b"cassandra", src=KAT["remote"], dst_addr=b"2.2.2.2:80",
                 policy=case["policy_name"].encode())
        assert c.rc == F_OK
        for call in case["calls"]:
            rc, ops = c.on_data([bytes.fromhex(x) for x in call["chunks"]], reply=call["reply"], cap=len(call["ops"]))
            assert rc == F_OK and [list(x) for x in ops] == call["ops"], case["name"]
            assert c.injected_reply() == bytes.fromhex(call["inject"]), case["name"]
            c.reply.len = 0
        c.close()
    _lib.CloseModule(inst)


@pytest.mark.gpu
def test_gpu_cassandra_random_streams_vs_oracle():
    inst = open_module([(b"node-id", b"gpu-cassandra-rand")], "0")
    assert inst != 0
    rng = np.random.default_rng(23)
    n_frames = n_denied = 0
    for i in range(6):
        rules = _rand_rules(rng)
        remotes = (1, 3, 4) if i % 3 else (5,)
        pol = _cass_policy("cq", rules, remotes)
        t = json.dumps([pol]).encode()
        assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK, rules
        o = ProxylibOracle([pol])
        f, d = _run_streams(inst, rng, b"cq", lambda p: o.matches_path("cq", True, 80, 1, p))
        n_frames += f
        n_denied += d
    assert n_frames > 100 and 0 < n_denied < n_frames
    _lib.CloseModule(inst)
