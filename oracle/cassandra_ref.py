"""CPU restatement of the proxylib Cassandra parser — TEST INFRASTRUCTURE ONLY
(the checker for tests/; never imported by the product path).

Follows /root/reference/proxylib/cassandra/cassandraparser.go:
  OnData                  :171-256  (framing, verdict over every path, unauthorized inject)
  parseQuery              :344-455
  cassandraParseRequest   :457-578  (query/prepare, batch, execute, other opcodes)
  sendUnpreparedMsg       :580-598
  cassandraParseReply     :600-642  (RESULT/prepared → prepared-id → path)
and the op loop of proxylib/proxylib/connection.go:118-174.

Go runtime semantics it keeps: a frame is a slice of the joined input whose
capacity runs to the end of that input (bytes.Join of one slice: an append to
nil, capacity rounded to a Go 1.10 malloc size class and zero-filled), so
slice expressions may read past the frame; index expressions past the frame,
and slices past the capacity, panic → PARSER_ERROR.  Queries are lowered and
split with Go's strings.ToLower / strings.Fields over decoded runes
(memcache_ref.go_to_lower / go_fields; Go 1.10 = Unicode 10.0).  Pinned by
the reference's cassandraparser_test.go cases (tests/golden/cassandra_kat.json).
"""
from __future__ import annotations

from .memcache_ref import go_fields, go_to_lower

MORE, PASS, DROP, INJECT, ERROR = 0, 1, 2, 3, 4
NOP = 256
ERROR_INVALID_FRAME_TYPE, ERROR_INVALID_FRAME_LENGTH = 2, 3
F_OK, F_PARSER_ERROR = 0, 2

_SIZE_CLASSES = (8, 16, 32, 48, 64, 80, 96, 112, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288, 320, 352,
                 384, 416, 448, 480, 512, 576, 640, 704, 768, 896, 1024, 1152, 1280, 1408, 1536, 1792, 2048, 2304,
                 2688, 3072, 3200, 3456, 4096, 4864, 5376, 6144, 6528, 6784, 6912, 8192, 9472, 9728, 10240, 10880,
                 12288, 13568, 14336, 16384, 18432, 19072, 20480, 21760, 24576, 27264, 28672, 32768)

OPCODES = {0x00: "error", 0x01: "startup", 0x02: "ready", 0x03: "authenticate", 0x05: "options",
           0x06: "supported", 0x07: "query", 0x08: "result", 0x09: "prepare", 0x0A: "execute",
           0x0B: "register", 0x0C: "event", 0x0D: "batch", 0x0E: "auth_challenge", 0x0F: "auth_response",
           0x10: "auth_success"}

UNAUTH = bytes([0, 0, 0, 0, 0, 0, 0, 0, 0x1a, 0, 0, 0x21, 0, 0, 0x14]) + b"Request Unauthorized"
UNPREPARED = bytes([0, 0, 0, 0, 0, 0, 0, 0, 0x1a, 0, 0, 0x25, 0])


class _Panic(Exception):
    pass


def _roundup(n: int) -> int:
    if n == 0:
        return 0
    for c in _SIZE_CLASSES:
        if n <= c:
            return c
    return -(-n // 8192) * 8192


class _Buf:
    """data[0:flen] with capacity cap (bytes past len(raw) read as zero)."""

    def __init__(self, raw: bytes, flen: int, cap: int):
        self.raw, self.flen, self.cap = raw, flen, cap

    def idx(self, i: int) -> int:
        if i >= self.flen:
            raise _Panic()
        return self.raw[i]

    def sl(self, lo: int, hi: int) -> bytes:
        if lo > hi or hi > self.cap:
            raise _Panic()
        return self.raw[lo:hi] + bytes(max(0, hi - max(lo, len(self.raw))))

    def u32(self, lo: int) -> int:
        return int.from_bytes(self.sl(lo, lo + 4), "big")

    def u16(self, lo: int) -> int:
        return int.from_bytes(self.sl(lo, lo + 2), "big")


_fields = go_fields
_lower = go_to_lower


class Connection:
    """One proxylib connection running the cassandra parser; `matches(path)`
    is PolicyMatches, reply_buf the reply-direction inject buffer."""

    def __init__(self, matches, buf_cap: int = 1024):
        self.matches = matches
        self.buf_cap = buf_cap
        self.reply_buf = bytearray()
        self.keyspace = b""
        self.by_stream: dict[int, bytes] = {}
        self.by_id: dict[bytes, bytes] = {}

    def _inject(self, data: bytes) -> None:
        room = self.buf_cap - len(self.reply_buf)
        self.reply_buf += data[:max(0, room)]

    # parseQuery (:344-455)
    def _query(self, q: bytes):
        q = q.rstrip(b";")
        f = _fields(_lower(q))
        if any(len(x) >= 2 and x[:2] in (b"--", b"/*", b"//") for x in f):
            return b"", b""
        if len(f) < 2:
            return b"", b""
        action, table = f[0], b""
        if action in (b"select", b"delete"):
            for i in range(1, len(f)):
                if f[i] == b"from":
                    if i + 1 >= len(f):
                        raise _Panic()
                    table = _lower(f[i + 1])
            if not table:
                return b"", b""
        elif action == b"insert":
            if len(f) < 3:
                return b"", b""
            table = _lower(f[2])
        elif action == b"update":
            table = _lower(f[1])
        elif action == b"use":
            self.keyspace = f[1].strip(b"\"\\'")
            table = self.keyspace
        elif action in (b"alter", b"create", b"drop", b"truncate", b"list"):
            action = action + b"-" + f[1]
            if f[1] in (b"table", b"keyspace"):
                if len(f) < 3:
                    return b"", b""
                table = f[2]
                if table == b"if":
                    if action == b"create-table":
                        if len(f) < 6:
                            return b"", b""
                        table = f[5]
                    elif action in (b"drop-table", b"drop-keyspace"):
                        if len(f) < 5:
                            return b"", b""
                        table = f[4]
            if f[1] == b"materialized":
                action += b"-view"
            elif f[1] == b"custom":
                action = b"create-index"
        else:
            return b"", b""
        if table and b"." not in table and action != b"use":
            table = self.keyspace + b"." + table
        return action, table

    # cassandraParseRequest (:457-578)
    def _request(self, d: _Buf):
        if d.idx(0) & 0x80:
            return ERROR_INVALID_FRAME_TYPE, None
        if d.idx(1) & 0x01:
            return ERROR_INVALID_FRAME_TYPE, None
        op = d.idx(4)
        path = OPCODES.get(op, "").encode()
        if op in (0x07, 0x09):
            qlen = d.u32(9)
            query = d.sl(13, (13 + qlen) & 0xFFFFFFFF)
            action, table = self._query(query)
            if not action:
                return ERROR_INVALID_FRAME_TYPE, None
            path = b"/" + path + b"/" + action + b"/" + table
            if op == 0x09:
                self.by_stream[d.u16(2)] = path.replace(b"prepare", b"execute", 1)
            return 0, [path]
        if op == 0x0D:
            d.sl(10, 11)
            raise _Panic()  # Uint16 of a one-byte slice
        if op == 0x0A:
            n = d.u16(9)
            pid = d.sl(11, 11 + n)
            p = self.by_id.get(pid, b"")
            if not p:
                m = bytearray(UNPREPARED)
                m[0] = 0x80 | (d.idx(0) & 7)
                m[2:4] = d.sl(2, 4)
                self._inject(bytes(m))
                self._inject(d.sl(9, 11 + n))
                return ERROR_INVALID_FRAME_TYPE, None
            return 0, [p]
        return 0, [b"/" + path]

    # cassandraParseReply (:600-642)
    def _reply(self, d: _Buf):
        if d.idx(0) & 0x80 != 0x80 or d.idx(1) & 1:
            return
        stream = d.u16(2)
        if d.idx(4) == 0x08 and d.u32(9) == 4:
            n = d.u16(13)
            pid = d.sl(15, 15 + n)
            p = self.by_stream.get(stream, b"")
            if p:
                self.by_id[pid] = p

    # CassandraParser.OnData (:171-256)
    def _on_data(self, reply: bool, bufs: list[bytes]):
        raw = b"".join(bufs)
        cap = _roundup(len(raw)) if len(bufs) == 1 else len(raw)
        if len(raw) < 9:
            return MORE, 9 - len(raw)
        rlen = int.from_bytes(raw[5:9], "big")
        if rlen > 1 << 28:
            return ERROR, ERROR_INVALID_FRAME_LENGTH
        total = 9 + rlen
        if total > len(raw):
            return MORE, total - len(raw)
        d = _Buf(raw, total, cap)
        if reply:
            self._reply(d)
            return PASS, total
        err, paths = self._request(d)
        if err:
            return ERROR, err
        ok = True
        for p in paths:
            if not self.matches(p):
                ok = False
        if not ok:
            m = bytearray(UNAUTH)
            m[0] = 0x80 | (d.idx(0) & 7)
            m[2], m[3] = d.idx(2), d.idx(3)
            self._inject(bytes(m))
            return DROP, total
        return PASS, total

    def on_data(self, reply: bool, chunks: list[bytes], ops_cap: int):
        """connection.go:118-174: (FilterResult, ops)."""
        bufs = [bytes(c) for c in chunks]
        ops = []
        try:
            while len(ops) < ops_cap:
                op, n = self._on_data(reply, bufs)
                if op == NOP:
                    break
                if n == 0:
                    return F_PARSER_ERROR, ops
                ops.append((op, n))
                if op == MORE:
                    break
                if op in (PASS, DROP):
                    b = n
                    while b > 0 and bufs:
                        if b < len(bufs[0]):
                            bufs[0] = bufs[0][b:]
                            b = 0
                        else:
                            b -= len(bufs[0])
                            bufs.pop(0)
        except _Panic:
            return F_PARSER_ERROR, ops
        return F_OK, ops
