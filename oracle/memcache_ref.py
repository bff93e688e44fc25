"""CPU restatement of proxylib's memcached parser and its policy rule.  TEST
INFRASTRUCTURE ONLY (checker for tests/); it shares no code with cilium_amd
and follows the Go code statement by statement, in pure Python (small cases):

  Rule.Matches / L7RuleParser     proxylib/memcached/parser.go:46-148
  MemcacheOpCodeMap               proxylib/memcached/parser.go:212-474
  protocol choice (first byte)    proxylib/memcached/parser.go:186-202
  text OnData / untilEnd / inject proxylib/memcached/text/parser.go:72-327
  binary OnData / inject queue    proxylib/memcached/binary/parser.go:56-205
  the op loop, advanceInput       proxylib/proxylib/connection.go:103-174
  Inject (append what fits)       proxylib/proxylib/connection.go:190-209

Go runtime panics (a slice index past the end) are the _Panic exception,
which the op loop turns into PARSER_ERROR like connection.go:119-135.  Key
regexes use oracle.proxylib_ref.go_regexp (the RE2 subset the tests use).
"""
from __future__ import annotations

from .proxylib_ref import go_regexp

MORE, PASS, DROP, INJECT, ERROR, NOP = 0, 1, 2, 3, 4, 256
F_OK, F_PARSER_ERROR = 0, 2
ERROR_INVALID_FRAME_TYPE = 2

TEXT_DENIED = b"CLIENT_ERROR access denied\r\n"
BIN_DENIED = bytes([0x81, 0, 0, 0, 0, 0, 0, 8, 0, 0, 0, 0x0d] + [0] * 12) + b"access denied"


class ParseError(ValueError):
    pass


class _Panic(Exception):
    pass


def _cmds(text, binary):
    return (frozenset(text), frozenset(binary))


_STORAGE_T = ("add", "set", "replace", "append", "prepend", "cas", "incr", "decr")
OPCODES = {
    "add": _cmds(["add"], [2, 18]), "set": _cmds(["set"], [1, 17]), "replace": _cmds(["replace"], [3, 19]),
    "append": _cmds(["append"], [14, 25]), "prepend": _cmds(["prepend"], [15, 26]), "cas": _cmds(["cas"], []),
    "incr": _cmds(["incr"], [5, 21]), "decr": _cmds(["decr"], [6, 22]),
    "storage": _cmds(_STORAGE_T, [1, 2, 3, 5, 6, 17, 18, 19, 21, 22, 25, 26]),
    "get": _cmds(["get", "gets"], [0, 9, 12, 13]), "delete": _cmds(["delete"], [4, 20]),
    "touch": _cmds(["touch"], [28]), "gat": _cmds(["gat", "gats"], [29, 30]),
    "writeGroup": _cmds(_STORAGE_T + ("delete", "touch"), [1, 2, 3, 4, 5, 6, 17, 18, 19, 20, 21, 22, 25, 26, 28]),
    "slabs": _cmds(["slabs"], []), "lru": _cmds(["lru"], []), "lru_crawler": _cmds(["lru_crawler"], []),
    "watch": _cmds(["watch"], []), "stats": _cmds(["stats"], [16]), "flush_all": _cmds(["flush_all"], [8, 24]),
    "cache_memlimit": _cmds(["cache_memlimit"], []), "version": _cmds(["version"], [11]),
    "misbehave": _cmds(["misbehave"], []), "quit": _cmds(["quit"], [7, 23]), "noop": _cmds([], [10]),
    "verbosity": _cmds([], [27]),
}
for _i, _n in enumerate(["sasl-list-mechs", "sasl-auth", "sasl-step"]):
    OPCODES[_n] = _cmds([], [32 + _i])
for _i, _n in enumerate(["rget", "rset", "rsetq", "rappend", "rappendq", "rprepend", "rprependq", "rdelete",
                         "rdeleteq", "rincr", "rincrq", "rdecr", "rdecrq", "set-vbucket", "get-vbucket",
                         "del-vbucket", "tap-connect", "tap-mutation", "tap-delete", "tap-flush", "tap-opaque",
                         "tap-vbucket-set", "tap-checkpoint-start", "tap-checkpoint-end"]):
    OPCODES[_n] = _cmds([], [48 + _i])


class Meta:
    """meta.MemcacheMeta: command (text; "" for binary), opcode, keys."""

    def __init__(self, command: bytes = b"", opcode: int = 0, keys=()):
        self.command, self.opcode, self.keys = command, opcode, list(keys)

    def is_binary(self) -> bool:
        return len(self.command) == 0


class Rule:
    """memcached Rule (parser.go:35-110) from one L7 rule map."""

    def __init__(self, rule: dict):
        self.commands, found = (frozenset(), frozenset()), False
        self.key_exact = self.key_prefix = b""
        self.regex = None
        for k, v in rule.items():
            if k == "command":
                found = v in OPCODES
                self.commands = OPCODES.get(v, (frozenset(), frozenset()))
            elif k == "keyExact":
                self.key_exact = v.encode("utf-8", "surrogateescape")
            elif k == "keyPrefix":
                self.key_prefix = v.encode("utf-8", "surrogateescape")
            elif k == "keyRegex":
                self.regex = go_regexp(v)
            else:
                raise ParseError("Unsupported key: " + k)
        self.empty = False
        if not found:
            if self.key_exact or self.key_prefix or self.regex is not None:
                raise ParseError("command not specified but key was provided")
            self.empty = True

    def matches(self, m: Meta) -> bool:
        if self.empty:
            return True
        if m.is_binary():
            if m.opcode not in self.commands[1]:
                return False
        elif m.command.decode("latin-1") not in self.commands[0]:
            return False
        if self.key_exact:
            return all(k == self.key_exact for k in m.keys)
        if self.key_prefix:
            return all(k.startswith(self.key_prefix) for k in m.keys)
        if self.regex is not None:
            return all(self.regex.search(k.decode("latin-1")) for k in m.keys)
        return True


# ---- bytes.Fields over Go's UTF-8 decoding (unicode.IsSpace)
_SPACE = {9, 10, 11, 12, 13, 32, 0x85, 0xA0, 0x1680, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000} | set(range(0x2000, 0x200B))


def _rune(b: bytes, i: int):
    """utf8.DecodeRune: (rune, width); invalid → (0xFFFD, 1)."""
    c = b[i]
    if c < 0x80:
        return c, 1
    for n, lo, hi in ((2, 0xC2, 0xDF), (3, 0xE0, 0xEF), (4, 0xF0, 0xF4)):
        if lo <= c <= hi:
            seq = b[i:i + n]
            if len(seq) < n or any(x & 0xC0 != 0x80 for x in seq[1:]):
                return 0xFFFD, 1
            if (c == 0xE0 and seq[1] < 0xA0) or (c == 0xED and seq[1] > 0x9F) or \
               (c == 0xF0 and seq[1] < 0x90) or (c == 0xF4 and seq[1] > 0x8F):
                return 0xFFFD, 1
            r = c & (0x7F >> n)
            for x in seq[1:]:
                r = r << 6 | (x & 0x3F)
            return r, n
    return 0xFFFD, 1


def go_fields(b: bytes) -> list[bytes]:
    out, i, start = [], 0, -1
    while i < len(b):
        r, w = _rune(b, i)
        if r in _SPACE:
            if start >= 0:
                out.append(b[start:i])
                start = -1
        elif start < 0:
            start = i
        i += w
    if start >= 0:
        out.append(b[start:])
    return out


# unicode.ToLower as Go 1.10 applies it (Unicode 10.0 simple mapping): the
# first code point of Python's one-character lower() (U+0130's full mapping
# starts with Go's U+0069), minus the case pairs Unicode 11-13 added.
_POST_UNICODE_10 = ((0x1C90, 0x1CBF), (0x16E40, 0x16E5F), (0xA7B8, 0xA7CA), (0xA7F5, 0xA7F6))


def go_lower_rune(r: int) -> int:
    if r < 0x80:
        return r + 32 if 65 <= r <= 90 else r
    if 0xD800 <= r <= 0xDFFF or r > 0x10FFFF or any(lo <= r <= hi for lo, hi in _POST_UNICODE_10):
        return r
    return ord(chr(r).lower()[0])


def _enc(r: int) -> bytes:
    if 0xD800 <= r <= 0xDFFF or r > 0x10FFFF:
        r = 0xFFFD
    return chr(r).encode("utf-8")


def go_to_lower(b: bytes) -> bytes:
    """strings.ToLower (Go 1.10): ASCII lowered in place; otherwise
    strings.Map(unicode.ToLower): bytes up to the first rune the mapping
    changes are kept verbatim, every rune from there on is re-encoded (an
    invalid byte becomes U+FFFD)."""
    if all(c < 0x80 for c in b):
        return bytes(c + 32 if 65 <= c <= 90 else c for c in b)
    i = 0
    while i < len(b):
        r, w = _rune(b, i)
        if go_lower_rune(r) != r:
            break
        i += w
    if i == len(b):
        return b
    out = bytearray(b[:i])
    while i < len(b):
        r, w = _rune(b, i)
        out += _enc(go_lower_rune(r))
        i += w
    return bytes(out)


def go_atoi(s: bytes):
    """strconv.Atoi on a 64-bit platform: None on error."""
    t = s.decode("latin-1")
    body = t[1:] if t[:1] in ("+", "-") else t
    if not body or not all("0" <= ch <= "9" for ch in body):
        return None
    v = int(t)
    return v if -(1 << 63) <= v < (1 << 63) else None


def _wrap64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >> 63 else v


def _idx(lst, i):
    if i >= len(lst):
        raise _Panic()
    return lst[i]


def _slice(lst, lo, hi):
    if lo > hi or hi > len(lst):
        raise _Panic()
    return lst[lo:hi]


class Connection:
    """One proxylib connection running the memcache parser, with inject
    buffers of capacity ``buf_cap`` and a PolicyMatches callback."""

    def __init__(self, matches, buf_cap: int = 1024):
        self.matches = matches
        self.buf_cap = buf_cap
        self.reply_buf = bytearray()
        self.mode = None
        # text
        self.reply_queue: list[tuple[bytes, bool]] = []
        self.watching = False
        # binary
        self.requests = self.replies = 0
        self.inject_queue: list[tuple[int, int]] = []

    def _inject(self, data: bytes) -> None:
        room = self.buf_cap - len(self.reply_buf)
        self.reply_buf += data[:max(room, 0)]

    # -- text/parser.go:72-262
    def _text(self, reply: bool, bufs: list[bytes]):
        if reply:
            n = 0
            while self.reply_queue and self.reply_queue[0][1]:
                self._inject(TEXT_DENIED)
                self.reply_queue.pop(0)
                n += 1
            if n:
                return INJECT, n * len(TEXT_DENIED)
            if not bufs:
                return NOP, 0
        data = b"".join(bufs)
        lf = data.find(b"\r\n")
        if lf < 0:
            return MORE, (1 if data.endswith(b"\r") else 2)
        tokens = go_fields(data[:lf])
        if not reply:
            command = _idx(tokens, 0)
            frame, noreply, keys = lf + 2, False, []
            if command.startswith(b"get") or command.startswith(b"gat"):
                keys = _slice(tokens, 1 if command.startswith(b"get") else 2, len(tokens))
            elif command in (b"set", b"add", b"replace", b"append", b"prepend", b"cas"):
                keys = _slice(tokens, 1, 2)
                nb = go_atoi(_idx(tokens, 4))
                if nb is None:
                    return ERROR, 0
                frame = _wrap64(frame + nb + 2)
                noreply = len(tokens) == (7 if command[:1] == b"c" else 6)
            elif command == b"delete":
                keys = _slice(tokens, 1, 2)
                noreply = len(tokens) == 3
            elif command in (b"incr", b"decr", b"touch"):
                keys = _slice(tokens, 1, 2)
                noreply = len(tokens) == 4
            elif command in (b"slabs", b"lru", b"lru_crawler", b"stats", b"version", b"misbehave"):
                pass
            elif command in (b"flush_all", b"cache_memlimit"):
                noreply = tokens[-1] == b"noreply"
            elif command == b"quit":
                noreply = True
            elif command == b"watch":
                self.watching = True
            else:
                return ERROR, 0
            if self.matches(Meta(command, 0, keys)):
                if not noreply:
                    self.reply_queue.append((command, False))
                return PASS, frame
            if not noreply:
                if not self.reply_queue:
                    self._inject(TEXT_DENIED)
                else:
                    self.reply_queue.append((command, True))
            return DROP, frame
        intent = _idx(self.reply_queue, 0)[0]
        if self.watching:
            return PASS, lf + 2
        if _idx(tokens, 0) in (b"ERROR", b"CLIENT_ERROR", b"SERVER_ERROR") or intent in (
                b"set", b"add", b"replace", b"append", b"prepend", b"cas", b"delete", b"incr", b"decr", b"touch",
                b"slabs", b"lru", b"flush_all", b"cache_memlimit", b"version", b"misbehave"):
            self.reply_queue.pop(0)
            return PASS, lf + 2
        if intent.startswith(b"get") or intent.startswith(b"gat") or intent == b"stats" or intent == b"lru_crawler":
            if intent == b"lru_crawler" and tokens[0] in (b"OK", b"BUSY", b"BADCLASS"):
                self.reply_queue.pop(0)
                return PASS, lf + 2
            e = data.find(b"\r\nEND\r\n")
            if e > 0:
                self.reply_queue.pop(0)
                return PASS, e + 7
            return MORE, 1
        return ERROR, 0

    # -- binary/parser.go:56-191
    def _bin_deny(self, magic: int) -> None:
        self._inject(bytes([magic]) + BIN_DENIED[1:])
        self.replies += 1

    def _binary(self, reply: bool, bufs: list[bytes]):
        if reply:
            if self.inject_queue and self.inject_queue[0][1] == self.replies + 1:
                self._bin_deny(self.inject_queue.pop(0)[0])
                return INJECT, len(BIN_DENIED)
            if not bufs:
                return NOP, 0
        data = b"".join(bufs)
        if len(data) < 24:
            return MORE, 24 - len(data)
        body = int.from_bytes(data[8:12], "big")
        keylen = int.from_bytes(data[2:4], "big")
        extras = data[4]
        if keylen > 0 and 24 + keylen + extras > len(data):
            return MORE, 24 + keylen + extras - len(data)
        if data[0] & 0x80 != 0x80:
            return ERROR, ERROR_INVALID_FRAME_TYPE
        frame = (body + 24) & 0xFFFFFFFF
        if reply:
            self.replies += 1
            return PASS, frame
        self.requests += 1
        key = data[24 + extras:24 + extras + keylen] if keylen else b""
        if self.matches(Meta(b"", data[1], [key])):
            return PASS, frame
        magic = 0x81 | data[0]
        if self.requests == self.replies + 1:
            self._bin_deny(magic)
        else:
            self.inject_queue.append((magic, self.requests))
        self.inject_queue.append((magic, self.requests))
        return DROP, frame

    # -- connection.go:118-174 with parser.go:186-202
    def on_data(self, reply: bool, chunks: list[bytes], ops_cap: int):
        bufs = [bytes(c) for c in chunks]
        ops = []
        try:
            while len(ops) < ops_cap:
                if self.mode is None:
                    if not bufs or not bufs[0]:
                        break  # NOP
                    self.mode = "bin" if bufs[0][0] >= 128 else "text"
                op, n = (self._binary if self.mode == "bin" else self._text)(reply, bufs)
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
                if op == INJECT and (not reply or len(self.reply_buf) >= self.buf_cap):
                    break
        except _Panic:
            return F_PARSER_ERROR, ops
        return F_OK, ops
