"""Kafka request wire encoding — the client side of what the Kafka proxy
reads, for synthetic batches (bench.py, tests) and for callers that hold
requests as fields.

Follows the encoders of the vendored optiopay/kafka proto package (cilium
fork @01ce283b, Gopkg.toml:58-60):

  serialization.go:215-393   encoder (big-endian ints, int16-length strings,
                             int32-length bytes with nil = -1, array lengths
                             with nil = -1)
  messages.go:228-320        writeMessageSet (offset, size, CRC32 over the
                             message, magic, attributes = codec, key, value;
                             gzip / snappy wrap the inner set in one message
                             whose offset is the last message's)
  messages.go:539-568        MetadataReq.Bytes (nullable topics, v4 flag)
  messages.go:1649-1688      ProduceReq.Bytes (transactional id from v3)
  messages.go Fetch/Offset/OffsetCommit/OffsetFetch/ConsumerMetadata Bytes

One difference is deliberate: writeMessageSet always writes magic 0 with no
timestamp, which the reader (readMessageSet reads a timestamp for request
versions >= 1) misparses; ``message_set(..., timestamps=True)`` writes the
magic-1 layout real clients send for produce v1+.
"""
from __future__ import annotations

import gzip
import struct
import zlib
from typing import Iterable, Optional, Sequence

import numpy as np

PRODUCE, FETCH, OFFSET, METADATA, OFFSET_COMMIT, OFFSET_FETCH, CONSUMER_METADATA = 0, 1, 2, 3, 8, 9, 10
CODEC_NONE, CODEC_GZIP, CODEC_SNAPPY = 0, 1, 2


def i8(v: int) -> bytes:
    return struct.pack(">b", v)


def i16(v: int) -> bytes:
    return struct.pack(">h", v)


def i32(v: int) -> bytes:
    return struct.pack(">i", v)


def i64(v: int) -> bytes:
    return struct.pack(">q", v)


def string(s: Optional[bytes]) -> bytes:
    """EncodeString: uint16 length then the bytes (nil encodes as "")."""
    s = s or b""
    return struct.pack(">H", len(s) & 0xFFFF) + s


def bytes_(b: Optional[bytes]) -> bytes:
    """EncodeBytes: int32 length (-1 for nil) then the bytes."""
    return i32(-1) if b is None else i32(len(b)) + b


def array(items: Optional[Sequence], enc) -> bytes:
    if items is None:
        return i32(-1)
    return i32(len(items)) + b"".join(enc(x) for x in items)


# ---------------------------------------------------------------- snappy --
def _uvarint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _literal(b: bytes) -> bytes:
    n = len(b) - 1
    if n < 60:
        return bytes([n << 2]) + b
    k = (n.bit_length() + 7) // 8
    return bytes([(59 + k) << 2]) + n.to_bytes(k, "little") + b


def _copy(offset: int, length: int) -> bytes:
    out = b""
    while length > 0:
        n = min(length, 64)
        if 4 <= n <= 11 and offset < 2048:
            out += bytes([((offset >> 8) << 5) | ((n - 4) << 2) | 1, offset & 0xFF])
        elif offset < 65536:
            out += bytes([((n - 1) << 2) | 2]) + struct.pack("<H", offset)
        else:
            out += bytes([((n - 1) << 2) | 3]) + struct.pack("<I", offset)
        length -= n
    return out


def snappy_block(data: bytes) -> bytes:
    """A snappy block (golang/snappy format): greedy 4-byte matches."""
    out = bytearray(_uvarint(len(data)))
    table: dict = {}
    i = lit = 0
    while i + 4 <= len(data):
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is not None and i - j < 65536:
            n = 4
            while i + n < len(data) and data[j + n] == data[i + n]:
                n += 1
            if lit < i:
                for s in range(lit, i, 65536):
                    out += _literal(data[s:min(i, s + 65536)])
            out += _copy(i - j, n)
            i += n
            lit = i
        else:
            i += 1
    for s in range(lit, len(data), 65536):
        out += _literal(data[s:min(len(data), s + 65536)])
    return bytes(out)


SNAPPY_JAVA_MAGIC = b"\x82SNAPPY\x00"


def snappy_xerial(data: bytes, chunk: int = 32768) -> bytes:
    """xerial framing (proto/snappy.go:23-50): magic, version 1, compat 1,
    then length-prefixed blocks."""
    out = SNAPPY_JAVA_MAGIC + struct.pack(">ii", 1, 1)
    for s in range(0, max(len(data), 1), chunk):
        blk = snappy_block(data[s:s + chunk])
        out += struct.pack(">i", len(blk)) + blk
    return out


# ---------------------------------------------------------- message sets --
def message(key: Optional[bytes], value: Optional[bytes], codec: int = 0, offset: int = 0,
            timestamp: Optional[int] = None) -> bytes:
    """One message of a set: offset, size, CRC32, magic, attributes,
    [timestamp], key, value."""
    body = i8(0 if timestamp is None else 1) + i8(codec)
    if timestamp is not None:
        body += i64(timestamp)
    body += bytes_(key) + bytes_(value)
    m = struct.pack(">I", zlib.crc32(body) & 0xFFFFFFFF) + body
    return i64(offset) + i32(len(m)) + m


def message_set(messages: Sequence, codec: int = CODEC_NONE, timestamps: bool = False, xerial: bool = False) -> bytes:
    """messages: (key, value) pairs (offsets 0..n-1)."""
    ts = 0 if timestamps else None
    inner = b"".join(message(k, v, 0, o, ts) for o, (k, v) in enumerate(messages))
    if codec == CODEC_NONE or not messages:
        return inner
    if codec == CODEC_GZIP:
        val = gzip.compress(inner, mtime=0)
    else:
        val = snappy_xerial(inner) if xerial else snappy_block(inner)
    return message(None, val, codec, len(messages) - 1, ts)


# -------------------------------------------------------------- requests --
def _request(kind: int, version: int, client: bytes, body: bytes, corr: int = 1) -> bytes:
    rest = i16(kind) + i16(version) + i32(corr) + string(client) + body
    return i32(len(rest)) + rest


def produce(version: int, client: bytes, topics: Sequence, codec: int = CODEC_NONE, acks: int = 1,
            timeout_ms: int = 1000, txn: Optional[bytes] = None, corr: int = 1, xerial: bool = False) -> bytes:
    """topics: [(name, [(partition, [(key, value), ...]), ...]), ...]"""
    body = string(txn) if version >= 3 else b""
    body += i16(acks) + i32(timeout_ms)

    def part(p):
        ms = message_set(p[1], codec, timestamps=version >= 1, xerial=xerial)
        return i32(p[0]) + i32(len(ms)) + ms
    body += array(topics, lambda t: string(t[0]) + array(t[1], part))
    return _request(PRODUCE, version, client, body, corr)


def fetch(version: int, client: bytes, topics: Sequence, corr: int = 1) -> bytes:
    """topics: [(name, [partition, ...]), ...]"""
    body = i32(-1) + i32(100) + i32(1)
    if version >= 3:
        body += i32(1 << 20)
    if version >= 4:
        body += i8(0)

    def part(p):
        return i32(p) + i64(0) + (i64(0) if version >= 5 else b"") + i32(1 << 16)
    body += array(topics, lambda t: string(t[0]) + array(t[1], part))
    return _request(FETCH, version, client, body, corr)


def offset(version: int, client: bytes, topics: Sequence, corr: int = 1) -> bytes:
    body = i32(-1) + (i8(0) if version >= 2 else b"")

    def part(p):
        return i32(p) + i64(-1) + (i32(1) if version == 0 else b"")
    body += array(topics, lambda t: string(t[0]) + array(t[1], part))
    return _request(OFFSET, version, client, body, corr)


def metadata(version: int, client: bytes, topics: Optional[Sequence[bytes]], auto_create: bool = False,
             corr: int = 1) -> bytes:
    body = array(topics, string)
    if version >= 4:
        body += i8(1 if auto_create else 0)
    return _request(METADATA, version, client, body, corr)


def offset_commit(version: int, client: bytes, group: bytes, topics: Sequence, corr: int = 1) -> bytes:
    body = string(group)
    if version >= 1:
        body += i32(1) + string(b"member")
    if version >= 2:
        body += i64(-1)

    def part(p):
        return i32(p) + i64(7) + (i64(0) if version == 1 else b"") + string(b"")
    body += array(topics, lambda t: string(t[0]) + array(t[1], part))
    return _request(OFFSET_COMMIT, version, client, body, corr)


def offset_fetch(version: int, client: bytes, group: bytes, topics: Optional[Sequence], corr: int = 1) -> bytes:
    body = string(group) + array(topics, lambda t: string(t[0]) + array(t[1], i32))
    return _request(OFFSET_FETCH, version, client, body, corr)


def consumer_metadata(version: int, client: bytes, group: bytes, corr: int = 1) -> bytes:
    body = string(group) + (i8(0) if version >= 1 else b"")
    return _request(CONSUMER_METADATA, version, client, body, corr)


def other(kind: int, version: int, client: bytes, body: bytes = b"", corr: int = 1) -> bytes:
    """Any other apiKey (the proxy parses only the header)."""
    return _request(kind, version, client, body, corr)


def encode(api_key: int, version: int, client: bytes, topics: Sequence[bytes], rng: Optional[np.random.Generator] = None,
           codec: int = CODEC_NONE) -> bytes:
    """A request of the given apiKey carrying `topics` (one partition each)."""
    parts = [(t, [0]) for t in topics]
    if api_key == PRODUCE:
        n = 1 if rng is None else int(rng.integers(1, 4))
        msgs = [(None, b"value-%d" % j) for j in range(n)]
        return produce(version, client, [(t, [(0, msgs)]) for t in topics], codec=codec)
    if api_key == FETCH:
        return fetch(version, client, parts)
    if api_key == OFFSET:
        return offset(version, client, parts)
    if api_key == METADATA:
        return metadata(version, client, list(topics))
    if api_key == OFFSET_COMMIT:
        return offset_commit(version, client, b"group", parts)
    if api_key == OFFSET_FETCH:
        return offset_fetch(version, client, b"group", parts)
    if api_key == CONSUMER_METADATA:
        return consumer_metadata(version, client, b"group")
    return other(api_key, version, client, b"\0" * 8)


def concat(requests: Iterable[bytes]):
    """Requests → (raw uint8, offsets uint64 of n + 1)."""
    reqs = list(requests)
    off = np.zeros(len(reqs) + 1, np.uint64)
    off[1:] = np.cumsum([len(r) for r in reqs], dtype=np.uint64)
    raw = np.frombuffer(b"".join(reqs), np.uint8) if reqs else np.zeros(0, np.uint8)
    return raw, off
