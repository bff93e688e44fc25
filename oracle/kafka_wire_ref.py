"""Kafka request decoding restated in pure Python — TEST INFRASTRUCTURE ONLY
(the checker of tests/ for the engine's wire decoder; never imported by
cilium_amd).  It follows, step by step, what the Kafka proxy does with the
bytes of one request:

  pkg/kafka/request.go:186-229         ReadRequest (length < 12 check, version)
  optiopay/kafka proto (vendored, cilium fork @01ce283b, Gopkg.toml:58-60)
    messages.go:124-166                 ReadReq (size, kind, allocParseBuf)
    messages.go:504-537                 ReadMetadataReq (nullable topics, v4 flag)
    messages.go:767-830                 ReadFetchReq
    messages.go:1033-1055               ReadConsumerMetadataReq
    messages.go:1173-1230               ReadOffsetCommitReq
    messages.go:1389-1430               ReadOffsetFetchReq (nullable topics)
    messages.go:1591-1650               ReadProduceReq (+ readMessageSet)
    messages.go:1810-1860               ReadOffsetReq
    messages.go:352-494                 readMessageSet (CRC32, gzip, snappy; the
                                        parser runs with SimplifiedMessageSetParsing
                                        false, pkg/proxy/kafka.go:449-451)
    serialization.go:32-190             decoder (sticky errors, DecodeString,
                                        DecodeArrayLen, DecodeBytes)
    snappy.go:23-50 + golang/snappy decode_other.go (block format, xerial framing)
    utils.go:9,18-24                    maxParseBufSize, allocParseBuf

A request slice is the connection's bytes from the start of one request:
ReadReq reads exactly 4 + size bytes of it.  decode() returns None when
ReadRequest returns an error (the proxy then closes the connection,
pkg/proxy/kafka.go:340-347), else (kind, version, request class, clientID,
topics) where class is "typed" (the 6 topic-carrying kinds), "consumer"
(ConsumerMetadata) or "nil" (every other apiKey: request == nil).
"""
from __future__ import annotations

import gzip
import struct
import zlib

MAX_PARSE_BUF = 100 * 65535  # utils.go:9 maxParseBufSize = 100 * math.MaxUint16


class _Err(Exception):
    """A decode error: eof=True for io.EOF / io.ErrUnexpectedEOF."""

    def __init__(self, eof: bool):
        self.eof = eof


class _Stream:
    """io.Reader over bytes; reads share one position (bytes.Buffer /
    bytes.Reader), optionally through an io.LimitReader."""

    def __init__(self, buf: bytes):
        self.buf, self.pos = buf, 0

    def read_full(self, n: int, limit=None) -> bytes:
        avail = len(self.buf) - self.pos
        if limit is not None:
            avail = min(avail, limit[0])
        if n > avail:
            # io.ReadFull consumes what there is, then EOF / ErrUnexpectedEOF
            self.pos += avail
            if limit is not None:
                limit[0] -= avail
            raise _Err(True)
        out = self.buf[self.pos:self.pos + n]
        self.pos += n
        if limit is not None:
            limit[0] -= n
        return out


class _Dec:
    """proto decoder: the first error sticks and later reads return 0/""."""

    def __init__(self, st: _Stream, limit=None):
        self.st, self.limit, self.err = st, limit, None

    def _read(self, n):
        if self.err is not None:
            return None
        try:
            return self.st.read_full(n, self.limit)
        except _Err as e:
            self.err = e
            return None

    def i8(self):
        b = self._read(1)
        return 0 if b is None else struct.unpack(">b", b)[0]

    def i16(self):
        b = self._read(2)
        return 0 if b is None else struct.unpack(">h", b)[0]

    def i32(self):
        b = self._read(4)
        return 0 if b is None else struct.unpack(">i", b)[0]

    def u32(self):
        b = self._read(4)
        return 0 if b is None else struct.unpack(">I", b)[0]

    def i64(self):
        b = self._read(8)
        return 0 if b is None else struct.unpack(">q", b)[0]

    def string(self):
        if self.err is not None:
            return b""
        n = self.i16()
        if self.err is not None or n < 1:
            return b""
        b = self._read(n)
        return b"" if b is None else b

    def bytes_(self):
        if self.err is not None:
            return None
        n = self.i32()
        if self.err is not None or n < 1:
            return None
        if n > MAX_PARSE_BUF:
            self.err = _Err(False)  # messageSizeError
            return None
        return self._read(n)

    def array_len(self, nullable: bool) -> int:
        n = self.i32()  # 0 when an error is already pending
        if n < 0:
            if nullable:
                return -1
            raise _Err(False)  # ErrInvalidArrayLen
        if n > MAX_PARSE_BUF:
            raise _Err(False)
        return n


# ------------------------------------------------------------- snappy ----
def _uvarint(b: bytes):
    x = s = 0
    for i, c in enumerate(b):
        if i == 10:
            return 0, -(i + 1)  # overflow
        if c < 0x80:
            if i == 9 and c > 1:
                return 0, -(i + 1)
            return x | c << s, i + 1
        x |= (c & 0x7F) << s
        s += 7
    return 0, 0


def _snappy_block(src: bytes) -> bytes:
    """golang/snappy Decode (decode.go + decode_other.go)."""
    v, n = _uvarint(src)
    if n <= 0 or v > 0xFFFFFFFF:
        raise _Err(False)
    if v > MAX_PARSE_BUF:
        # decoded or not, readMessageSet rejects a set this long
        raise _Err(False)
    dst = bytearray(v)
    d, s = 0, n
    while s < len(src):
        tag = src[s] & 3
        if tag == 0:
            x = src[s] >> 2
            if x < 60:
                s += 1
            else:
                k = x - 59
                s += 1 + k
                if s > len(src):
                    raise _Err(False)
                x = int.from_bytes(src[s - k:s], "little")
            length = x + 1
            if length <= 0:
                raise _Err(False)
            if length > len(dst) - d or length > len(src) - s:
                raise _Err(False)
            dst[d:d + length] = src[s:s + length]
            d += length
            s += length
            continue
        if tag == 1:
            s += 2
            if s > len(src):
                raise _Err(False)
            length = 4 + ((src[s - 2] >> 2) & 7)
            offset = ((src[s - 2] & 0xE0) << 3) | src[s - 1]
        elif tag == 2:
            s += 3
            if s > len(src):
                raise _Err(False)
            length = 1 + (src[s - 3] >> 2)
            offset = src[s - 2] | src[s - 1] << 8
        else:
            s += 5
            if s > len(src):
                raise _Err(False)
            length = 1 + (src[s - 5] >> 2)
            offset = int.from_bytes(src[s - 4:s], "little")
        if offset <= 0 or d < offset or length > len(dst) - d:
            raise _Err(False)
        for _ in range(length):
            dst[d] = dst[d - offset]
            d += 1
    if d != len(dst):
        raise _Err(False)
    return bytes(dst)


SNAPPY_JAVA_MAGIC = b"\x82SNAPPY\x00"


def snappy_decode(b: bytes) -> bytes:
    """proto/snappy.go:23-50: xerial framing when the magic leads, else one
    block.  (A truncated xerial frame panics in Go; here it is an error.)"""
    if not b.startswith(SNAPPY_JAVA_MAGIC):
        return _snappy_block(b)
    if len(b) < 16:
        raise _Err(False)
    if struct.unpack(">I", b[8:12])[0] != 1:
        raise _Err(False)
    out, i = b"", 16
    while i < len(b):
        if i + 4 > len(b):
            raise _Err(False)
        n = struct.unpack(">I", b[i:i + 4])[0]
        i += 4
        if i + n > len(b):
            raise _Err(False)
        out += _snappy_block(b[i:i + n])
        i += n
    return out


def gunzip(b: bytes) -> bytes:
    """compress/gzip NewReader + ioutil.ReadAll (Go 1.10): members back to
    back (multistream), each a 10-byte header (magic 1f 8b, method 8; FEXTRA,
    FNAME/FCOMMENT strings of < 512 bytes, FHCRC checked), raw deflate, then
    CRC32 and ISIZE.  Input ending cleanly before a header ends the stream;
    anything else that is not a member is an error."""
    out, pos, total = [], 0, 0
    first = True
    while True:
        if pos == len(b) and not first:
            return b"".join(out)
        if len(b) - pos < 10:
            raise _Err(False)
        h = b[pos:pos + 10]
        if h[0] != 0x1F or h[1] != 0x8B or h[2] != 8:
            raise _Err(False)
        flg = h[3]
        q = pos + 10
        if flg & 4:  # FEXTRA
            if q + 2 > len(b):
                raise _Err(False)
            xl = b[q] | b[q + 1] << 8
            q += 2 + xl
            if q > len(b):
                raise _Err(False)
        for bit in (8, 16):  # FNAME, FCOMMENT: NUL-terminated, 511 bytes at most
            if flg & bit:
                z = b.find(b"\0", q, q + 512)
                if z < 0:
                    raise _Err(False)
                q = z + 1
        if flg & 2:  # FHCRC
            if q + 2 > len(b):
                raise _Err(False)
            if (zlib.crc32(b[pos:q]) & 0xFFFF) != (b[q] | b[q + 1] << 8):
                raise _Err(False)
            q += 2
        do = zlib.decompressobj(-15)
        try:
            # past maxParseBufSize the set is rejected whatever follows
            data = do.decompress(b[q:], MAX_PARSE_BUF + 1 - total)
        except zlib.error:
            raise _Err(False)
        total += len(data)
        if total > MAX_PARSE_BUF or not do.eof or len(do.unused_data) < 8:
            raise _Err(False)
        crc, isize = struct.unpack("<II", do.unused_data[:8])
        if crc != zlib.crc32(data) & 0xFFFFFFFF or isize != len(data) & 0xFFFFFFFF:
            raise _Err(False)
        out.append(data)
        pos = len(b) - len(do.unused_data) + 8
        first = False


# ------------------------------------------------------- message sets ----
def _read_message_set(st: _Stream, size: int, version: int, depth: int = 0) -> None:
    """readMessageSet: raises _Err on the errors it returns, returns on the
    early exits it takes (EOF inside the set, empty / short / bad-CRC
    message, unknown compression)."""
    if size < 0:
        return
    if size > MAX_PARSE_BUF:
        raise _Err(False)
    lim = [size]
    dec = _Dec(st, lim)
    while True:
        dec.i64()  # offset
        if dec.err is not None:
            if dec.err.eof:
                return
            raise dec.err
        msize = dec.i32()
        if dec.err is not None:
            if dec.err.eof:
                return
            raise dec.err
        if msize <= 0:
            return
        if msize > MAX_PARSE_BUF:
            raise _Err(False)
        try:
            msgbuf = st.read_full(msize, lim)
        except _Err as e:
            if e.eof:
                return
            raise
        md = _Dec(_Stream(msgbuf))
        crc = md.u32()
        if msize <= 4:
            return
        if crc != zlib.crc32(msgbuf[4:]) & 0xFFFFFFFF:
            return
        md.i8()  # magic
        attributes = md.i8()
        if version >= 1:
            md.i64()  # timestamp
        comp = attributes & 3
        if comp == 0:
            md.bytes_()
            md.bytes_()
            if md.err is not None:
                raise md.err
        elif comp in (1, 2):
            md.bytes_()
            val = md.bytes_()
            if md.err is not None:
                raise md.err
            val = val or b""
            decoded = gunzip(val) if comp == 1 else snappy_decode(val)
            _read_message_set(_Stream(decoded), len(decoded), version, depth + 1)
        else:
            return  # `return nil, err` with err == nil


# ----------------------------------------------------------- requests ----
TYPED = {0: "produce", 1: "fetch", 2: "offset", 3: "metadata", 8: "offset_commit", 9: "offset_fetch"}
CONSUMER_METADATA = 10


def _topic_array(dec: _Dec, per_partition, nullable=False):
    """A topics array of {name, partitions[]} (partitions non-nullable)."""
    n = dec.array_len(nullable)
    if n < 0:
        return None
    names = []
    for _ in range(n):
        names.append(dec.string())
        m = dec.array_len(False)
        for _ in range(m):
            per_partition()
            if dec.err is not None:
                break
        if dec.err is not None:
            break  # every later read is a no-op: the outcome is the error
    return names


def decode(raw: bytes):
    """ReadRequest on the bytes of one request: None on error, else
    (api_key, version, cls, client_id, topics)."""
    try:
        return _decode(raw)
    except _Err:
        return None


def _decode(raw: bytes):
    st = _Stream(raw)
    d = _Dec(st)
    size = d.i32()
    if d.err is not None:
        raise d.err
    if size <= 0:
        raise _Err(True)
    kind = d.i16()
    if d.err is not None:
        raise d.err
    if size + 4 > MAX_PARSE_BUF:
        raise _Err(False)
    b = bytearray(size + 4)
    b[0:4] = struct.pack(">i", size)
    if len(b) >= 6:
        b[4:6] = struct.pack(">h", kind)
    if len(b) > 6:
        b[6:] = st.read_full(len(b) - 6)
    if len(b) < 12:
        raise _Err(False)  # "unexpected end of request (length < 12 bytes)"
    version = struct.unpack(">h", bytes(b[6:8]))[0]
    msg = bytes(b)
    if kind not in TYPED and kind != CONSUMER_METADATA:
        return kind, version, "nil", b"", []
    s = _Stream(msg)
    dec = _Dec(s)
    dec.i32()
    dec.i16()
    ver = dec.i16()
    dec.i32()  # correlation id
    client = dec.string()
    topics = []
    if kind == CONSUMER_METADATA:
        dec.string()  # consumer group
        if ver >= 1:
            dec.i8()
        if dec.err is not None:
            raise dec.err
        return kind, version, "consumer", client, []
    if kind == 0:  # produce
        if ver >= 3:
            dec.string()  # transactional id
        dec.i16()
        dec.i32()
        n = dec.array_len(False)
        for _ in range(n):
            if dec.err is not None:
                break
            topics.append(dec.string())
            m = dec.array_len(False)
            for _ in range(m):
                dec.i32()
                if dec.err is not None:
                    raise dec.err
                mss = dec.i32()
                if dec.err is not None:
                    raise dec.err
                _read_message_set(s, mss, ver)
    elif kind == 1:  # fetch
        dec.i32()
        dec.i32()
        dec.i32()
        if ver >= 3:
            dec.i32()
        if ver >= 4:
            dec.i8()

        def part():
            dec.i32()
            dec.i64()
            if ver >= 5:
                dec.i64()
            dec.i32()
        topics = _topic_array(dec, part)
    elif kind == 2:  # offset
        dec.i32()
        if ver >= 2:
            dec.i8()

        def part():
            dec.i32()
            dec.i64()
            if ver == 0:
                dec.i32()
        topics = _topic_array(dec, part)
    elif kind == 3:  # metadata
        n = dec.array_len(True)
        topics = None if n < 0 else []
        for _ in range(max(n, 0)):
            if dec.err is not None:
                break
            topics.append(dec.string())
        if ver >= 4:
            dec.i8()
    elif kind == 8:  # offset commit
        dec.string()
        if ver >= 1:
            dec.i32()
            dec.string()
        if ver >= 2:
            dec.i64()

        def part():
            dec.i32()
            dec.i64()
            if ver == 1:
                dec.i64()
            dec.string()
        topics = _topic_array(dec, part)
    elif kind == 9:  # offset fetch
        dec.string()

        def part():
            dec.i32()
        topics = _topic_array(dec, part, nullable=True)
    if dec.err is not None:
        raise dec.err
    return kind, version, "typed", client, topics or []
