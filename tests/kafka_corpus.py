"""Seeded corpora of Kafka request wire bytes for the decoder parity tests:
well-formed requests of every kind the proxy parses (all versions the
vendored decoders distinguish, nullable arrays, long topic lists, message
sets with none / gzip / snappy / xerial-snappy / nested codecs), and
mutations of them (truncation, byte flips, size and length fields rewritten,
CRC damage, gzip member damage), each as the connection's bytes from the
start of one request (sometimes with the next request's bytes behind it)."""
from __future__ import annotations

import gzip
import io
import struct

import numpy as np

from cilium_amd import kafka_requests as K

OTHER_KEYS = [4, 5, 6, 7, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 36, 37, 42, 100, 1000, -1, -7]


def gzip_named(data: bytes, name: str = "set.bin", comment: bool = False) -> bytes:
    """A gzip member with FNAME (and FCOMMENT / FHCRC flags set by hand)."""
    bio = io.BytesIO()
    with gzip.GzipFile(filename=name, mode="wb", fileobj=bio, mtime=0) as f:
        f.write(data)
    out = bytearray(bio.getvalue())
    if comment:
        # insert FCOMMENT after FNAME: flag 0x10, a NUL-terminated comment
        z = out.index(0, 10) + 1
        out[3] |= 0x10
        out[z:z] = b"a comment\0"
    return bytes(out)


def _topics(rng, pool, n):
    return [pool[int(rng.integers(0, len(pool)))] if rng.random() < 0.8 else b"unknown-%d" % int(rng.integers(0, 99))
            for _ in range(n)]


def _msgs(rng):
    n = int(rng.integers(0, 4))
    return [(None if rng.random() < 0.7 else b"k%d" % j, bytes(rng.integers(0, 256, int(rng.integers(0, 40)), np.uint8)))
            for j in range(n)]


def _compressed_value(rng, inner: bytes) -> tuple[int, bytes]:
    r = rng.random()
    if r < 0.3:
        return K.CODEC_GZIP, gzip.compress(inner, mtime=0)
    if r < 0.4:
        return K.CODEC_GZIP, gzip.compress(inner[: len(inner) // 2], mtime=0) + gzip.compress(inner[len(inner) // 2:],
                                                                                              mtime=0)
    if r < 0.5:
        return K.CODEC_GZIP, gzip_named(inner, comment=rng.random() < 0.5)
    if r < 0.85:
        return K.CODEC_SNAPPY, K.snappy_block(inner)
    return K.CODEC_SNAPPY, K.snappy_xerial(inner, int(rng.integers(8, 64)))


def message_set(rng, version: int, codecs: bool = True) -> bytes:
    """A produce partition's message set: plain, compressed or nested."""
    ts = 0 if version >= 1 else None
    plain = b"".join(K.message(k, v, 0, o, ts) for o, (k, v) in enumerate(_msgs(rng)))
    r = rng.random()
    if r < 0.55 or not plain or not codecs:
        return plain
    codec, val = _compressed_value(rng, plain)
    if r > 0.95:  # compressed inside compressed
        inner = K.message(None, val, codec, 0, ts)
        codec, val = _compressed_value(rng, inner)
    return plain[: int(rng.integers(0, len(plain) + 1))] * (rng.random() < 0.2) + K.message(None, val, codec, 3, ts)


def produce(rng, version, client, topics, codecs=True):
    body = K.string(b"txn" if rng.random() < 0.5 else b"") if version >= 3 else b""
    body += K.i16(-1) + K.i32(5000)
    parts = []
    for t in topics:
        ps = b""
        npart = int(rng.integers(1, 3))
        for p in range(npart):
            ms = message_set(rng, version, codecs)
            ps += K.i32(p) + K.i32(len(ms)) + ms
        parts.append(K.string(t) + K.i32(npart) + ps)
    body += K.i32(len(topics)) + b"".join(parts)
    return K._request(K.PRODUCE, version, client, body, int(rng.integers(0, 1 << 31)))


def well_formed(rng, topic_pool, client_pool, codecs: bool = True) -> bytes:
    r = rng.random()
    key = [K.PRODUCE, K.FETCH, K.OFFSET, K.METADATA, K.OFFSET_COMMIT, K.OFFSET_FETCH, K.CONSUMER_METADATA,
           None][int(rng.integers(0, 8))]
    version = int(rng.integers(0, 8))
    client = client_pool[int(rng.integers(0, len(client_pool)))] if rng.random() < 0.9 else b""
    nt = int(rng.integers(0, 5))
    if r < 0.04:
        nt = int(rng.integers(13, 40))
    elif r < 0.05:
        nt = int(rng.integers(250, 300))
    topics = _topics(rng, topic_pool, nt)
    parts = [(t, list(range(int(rng.integers(0, 3))))) for t in topics]
    if key == K.PRODUCE:
        return produce(rng, version, client, topics, codecs)
    if key == K.FETCH:
        return K.fetch(version, client, parts)
    if key == K.OFFSET:
        return K.offset(version, client, parts)
    if key == K.METADATA:
        return K.metadata(version, client, None if rng.random() < 0.15 else topics, rng.random() < 0.5)
    if key == K.OFFSET_COMMIT:
        return K.offset_commit(version, client, b"group", parts)
    if key == K.OFFSET_FETCH:
        return K.offset_fetch(version, client, b"group", None if rng.random() < 0.15 else parts)
    if key == K.CONSUMER_METADATA:
        return K.consumer_metadata(version, client, b"group")
    return K.other(OTHER_KEYS[int(rng.integers(0, len(OTHER_KEYS)))], version, client,
                   bytes(rng.integers(0, 256, int(rng.integers(0, 24)), np.uint8)))


def mutate(rng, raw: bytes) -> bytes:
    b = bytearray(raw)
    m = int(rng.integers(0, 9))
    if m == 0 and len(b) > 1:  # truncation (the connection ended)
        return bytes(b[: int(rng.integers(0, len(b)))])
    if m == 1:  # byte flips
        for _ in range(int(rng.integers(1, 4))):
            i = int(rng.integers(0, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
        return bytes(b)
    if m == 2:  # the size field rewritten (the decoders see a longer or shorter request)
        size = struct.unpack(">i", bytes(b[:4]))[0] + int(rng.integers(-12, 13))
        b[:4] = struct.pack(">i", size)
        return bytes(b) + bytes(int(rng.integers(0, 16)))
    if m == 3 and len(b) > 16:  # a 2- or 4-byte length somewhere set to an edge value
        i = int(rng.integers(4, len(b) - 4))
        w = 2 if rng.random() < 0.5 else 4
        v = [0, -1, 1, 0x7FFF, -0x8000, 0x7FFFFFFF, 100 * 65535, 100 * 65535 + 1][int(rng.integers(0, 8))]
        b[i:i + w] = struct.pack(">h" if w == 2 else ">i", max(min(v, 0x7FFF), -0x8000) if w == 2 else v)
        return bytes(b)
    if m == 4:  # trailing bytes of the next request
        return bytes(b) + bytes(rng.integers(0, 256, int(rng.integers(1, 32)), np.uint8))
    if m == 5 and len(b) > 40:  # damage near the end (message sets, CRCs, gzip trailers)
        i = int(rng.integers(len(b) - 40, len(b)))
        b[i] = (b[i] + 1 + int(rng.integers(0, 255))) & 0xFF
        return bytes(b)
    if m == 6:  # the apiKey changed under the same body
        b[4:6] = struct.pack(">h", [0, 1, 2, 3, 8, 9, 10][int(rng.integers(0, 7))])
        return bytes(b)
    if m == 7:  # the version changed under the same body
        b[6:8] = struct.pack(">h", int(rng.integers(-2, 10)))
        return bytes(b)
    return bytes(b)


def corpus(seed: int, n: int, topic_pool, client_pool, mutate_frac: float = 0.5, codecs: bool = True):
    """n requests (bytes), a fraction of them mutated; codecs=False: no
    compressed message sets."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        r = well_formed(rng, topic_pool, client_pool, codecs)
        if rng.random() < mutate_frac:
            r = mutate(rng, r)
        out.append(r)
    return out


def records_view(reqs, arena, status):
    """Decoder outputs → comparable tuples (topics resolved from the arena)."""
    out = []
    for i in range(len(reqs)):
        q = reqs[i]
        nt = int(q["n_topics"])
        if nt <= 12:
            ts = tuple(int(x) for x in q["topic_ids"][:nt])
        else:
            cnt = int(q["topic_ids"][1]) if nt == 255 else nt
            o = int(q["topic_ids"][0])
            ts = tuple(int(x) for x in arena[o:o + cnt])
        out.append((int(status[i]), int(q["api_key"]), int(q["api_version"]), int(q["kind"]), int(q["policy"]),
                    int(q["remote"]), int(q["client_id"]), ts))
    return out


KIND_OF = {"typed": 1, "consumer": 2, "nil": 0}


def oracle_view(decoded, redirect, remote, intern):
    """oracle/kafka_wire_ref.decode results → the tuples records_view gives."""
    out = []
    for i, d in enumerate(decoded):
        if d is None:
            out.append((1, 0, 0, 0, 0xFFFF, int(remote[i]), 0, ()))
            continue
        kind, version, cls, client, topics = d
        out.append((0, kind, version, KIND_OF[cls], int(redirect[i]), int(remote[i]), intern("client", client),
                    tuple(intern("topic", t) for t in topics)))
    return out
