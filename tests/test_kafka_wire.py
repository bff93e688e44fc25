"""Kafka wire decode on the CPU: the engine's host decoder (kafka_wire.h +
kafka_wire.cc, the code that also finishes compressed requests for the GPU
path) against oracle/kafka_wire_ref.py, the pure-Python restatement of
ReadRequest (pkg/kafka/request.go:186-229) and the vendored optiopay/kafka
decoders; the encoder (cilium_amd/kafka_requests.py) against the oracle;
and the wire KATs of tests/golden/kafka_wire_kat.json (pkg/proxy/
kafka_test.go:184-258).

Parity for deflate streams that zlib and Go's compress/flate would judge
differently (both are RFC 1951 decoders; the corpus only holds streams both
accept or reject alike: valid, truncated, or with damaged trailers) is
unpinned.
"""
import gzip

import numpy as np
import pytest

from cilium_amd import kafka_requests as K
from cilium_amd.synth import kafka_policy
from kafka_corpus import corpus, gzip_named, oracle_view, records_view
from kat_util import load
from oracle import kafka_wire_ref as R


def _policy(host):
    pols, info = kafka_policy(n_rules=200, n_topics=60, n_clients=12, seed=5)
    host.update_kafka_policy(pols)
    return [t.encode() for t in info["topics"]], [c.encode() for c in info["clients"]]


def _check(host, reqs_bytes, redirect=None, remote=None):
    n = len(reqs_bytes)
    raw, off = K.concat(reqs_bytes)
    red = np.zeros(n, np.uint16) if redirect is None else redirect
    rem = (np.arange(n) % 7).astype(np.uint32) if remote is None else remote
    recs, arena, status = host.kafka_decode(raw, off, red, rem, diag_cpu=True)
    got = records_view(recs, arena, status)
    want = oracle_view([R.decode(r) for r in reqs_bytes], red, rem, host.kafka_intern)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, reqs_bytes[i][:64].hex(), g, w)
    return got


def test_encoder_roundtrip():
    """Every encoder output decodes to what was encoded."""
    assert R.decode(K.metadata(4, b"c", [b"a", b"b"], True)) == (3, 4, "typed", b"c", [b"a", b"b"])
    assert R.decode(K.metadata(1, b"c", None)) == (3, 1, "typed", b"c", [])
    for v in range(0, 8):
        parts = [(b"t1", [0, 1]), (b"t2", [])]
        assert R.decode(K.fetch(v, b"c", parts))[3:] == (b"c", [b"t1", b"t2"])
        assert R.decode(K.offset(v, b"c", parts))[3:] == (b"c", [b"t1", b"t2"])
        assert R.decode(K.offset_commit(v, b"c", b"g", parts))[3:] == (b"c", [b"t1", b"t2"])
        assert R.decode(K.offset_fetch(v, b"c", b"g", parts))[3:] == (b"c", [b"t1", b"t2"])
        assert R.decode(K.consumer_metadata(v, b"c", b"g")) == (10, v, "consumer", b"c", [])
        for codec in (0, 1, 2):
            msgs = [(None, b"x" * 300), (b"k", b"y")]
            assert R.decode(K.produce(v, b"c", [(b"t", [(0, msgs)])], codec=codec))[3:] == (b"c", [b"t"])
    m = K.message_set([(None, b"abc" * 99)] * 4)
    assert R.snappy_decode(K.snappy_block(m)) == m
    assert R.snappy_decode(K.snappy_xerial(m, 50)) == m
    assert R.gunzip(gzip_named(m, comment=True)) == m


def test_wire_kat_oracle_and_host(host):
    """tests/golden/kafka_wire_kat.json through the oracle and the host decoder."""
    k = load("kafka_wire_kat.json")
    host.update_kafka_policy([{"name": "r", "selectors": [{"identities": None, "rules": k["rules"]}]}])
    raws = [bytes.fromhex(c["hex"]) for c in k["cases"]]
    for c, r in zip(k["cases"], raws):
        d = R.decode(r)
        if c["decoded"] is None:
            assert d is None, c["source"]
        else:
            kind, ver, cls, client, topics = c["decoded"]
            assert d == (kind, ver, cls, client.encode(), [t.encode() for t in topics]), c["source"]
    got = _check(host, raws)
    assert [g[0] for g in got] == [0 if c["decoded"] else 1 for c in k["cases"]]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_host_decoder_vs_oracle_fuzz(host, seed):
    """1500 requests per seed, half of them mutated, bit-exact records."""
    topics, clients = _policy(host)
    reqs = corpus(seed, 1500, topics, clients)
    got = _check(host, reqs)
    st = np.array([g[0] for g in got])
    assert (st == 0).sum() > 300 and (st == 1).sum() > 150  # both outcomes well covered


def test_host_decoder_edges(host):
    """Hand-made edges: empty input, header-only requests, the 12-byte
    boundary, maxParseBufSize, null arrays, huge declared counts, a message
    cut short, bad CRC, unknown codec, gzip trailer damage, nested codecs,
    decoded sets over maxParseBufSize, 255+ topics."""
    topics, clients = _policy(host)
    big = K.message_set([(None, b"z" * 1000)] * 7000)  # ~7 MB decoded > maxParseBufSize
    over_gz = K.message(None, gzip.compress(big, mtime=0), 1)
    over_sn = K.message(None, K.snappy_block(big), 2)
    ok_set = K.message_set([(None, b"first"), (None, b"second")])
    bad_crc = bytearray(ok_set)
    bad_crc[14] ^= 1
    unknown_codec = K.message(None, b"v", 3)
    gz_set = K.message_set([(None, b"first")], K.CODEC_GZIP)
    gz_bad = bytearray(gz_set)
    gz_bad[-3] ^= 0x40
    nested = K.message(None, gzip.compress(K.message(None, K.snappy_block(ok_set), 2), mtime=0), 1)

    def prod(ms, v=0):
        body = K.i16(1) + K.i32(100) + K.i32(1) + K.string(b"t") + K.i32(1) + K.i32(0) + K.i32(len(ms)) + ms
        return K._request(0, v, b"c", body)
    edges = [
        b"", b"\0", b"\0\0\0", b"\0\0\0\x08\0\x03", b"\0\0\0\x08\0\x03\0\0\0\0\0\0",
        b"\0\0\0\x07\0\x03\0\0\0\0\0\0", b"\x7f\xff\xff\xff\0\0",
        K.metadata(0, b"", None), K.metadata(0, b"c", []),
        K._request(3, 0, b"c", K.i32(0x7FFFFFFF)), K._request(3, 0, b"c", K.i32(-5)),
        K._request(1, 0, b"c", K.i32(0) * 3 + K.i32(-1)), K._request(9, 0, b"c", K.string(b"g") + K.i32(-1)),
        prod(ok_set), prod(ok_set[:-3]), prod(bytes(bad_crc)), prod(unknown_codec + ok_set), prod(gz_set),
        prod(bytes(gz_bad)), prod(nested), prod(over_gz), prod(over_sn), prod(ok_set, 1), prod(K.i64(0) + K.i32(0)),
        prod(K.i64(0) + K.i32(-3)), prod(K.i64(0) + K.i32(100 * 65535 + 1)), prod(K.i64(0) + K.i32(4) + b"\0" * 4),
        K.metadata(0, b"c", [b"t%d" % i for i in range(300)]), K.metadata(0, b"c", [topics[0]] * 255),
        K.metadata(0, b"c", [topics[1]] * 254), K.metadata(0, b"c", [topics[2]] * 13),
    ]
    got = _check(host, edges)
    assert got[0][0] == 1 and got[7][0] == 0


def _nested_produce(depth: int) -> bytes:
    """A produce v0 request whose message set is `depth` gzip sets nested
    one inside the other around one plain message."""
    ms = K.message_set([(None, b"v")])
    for _ in range(depth):
        ms = K.message(None, gzip.compress(ms, mtime=0), K.CODEC_GZIP, 0)
    body = K.i16(1) + K.i32(1000)
    body += K.array([(b"t", [(0, ms)])],
                    lambda t: K.string(t[0]) + K.array(t[1], lambda p: K.i32(p[0]) + K.i32(len(p[1])) + p[1]))
    return K._request(K.PRODUCE, 0, b"c", body)


def test_nested_compression_bounds(host):
    """HostInflate's intended deviation (kafka_wire.cc): up to 64 nested
    compressed sets decode as readMessageSet would; a 65th level is a decode
    error (Go's recursion has no depth limit, so the oracle still parses)."""
    _policy(host)
    ok = [_nested_produce(d) for d in (1, 8, 64)]
    _check(host, ok)
    deep = _nested_produce(65)
    assert R.decode(deep) is not None  # the reference semantics parse it
    raw, off = K.concat([deep])
    _, _, status = host.kafka_decode(raw, off, np.zeros(1, np.uint16), np.zeros(1, np.uint32), diag_cpu=True)
    assert int(status[0]) != 0
