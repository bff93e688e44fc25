"""Kafka wire decode on the GPU (kafka_decode_kernel, kernels_kafka.hip)
through the C ABI: records bit-exact against the host decoder and
oracle/kafka_wire_ref.py, raw bytes → verdicts against the Kafka oracle,
the reference's wire KATs (pkg/proxy/kafka_test.go:184-258), and a
full-size batch checked by copies (every copy of a request decodes to its
original's record).  Compressed produce requests are deferred by the device
and finished by the host decoder inside the same call; the test counts both
kinds so each path is exercised.
"""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import kafka_requests as K
from cilium_amd.classifier import KAFKA_REQ_DTYPE
from cilium_amd.synth import kafka_policy
from kafka_corpus import corpus, oracle_view, records_view
from kat_util import load
from oracle import kafka_wire_ref as R

pytestmark = pytest.mark.gpu


def _policy(gpu, host=None):
    pols, info = kafka_policy(n_rules=200, n_topics=60, n_clients=12, seed=5)
    gpu.update_kafka_policy(pols)
    if host is not None:
        host.update_kafka_policy(pols)
    return pols, [t.encode() for t in info["topics"]], [c.encode() for c in info["clients"]], info["ids"]


def test_gpu_wire_kat(gpu):
    """The reference's proxy test flow as raw bytes → verdicts."""
    k = load("kafka_wire_kat.json")
    gpu.update_kafka_policy([{"name": "r", "selectors": [{"identities": None, "rules": k["rules"]}]}])
    raws = [bytes.fromhex(c["hex"]) for c in k["cases"]]
    raw, off = K.concat(raws)
    n = len(raws)
    v = gpu.kafka_verdicts_raw(raw, off, np.zeros(n, np.uint16), np.zeros(n, np.uint32))
    assert v.tolist() == [c["expect"] for c in k["cases"]], [c["source"] for c in k["cases"]]


@pytest.mark.parametrize("seed", [11, 12])
def test_gpu_decode_vs_host_and_oracle(gpu, host, seed):
    _, topics, clients, ids = _policy(gpu, host)
    reqs = corpus(seed, 4000, topics, clients)
    n = len(reqs)
    raw, off = K.concat(reqs)
    red = np.zeros(n, np.uint16)
    rem = np.asarray(ids, np.uint32)[np.arange(n) % len(ids)]
    g = gpu.kafka_decode(raw, off, red, rem)
    h = host.kafka_decode(raw, off, red, rem, diag_cpu=True)
    gv, hv = records_view(*g), records_view(*h)
    assert gv == hv
    want = oracle_view([R.decode(r) for r in reqs], red, rem, host.kafka_intern)
    assert gv == want
    # records whose topics fit inline are byte-identical (arena offsets aside)
    inline = g[0]["n_topics"] <= N.CG_KAFKA_MAX_TOPICS
    assert (g[0][inline].view(np.uint8) == h[0][inline].view(np.uint8)).all()
    st = g[2]
    assert (st == N.CG_KAFKA_DECODE_OK).sum() > 1000 and (st == N.CG_KAFKA_DECODE_ERROR).sum() > 400


def test_gpu_verdicts_raw_vs_oracle(gpu, host):
    pols, topics, clients, ids = _policy(gpu, host)
    reqs = corpus(21, 6000, topics, clients, mutate_frac=0.3)
    n = len(reqs)
    raw, off = K.concat(reqs)
    red = np.zeros(n, np.uint16)
    rng = np.random.default_rng(3)
    rem = np.where(rng.random(n) < 0.9, np.asarray(ids)[rng.integers(0, len(ids), n)],
                   rng.integers(0, 10, n)).astype(np.uint32)
    got = gpu.kafka_verdicts_raw(raw, off, red, rem)
    dec = [R.decode(r) for r in reqs]
    ok = [i for i, d in enumerate(dec) if d is not None]
    ko = oracle.KafkaOracle(pols)
    v = ko.eval(red[ok], rem[ok], [dec[i][0] for i in ok], [dec[i][1] for i in ok],
                [{"typed": 1, "consumer": 2, "nil": 0}[dec[i][2]] for i in ok], [dec[i][3] for i in ok],
                [dec[i][4] for i in ok])
    want = np.full(n, N.CG_KAFKA_V_CLOSE, np.uint8)
    want[ok] = v
    assert (got == want).all(), np.nonzero(got != want)[0][:10]
    assert {0, 1, 2} <= set(np.unique(got).tolist())


def test_gpu_decode_dev_entry(gpu):
    """cg_kafka_decode_dev on device buffers (torch-allocated) and its
    CG_MAP_FULL report for a too-small arena."""
    import torch
    _, topics, clients, _ = _policy(gpu)
    reqs = [K.metadata(0, b"c", topics[:20]), K.fetch(3, clients[0], [(t, [0]) for t in topics[:3]]),
            K.produce(1, b"c", [(topics[0], [(0, [(None, b"v")])])], codec=K.CODEC_SNAPPY)]
    raw, off = K.concat(reqs)
    n = len(reqs)
    dev = torch.device("cuda:0")
    d_raw = torch.from_numpy(raw.copy()).to(dev)
    d_off = torch.from_numpy(off.view(np.int64).copy()).to(dev)
    d_red = torch.zeros(n, dtype=torch.int16, device=dev)
    d_rem = torch.zeros(n, dtype=torch.int32, device=dev)
    d_reqs = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(n, dtype=torch.uint8, device=dev)
    small = torch.zeros(4, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    with pytest.raises(N.CiliumGPUError) as e:
        gpu.kafka_decode_dev(d_raw, d_off, n, d_red, d_rem,
                             d_reqs, small, 4, d_st, stream)
    assert e.value.code == N.CG_MAP_FULL
    arena = torch.zeros(64, dtype=torch.int32, device=dev)
    used = gpu.kafka_decode_dev(d_raw, d_off, n, d_red, d_rem,
                                d_reqs, arena, 64, d_st, stream)
    assert used == 20
    torch.cuda.synchronize()
    recs = d_reqs.cpu().numpy().view(KAFKA_REQ_DTYPE)
    h = gpu.kafka_decode(raw, off, np.zeros(n, np.uint16), np.zeros(n, np.uint32))
    assert records_view(recs, arena.cpu().numpy().view(np.uint32), d_st.cpu().numpy()) == records_view(*h)


def test_gpu_decode_full_size_copies(gpu):
    """A 4M-request batch built from copies of 4096 distinct uncompressed
    requests: every copy decodes to its original's record."""
    import torch
    _, topics, clients, ids = _policy(gpu)
    pool = corpus(9, 4096, topics, clients, mutate_frac=0.2, codecs=False)
    raw, off = K.concat(pool)
    n0 = len(pool)
    red = np.zeros(n0, np.uint16)
    rem = np.asarray(ids, np.uint32)[np.arange(n0) % len(ids)]
    base = records_view(*gpu.kafka_decode(raw, off, red, rem))
    reps = 1024
    dev = torch.device("cuda:0")
    tot = int(off[-1])
    d_raw = torch.from_numpy(raw.copy()).to(dev).repeat(reps)
    offs = torch.from_numpy(off[:-1].view(np.int64).copy()).to(dev)
    d_off = (offs.unsqueeze(0) + torch.arange(reps, device=dev, dtype=torch.int64).unsqueeze(1) * tot).reshape(-1)
    d_off = torch.cat([d_off, torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    n = n0 * reps
    d_red = torch.zeros(n, dtype=torch.int16, device=dev)
    d_rem = torch.from_numpy(rem.view(np.int32)).to(dev).repeat(reps)
    d_reqs = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(n, dtype=torch.uint8, device=dev)
    cap = tot * reps // 2 + 16
    arena = torch.zeros(cap, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    gpu.kafka_decode_dev(d_raw, d_off, n, d_red, d_rem,
                         d_reqs, arena, cap, d_st, stream)
    torch.cuda.synchronize()
    recs = d_reqs.view(n, 64)
    inline = recs[:, 5] <= N.CG_KAFKA_MAX_TOPICS
    # inline records: each copy's 64 bytes equal its original's
    first = recs[:n0]
    same = (recs.view(reps, n0, 64) == first.unsqueeze(0)).all(dim=2)
    assert bool(same[:, inline[:n0]].all())
    assert bool((d_st.view(reps, n0) == d_st[:n0].unsqueeze(0)).all())
    # the originals against the host-staged decode
    got = records_view(first.cpu().numpy().reshape(-1).view(KAFKA_REQ_DTYPE), arena.cpu().numpy().view(np.uint32),
                       d_st[:n0].cpu().numpy())
    assert got == base


def test_gpu_compressed_sets_decoded_on_device(gpu, host):
    """Produce requests whose message sets hold gzip / snappy / xerial
    messages (kafka_corpus codecs, including two-member gzip and nested
    codecs) decode on the GPU (kafka_inflate_kernel, kw_inflate.h) to the
    host decoder's records and the oracle's; only what the device cannot
    finish (a second gzip member, a nested compressed set) reaches the host
    (cg_kafka_decode_stats)."""
    import ctypes as C
    _, topics, clients, ids = _policy(gpu, host)
    reqs = corpus(31, 3000, topics, clients, mutate_frac=0.1)
    n = len(reqs)
    raw, off = K.concat(reqs)
    red = np.zeros(n, np.uint16)
    rem = np.asarray(ids, np.uint32)[np.arange(n) % len(ids)]
    i0, d0 = C.c_uint64(), C.c_uint64()
    assert N.lib.cg_kafka_decode_stats(gpu.h, C.byref(i0), C.byref(d0)) == N.CG_OK
    g = gpu.kafka_decode(raw, off, red, rem)
    i1, d1 = C.c_uint64(), C.c_uint64()
    assert N.lib.cg_kafka_decode_stats(gpu.h, C.byref(i1), C.byref(d1)) == N.CG_OK
    h = host.kafka_decode(raw, off, red, rem, diag_cpu=True)
    assert records_view(*g) == records_view(*h)
    assert records_view(*g) == oracle_view([R.decode(r) for r in reqs], red, rem, host.kafka_intern)
    inflated, deferred = i1.value - i0.value, d1.value - d0.value
    print(f"compressed payloads decoded on the device: {inflated}, requests finished by the host: {deferred}")
    assert inflated > 100 and deferred < inflated / 2, (inflated, deferred)


def _produce_sets(version, client, topic_sets):
    """A produce request with one partition per topic, each holding the
    given message set."""
    body = (K.string(b"") if version >= 3 else b"") + K.i16(-1) + K.i32(5000)
    body += K.i32(len(topic_sets)) + b"".join(K.string(t) + K.i32(1) + K.i32(0) + K.i32(len(ms)) + ms
                                              for t, ms in topic_sets)
    return K._request(K.PRODUCE, version, client, body, 7)


def test_gpu_wide_compressed_produce_with_full_arena(gpu, host):
    """Compressed produce requests with 13-40 topics (their ids go to the
    topic arena through a second decode pass) in one call with payloads
    that fill the 64 MiB inflate arena (12 sets of 6 MB of zeros, gzip
    and snappy) and payloads whose gzip ISIZE claims 6.5 MB from a few
    bytes.  The second pass re-reads only the outer topic list (it reserves
    nothing), so every record equals the host decoder's and the oracle's
    whatever the arena holds; the unreserved deferrals are counted
    (cg_kafka_inflate_stats)."""
    import ctypes as C
    import gzip
    import struct
    _, topics, clients, ids = _policy(gpu, host)
    rng = np.random.default_rng(41)
    reqs = []
    for j in range(12):  # arena fillers
        inner = bytes(6_000_000)
        val = gzip.compress(inner, 9, mtime=0) if j % 2 == 0 else K.snappy_block(inner)
        ms = K.message(None, val, K.CODEC_GZIP if j % 2 == 0 else K.CODEC_SNAPPY, 0, 0)
        reqs.append(_produce_sets(2, clients[0], [(topics[j % len(topics)], ms)]))
    for j in range(6):  # gzip ISIZE claiming 6.5 MB
        z = bytearray(gzip.compress(K.message(None, b"v", 0, 0, 0), mtime=0))
        z[-4:] = struct.pack("<I", 6_500_000)
        reqs.append(_produce_sets(2, clients[1], [(topics[0], K.message(None, bytes(z), K.CODEC_GZIP, 0, 0))]))
    for j in range(200):  # wide compressed produce requests
        nt = int(rng.integers(13, 41))
        sets = []
        for t in range(nt):
            plain = b"".join(K.message(None, b"m%d" % m, 0, m, 0) for m in range(int(rng.integers(1, 4))))
            codec = K.CODEC_GZIP if rng.random() < 0.5 else K.CODEC_SNAPPY
            val = gzip.compress(plain, mtime=0) if codec == K.CODEC_GZIP else K.snappy_block(plain)
            sets.append((topics[int(rng.integers(0, len(topics)))], K.message(None, val, codec, 0, 0)))
        reqs.append(_produce_sets(2, clients[j % len(clients)], sets))
    order = rng.permutation(len(reqs))
    reqs = [reqs[i] for i in order]
    n = len(reqs)
    raw, off = K.concat(reqs)
    red = np.zeros(n, np.uint16)
    rem = np.asarray(ids, np.uint32)[np.arange(n) % len(ids)]
    u0, u1 = C.c_uint64(), C.c_uint64()
    assert N.lib.cg_kafka_inflate_stats(gpu.h, C.byref(u0)) == N.CG_OK
    g = gpu.kafka_decode(raw, off, red, rem)
    assert N.lib.cg_kafka_inflate_stats(gpu.h, C.byref(u1)) == N.CG_OK
    h = host.kafka_decode(raw, off, red, rem, diag_cpu=True)
    assert records_view(*g) == records_view(*h)
    assert records_view(*g) == oracle_view([R.decode(r) for r in reqs], red, rem, host.kafka_intern)
    assert u1.value - u0.value >= 7, (u0.value, u1.value)  # the six claims and at least one full arena
