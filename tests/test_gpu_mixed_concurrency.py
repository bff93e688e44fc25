"""Every host entry of one engine handle driven from several threads at
once: HTTP header lists (small calls on the host packer, large ones packed
on the GPU), raw HTTP/1 heads, Kafka records and L4 tuples, each call's
result equal to the one the same call gave alone (those checked against the
oracle first).  A proxy process calls the engine from many workers; the
staging slots, streams and snapshots are shared among them."""
import threading

import numpy as np
import pytest

import oracle
from cilium_amd import synth
from test_http_parse import _blob, _raw_requests

pytestmark = [pytest.mark.gpu]


def test_gpu_mixed_entries_from_threads(gpu):
    pols = synth.starwars_policy()
    gpu.update_http_policy(pols)
    rq = synth.starwars_requests(40_000, seed=71)
    args = (rq["policy"], rq["ingress"], rq["port"], rq["remote"])
    want_h = gpu.http_verdicts_fields(*args, rq["hdr_blob"], rq["hdr_off"])
    assert np.array_equal(want_h[:5000], oracle.HttpOracle(pols).eval(
        *(np.asarray(a)[:5000] for a in args), rq["hdr_blob"], rq["hdr_off"][:5001]))
    raw_blob, raw_off = _blob(_raw_requests(rq))
    assert np.array_equal(gpu.http_verdicts_raw(*args, raw_blob, raw_off), want_h)

    kp, kinfo = synth.kafka_policy(n_rules=300)
    gpu.update_kafka_policy(kp)
    krq = synth.kafka_requests(20_000, kinfo, seed=72)
    reqs, arena = gpu.pack_kafka(**krq)
    want_k = gpu.kafka_verdicts(reqs, arena)
    assert np.array_equal(want_k, oracle.KafkaOracle(kp).eval(**krq))

    keys, ports = synth.l4_table(n_entries=4096, n_ids=4096)
    tuples = synth.l4_tuples(200_000, keys, n_ids=4096, seed=73)
    pm = gpu.policy_map()
    pm.allow_keys(keys, ports)
    want_l4 = pm.verdicts(tuples)
    assert np.array_equal(want_l4, oracle.l4(keys, ports, tuples)[0])

    off = rq["hdr_off"]
    errors = []

    def http_worker(t):
        r = np.random.default_rng(500 + t)
        for _ in range(30):
            n = int(r.choice([1, 7, 64, 900, 3000, 12000]))
            a = int(r.integers(0, len(want_h) - n))
            sub = tuple(np.asarray(x)[a:a + n] for x in args)
            if t % 2:
                got = gpu.http_verdicts_fields(*sub, rq["hdr_blob"], np.ascontiguousarray(off[a:a + n + 1]))
            else:
                got = gpu.http_verdicts_raw(*sub, raw_blob, np.ascontiguousarray(raw_off[a:a + n + 1]))
            if not np.array_equal(got, want_h[a:a + n]):
                errors.append(("http", t, a, n))

    def kafka_worker(t):
        for _ in range(20):
            if not np.array_equal(gpu.kafka_verdicts(reqs, arena), want_k):
                errors.append(("kafka", t))

    def l4_worker(t):
        for _ in range(20):
            if not np.array_equal(pm.verdicts(tuples), want_l4):
                errors.append(("l4", t))

    ts = [threading.Thread(target=http_worker, args=(t,)) for t in range(6)]
    ts += [threading.Thread(target=kafka_worker, args=(t,)) for t in range(2)]
    ts += [threading.Thread(target=l4_worker, args=(t,)) for t in range(2)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(timeout=180)
        assert not x.is_alive(), "a call never returned"
    assert not errors, errors[:5]
