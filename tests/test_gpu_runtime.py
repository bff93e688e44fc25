"""Runtime hazards of the device entry points (the `_dev` calls a caller
queues on its own streams), each checked against the oracle:

- the http_kernel chunk-deal ticket: >256 launches queued on two streams
  without a sync (a launch's ticket word is per stream and zeroed in stream
  order, kernels_http.hip launch_http);
- snapshot retirement: tables replaced by a policy update while launches that
  read them are still queued (engine.h LaunchFence);
- the Kafka decode stage never reads past raw_off[n] (a d_raw buffer that ends
  exactly there, at an unaligned start);
- counters read from a thread other than the one that launched.
"""
import threading

import numpy as np
import pytest

import oracle
from cilium_amd import kafka_requests as K
from cilium_amd import synth
from cilium_amd.classifier import KAFKA_REQ_DTYPE

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_http_deal_many_launches_two_streams(gpu):
    torch = _torch()
    pols = synth.starwars_policy()
    gpu.update_http_policy(pols)
    rq = synth.starwars_requests(20_000, seed=77)
    b = gpu.pack_http(**rq)
    exp = oracle.HttpOracle(pols).eval(**rq)
    slot_exp = np.zeros(b.nslots, np.uint8)
    real = b.order < b.n
    slot_exp[real] = exp[b.order[real]]
    dev = torch.device("cuda", 0)
    d_batch = torch.from_numpy(b.batch.view(np.uint8)).to(dev)
    d_arena = torch.from_numpy(np.concatenate([b.arena.view(np.uint8), np.zeros(16, np.uint8)])).to(dev)
    launches = 300
    outs = torch.full((launches, b.nslots), 7, dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
    torch.cuda.synchronize()
    for k in range(launches):
        s = streams[k & 1]
        gpu.http_verdicts_dev(d_batch, b.nslots, d_arena, outs[k], stream=s.cuda_stream)
    torch.cuda.synchronize()
    want = torch.from_numpy(slot_exp).to(dev)
    bad = (outs != want.unsqueeze(0)).any(dim=1).nonzero().flatten().tolist()
    assert not bad, f"launches with wrong verdicts: {bad[:10]}"


def test_http_deal_two_threads_one_stream(gpu):
    """Two host threads issue cg_http_verdicts_dev on one shared stream: the
    ticket reset and its launch are enqueued under one lock, so no launch
    starts from another's spent ticket (every output checked)."""
    torch = _torch()
    pols = synth.starwars_policy()
    gpu.update_http_policy(pols)
    rq = synth.starwars_requests(20_000, seed=78)
    b = gpu.pack_http(**rq)
    exp = oracle.HttpOracle(pols).eval(**rq)
    slot_exp = np.zeros(b.nslots, np.uint8)
    real = b.order < b.n
    slot_exp[real] = exp[b.order[real]]
    dev = torch.device("cuda", 0)
    d_batch = torch.from_numpy(b.batch.view(np.uint8)).to(dev)
    d_arena = torch.from_numpy(np.concatenate([b.arena.view(np.uint8), np.zeros(16, np.uint8)])).to(dev)
    per_thread = 200
    outs = torch.full((2, per_thread, b.nslots), 7, dtype=torch.uint8, device=dev)
    shared = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    errors = []

    def issue(k):
        try:
            for j in range(per_thread):
                gpu.http_verdicts_dev(d_batch, b.nslots, d_arena, outs[k, j], stream=shared.cuda_stream)
        except Exception as e:  # noqa: BLE001 — surfaced below
            errors.append(e)

    ts = [threading.Thread(target=issue, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    want = torch.from_numpy(slot_exp).to(dev)
    bad = (outs.view(2 * per_thread, -1) != want.unsqueeze(0)).any(dim=1).nonzero().flatten().tolist()
    assert not bad, f"launches with wrong verdicts: {bad[:10]}"


def test_l4_tables_retired_after_queued_launches(gpu):
    """Queue several big L4 launches on a caller stream, then replace and
    rebuild the map's tables before they run: the queued launches still see
    the old tables (the old set is freed only after its fence)."""
    torch = _torch()
    keys, ports = synth.l4_table(n_entries=4096, n_ids=2048, seed=3)
    pm = gpu.policy_map()
    pm.allow_keys(keys, ports)
    tuples = synth.l4_tuples(4_000_000, keys, n_ids=2048, seed=4)
    exp = oracle.l4(keys, ports, tuples)[0]
    dev = torch.device("cuda", 0)
    d_t = torch.from_numpy(tuples.view(np.uint8)).to(dev)
    reps = 8
    outs = torch.zeros((reps, len(tuples)), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        torch.cuda._sleep(200_000_000)  # hold the stream so the launches below stay queued
    for r in range(reps):
        pm.verdicts_dev(d_t, len(tuples), outs[r], stream=s.cuda_stream)
    # replace the table: flush + a different key set, rebuilt by the next call
    pm.flush()
    keys2, ports2 = synth.l4_table(n_entries=1024, n_ids=2048, seed=99)
    pm.allow_keys(keys2, ports2)
    small = tuples[:4096].copy()
    got2 = pm.verdicts(small)  # rebuild + publish, then a host call on the new tables
    torch.cuda.synchronize()
    assert np.array_equal(got2, oracle.l4(keys2, ports2, small)[0])
    want = torch.from_numpy(exp).to(dev)
    assert bool((outs == want.unsqueeze(0)).all())
    pm.destroy()


def test_kafka_decode_buffer_ends_at_last_offset(gpu):
    """d_raw ends exactly at raw_off[n] (the requests sit at the end of a
    2 MiB allocation, from an odd address): every record matches the
    host-staged decode."""
    torch = _torch()
    pols, info = synth.kafka_policy(n_rules=100, n_topics=40, n_clients=8, seed=5)
    gpu.update_kafka_policy(pols)
    topics = [t.encode() for t in info["topics"]]
    clients = [c.encode() for c in info["clients"]]
    reqs = [K.metadata(0, clients[i % 8], topics[i % 7: i % 7 + 3]) for i in range(61)]
    reqs += [K.fetch(3, clients[1], [(t, [0]) for t in topics[:5]]) for _ in range(70)]
    raw, off = K.concat(reqs)
    n = len(reqs)
    dev = torch.device("cuda", 0)
    size = 2 << 20
    buf = torch.zeros(size, dtype=torch.uint8, device=dev)
    tot = int(off[-1])
    start = size - tot
    buf[start:] = torch.from_numpy(raw[:tot].copy()).to(dev)
    d_raw = buf[start:]
    assert d_raw.data_ptr() + tot == buf.data_ptr() + size
    d_off = torch.from_numpy(off.view(np.int64).copy()).to(dev)
    d_red = torch.zeros(n, dtype=torch.int16, device=dev)
    d_rem = torch.zeros(n, dtype=torch.int32, device=dev)
    d_reqs = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(n, dtype=torch.uint8, device=dev)
    arena = torch.zeros(4096, dtype=torch.int32, device=dev)
    gpu.kafka_decode_dev(d_raw, d_off, n, d_red, d_rem, d_reqs, arena, 4096, d_st,
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    h = gpu.kafka_decode(raw, off, np.zeros(n, np.uint16), np.zeros(n, np.uint32))
    g = d_reqs.cpu().numpy().view(KAFKA_REQ_DTYPE)
    inline = h[0]["n_topics"] <= 12
    assert (g[inline].view(np.uint8).reshape(-1, 64) == h[0][inline].view(np.uint8).reshape(-1, 64)).all()
    assert np.array_equal(d_st.cpu().numpy(), h[2])


def test_counters_from_another_thread(gpu):
    """Per-entry counters read (lookup/dump) from a thread that never set the
    device include every launch queued before the read."""
    keys, ports = synth.l4_table(n_entries=512, n_ids=256, seed=8)
    pm = gpu.policy_map()
    pm.allow_keys(keys, ports)
    tuples = synth.l4_tuples(200_000, keys, n_ids=256, seed=9)
    pm.verdicts(tuples)
    _, pk, by = oracle.l4(keys, ports, tuples)
    res = {}

    def reader():
        res["dump"] = pm.dump_to_slice()

    t = threading.Thread(target=reader)
    t.start()
    t.join()
    ents = [e for _, e in res["dump"]]
    assert sum(int(e.Packets) for e in ents) == int(pk.sum())
    assert sum(int(e.Bytes) for e in ents) == int(by.sum())
    pm.destroy()
