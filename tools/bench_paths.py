"""Throughput of the three non-north-star verdict kernels at their BASELINE
configs, one JSON line each (bench.py covers config 5, the 10K-rule HTTP set):

* L4 policymap (config 2): 16K-entry table, 100M tuples
* CIDR prefilter (config 3): 1M mixed v4/v6 prefixes, 1B addresses
* Kafka (config 4): 1K rules, 100M requests
* ipcache: 512K-entry IP → identity map, 1B addresses
* L4 with ipcache identities: config 2's map, identities resolved in-kernel
* proxylib r2d2: 512 r2d2 rules over 64 ports, ~100M requests
  on the HTTP kernel

Inputs are resident in HBM before timing; kernels are timed with HIP events
on their stream.  Each line carries the kernel's HBM roofline (algorithmic
bytes: packed input + output per item) and the CPU oracle timed on a sample.
Distinct synthetic items are generated on the host and tiled on the device
to the config's count; verdicts of the first copy are checked against the
oracle before timing.

    python tools/bench_paths.py [--paths l4,lpm,kafka] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0


def tile_dev(torch, host: np.ndarray, reps: int, dev):
    """Device array of `reps` back-to-back copies of host (doubling copies)."""
    raw = host.reshape(-1).view(np.uint8)
    d = torch.empty(raw.nbytes * reps, dtype=torch.uint8, device=dev)
    d[:raw.nbytes].copy_(torch.from_numpy(raw))
    done = 1
    while done < reps:
        k = min(done, reps - done)
        d[done * raw.nbytes:(done + k) * raw.nbytes].copy_(d[:k * raw.nbytes])
        done += k
    return d


PREWARM_S = 0.3  # --prewarm-seconds


def timed(torch, stream, fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    # untimed launches for PREWARM_S, so the timed ones start at the clocks
    # the GPU holds (a few warm-up launches leave it ~4% slow: bench.py)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < PREWARM_S:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    ev = []
    for _ in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        ev.append((a, b))
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / steps * 1e-3


def cpu_rate(fn, items, seconds):
    if seconds <= 0:
        return None
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        fn()
        n += items
    return n / (time.perf_counter() - t0)


def cpu_rate_mt(fn, chunks, threads, seconds):
    """cpu_rate over `threads` host threads: fn(chunk) on every chunk per
    round (fn must release the GIL, as the ctypes oracle calls do)."""
    if seconds <= 0:
        return None
    from concurrent.futures import ThreadPoolExecutor
    items = sum(len(c) for c in chunks)
    with ThreadPoolExecutor(threads) as ex:
        t0, n = time.perf_counter(), 0
        while time.perf_counter() - t0 < seconds:
            list(ex.map(fn, chunks))
            n += items
        return n / (time.perf_counter() - t0)


def line(metric, n, sec, bytes_per_item, kernel, cpu, cpu_sample, threads, extra):
    achieved = n * bytes_per_item / sec / 1e9
    return {"metric": metric, "value": n / sec, "unit": "verdicts/s", "n_gpus": 1, "ms_per_launch": sec * 1e3,
            "items_per_launch": n, "higher_is_better": True, "data": "synthetic",
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "kernel": kernel, "bytes_per_item": bytes_per_item},
            "cpu_baseline": {"value": cpu, "unit": "verdicts/s", "cores": threads, "kind": "port",
                             "sample": cpu_sample}, **extra}


def bench_l4(torch, dev, stream, cl, args, threads):
    import oracle
    from cilium_amd import synth
    keys, ports = synth.l4_table()
    pm = cl.policy_map()
    pm.allow_keys(keys, ports)
    D, reps = 10_000_000, 10
    tup = synth.l4_tuples(D, keys)
    got = pm.verdicts(tup[:2_000_000])
    exp, _, _ = oracle.l4(keys, ports, tup[:2_000_000])
    assert np.array_equal(got, exp), "L4 verdicts differ from the oracle"
    d_t = tile_dev(torch, tup, reps, dev)
    n = D * reps
    d_o = torch.empty(n, dtype=torch.int32, device=dev)
    sec = timed(torch, stream, lambda: pm.verdicts_dev(d_t, n, d_o, stream=stream.cuda_stream), args.steps, 2)
    chunks = [tup[i * 250_000:(i + 1) * 250_000] for i in range(threads)]
    cpu = cpu_rate_mt(lambda c: oracle.l4(keys, ports, c), chunks, threads, args.cpu_seconds)
    cpu1 = cpu_rate(lambda: oracle.l4(keys, ports, chunks[0]), len(chunks[0]), min(args.cpu_seconds, 2.0))
    kern = "l4_fp_kernel"  # a 16,384-entry map's fingerprints + counters fit LDS
    return line("L4 policymap verdicts/s (__policy_can_access), config 2", n, sec, 16, kern, cpu,
                f"{threads} x 250K tuples of the same workload, {threads} threads (single-core: {cpu1:.4g}/s)"
                if cpu else "", threads,
                {"config": {"workload": "BASELINE config 2: 16,384-entry policy map, 100M tuples",
                            "entries": int(len(keys)), "tuples": n}})


def bench_lpm(torch, dev, stream, cl, args, threads):
    import oracle
    from cilium_amd import synth
    pfx = synth.lpm_prefixes()
    pf = cl.prefilter(dyn4=True, dyn6=True, max_lpm=1 << 21)
    pf.insert(0, pfx)
    D, reps = 100_000_000, 10
    v4, v6, ep4, ep6 = synth.lpm_addresses(D, pfx)
    pf.set_endpoints(ep4, ep6)
    g4, g6 = pf.verdicts(v4[:1_000_000], v6[:400_000])
    o4, o6 = oracle.prefilter(pf.config, pfx, ep4, ep6, v4[:1_000_000], v6[:400_000], nthreads=threads)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6), "prefilter verdicts differ from the oracle"
    d4 = tile_dev(torch, v4, reps, dev)
    d6 = tile_dev(torch, v6, reps, dev)
    n4, n6 = len(v4) * reps, len(v6) * reps
    o4d = torch.empty(n4, dtype=torch.uint8, device=dev)
    o6d = torch.empty(n6, dtype=torch.uint8, device=dev)
    sec = timed(torch, stream, lambda: pf.verdicts_dev(d4, n4, o4d, d6, n6, o6d, stream=stream.cuda_stream),
                args.steps, 2)
    bpi = (n4 * 9 + n6 * 33) / (n4 + n6)
    s4, s6 = v4[:700_000], v6[:300_000]
    cpu = cpu_rate(lambda: oracle.prefilter(pf.config, pfx, ep4, ep6, s4, s6, nthreads=threads), 1_000_000,
                   args.cpu_seconds)
    return line("XDP prefilter verdicts/s (check_v4/check_v6), config 3", n4 + n6, sec, bpi, "lpm_kernel", cpu,
                f"1M addresses (70% v4) of the same workload, {threads} threads", threads,
                {"config": {"workload": "BASELINE config 3: 1M mixed v4/v6 prefixes, 1B addresses",
                            "prefixes": int(len(pfx)), "addresses": n4 + n6}})


def bench_kafka(torch, dev, stream, cl, args, threads):
    import oracle
    from cilium_amd import synth
    pols, info = synth.kafka_policy()
    cl.update_kafka_policy(pols)
    D, reps = 1_000_000, 100
    rq = synth.kafka_requests(D, info)
    reqs, arena = cl.pack_kafka(**rq)
    got = cl.kafka_verdicts(reqs[:200_000], arena)
    sub = {k: v[:200_000] for k, v in rq.items()}
    orc = oracle.KafkaOracle(pols)
    assert np.array_equal(got, orc.eval(**sub, nthreads=threads)), "Kafka verdicts differ from the oracle"
    d_r = tile_dev(torch, reqs, reps, dev)
    d_a = torch.from_numpy(arena).to(dev)
    n = D * reps
    d_o = torch.empty(n, dtype=torch.uint8, device=dev)
    sec = timed(torch, stream, lambda: cl.kafka_verdicts_dev(d_r, n, d_a, d_o, stream=stream.cuda_stream),
                args.steps, 2)
    # the split layout (cg_kafka_verdicts_split_dev): 16-byte heads, 48-byte
    # topic tails read only by the requests that need them
    raw = reqs.view(np.uint8).reshape(D, 64)
    d_h = tile_dev(torch, np.ascontiguousarray(raw[:, :16]), reps, dev)
    d_t = tile_dev(torch, np.ascontiguousarray(raw[:, 16:]), reps, dev)
    del d_r
    sec_split = timed(torch, stream, lambda: cl.kafka_verdicts_split_dev(d_h, d_t, n, d_a, d_o,
                                                                         stream=stream.cuda_stream), args.steps, 2)
    got_split = d_o[:200_000].cpu().numpy()
    assert np.array_equal(got_split, got), "split-layout Kafka verdicts differ"
    cpu = cpu_rate(lambda: orc.eval(**sub, nthreads=threads), 200_000, args.cpu_seconds)
    return line("Kafka verdicts/s (kafkaRedirect.canAccess → MatchesRule), config 4", n, sec_split, 17,
                "kafka_kernel (split heads/topics)", cpu, f"200K requests of the same workload, {threads} threads",
                threads, {"config": {"workload": "BASELINE config 4: 1K Kafka rules, 100M requests", "requests": n,
                                     "layout": "16-B heads + 48-B topic tails (algorithmic bytes: head + verdict)"},
                          "records_64b": {"value": n / sec, "ms": sec * 1e3, "bytes_per_item": 65}})


def kafka_wire_pool(D: int, info: dict, seed: int = 0x4B, codec_frac: float = 0.0):
    """D distinct wire requests of config 4's mix (apiKey / version / topics /
    clientID as synth.kafka_requests draws them); codec_frac of the produce
    requests carry their message sets compressed (gzip or snappy, one
    member / block each: what the device inflates by itself)."""
    from cilium_amd import kafka_requests as K
    from cilium_amd import synth
    rq = synth.kafka_requests(D, info, seed=seed)
    rng = np.random.default_rng(seed)
    reqs, codecs = [], []
    for i in range(D):
        codec = K.CODEC_NONE
        if int(rq["api_key"][i]) == K.PRODUCE and rng.random() < codec_frac:
            codec = K.CODEC_GZIP if rng.random() < 0.5 else K.CODEC_SNAPPY
        codecs.append(codec)
        reqs.append(K.encode(int(rq["api_key"][i]), int(rq["api_version"][i]), rq["client_id"][i], rq["topics"][i],
                             rng, codec=codec))
    return reqs, dict(rq, codec=codecs)


def bench_kafka_wire(torch, dev, stream, cl, args, threads, codec_frac: float = 0.0):
    """Config 4's request mix as wire bytes: kafka_decode_kernel (ReadRequest
    + the optiopay decoders, CRC-32 of every produce message), with
    codec_frac > 0 kafka_inflate_kernel for the compressed sets (gzip /
    snappy decoded on the device, their inner sets parsed), then
    kafka_kernel, per request."""
    import ctypes as C
    from oracle import kafka_wire_ref as R
    from cilium_amd import _native as N
    from cilium_amd import kafka_requests as K
    from cilium_amd import synth
    pols, info = synth.kafka_policy()
    cl.update_kafka_policy(pols)
    D, reps = 65_536, 256
    pool, rq = kafka_wire_pool(D, info, codec_frac=codec_frac)
    if os.environ.get("CILIUM_BENCH_KAFKA_SORTED"):
        # the same requests grouped by (apiKey, version): what a wave decodes
        # when its lanes take one code path (the divergence A/B)
        order = np.lexsort((np.asarray(rq["api_version"]), np.asarray(rq["api_key"])))
        pool = [pool[i] for i in order]
        rq = {k: (v[order] if isinstance(v, np.ndarray) else [v[i] for i in order]) for k, v in rq.items()}
    if codec_frac:
        # copies per call within the 64 MiB per-call inflate arena (each
        # compressed set reserves its decoded size, at most its request's
        # bytes here: a few short messages), so nothing waits for the host
        # for want of room
        zbytes = sum(len(r) for r, z in zip(pool, rq["codec"]) if z)
        reps = max(1, min(256, int((48 << 20) / max(1, zbytes))))
    raw, off = K.concat(pool)
    red = np.zeros(D, np.uint16)
    rem = np.asarray(rq["remote"], np.uint32)
    v = cl.kafka_verdicts_raw(raw[: int(off[4096])], off[:4097], red[:4096], rem[:4096])
    want = cl.kafka_verdicts(*cl.pack_kafka(**{k: x[:4096] for k, x in rq.items() if k != "codec"}))
    assert np.array_equal(v, want), "raw-bytes Kafka verdicts differ from the field-packed path"
    tot = int(off[-1])
    d_raw = tile_dev(torch, raw, reps, dev)
    offs = torch.from_numpy(off[:-1].view(np.int64).copy()).to(dev)
    d_off = (offs.unsqueeze(0) + torch.arange(reps, device=dev, dtype=torch.int64).unsqueeze(1) * tot).reshape(-1)
    d_off = torch.cat([d_off, torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    n = D * reps
    d_red = torch.zeros(n, dtype=torch.int16, device=dev)
    d_rem = torch.from_numpy(rem.view(np.int32)).to(dev).repeat(reps)
    d_reqs = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    cap = tot * reps // 2 + 16
    d_a = torch.empty(cap, dtype=torch.int32, device=dev)
    d_o = torch.empty(n, dtype=torch.uint8, device=dev)
    ss = stream.cuda_stream

    def decode():
        cl.kafka_decode_dev(d_raw, d_off, n, d_red, d_rem, d_reqs, d_a, cap, d_st, stream=ss)

    def both():
        decode()
        cl.kafka_verdicts_dev(d_reqs, n, d_a, d_o, stream=ss)
    i0, d0 = C.c_uint64(), C.c_uint64()
    N.check(N.lib.cg_kafka_decode_stats(cl.h, C.byref(i0), C.byref(d0)))
    sec = timed(torch, stream, decode, args.steps, 2)
    i1, d1 = C.c_uint64(), C.c_uint64()
    N.check(N.lib.cg_kafka_decode_stats(cl.h, C.byref(i1), C.byref(d1)))
    calls = args.steps + 2
    inflated, deferred = (i1.value - i0.value) / calls, (d1.value - d0.value) / calls
    sec2 = timed(torch, stream, both, args.steps, 1)
    # copies carry their original's verdict
    orig = d_o[:D].clone()
    assert bool((d_o.view(reps, D) == orig.unsqueeze(0)).all()), "copies' verdicts differ"
    assert np.array_equal(orig.cpu().numpy(), cl.kafka_verdicts_raw(raw, off, red, rem))
    bpi = tot / D + 8 + 2 + 4 + 64 + 1
    sample = pool[:20_000]
    cpu = cpu_rate(lambda: [R.decode(r) for r in sample], len(sample), args.cpu_seconds)
    kern = "kafka_decode_kernel + kafka_inflate_kernel" if codec_frac else "kafka_decode_kernel"
    mix = (f"{int(codec_frac * 100)}% of produce requests with gzip / snappy sets" if codec_frac
           else "uncompressed wire bytes")
    out = line(f"Kafka wire decode requests/s (ReadRequest on raw bytes), config 4 mix, {mix}", n, sec, bpi,
               kern, cpu, "20K requests of the same mix through oracle/kafka_wire_ref.decode, "
               "1 thread (pure Python)", 1,
               {"config": {"workload": f"BASELINE config 4 request mix as wire bytes, {mix} "
                           f"({tot / D:.1f} B/request avg), 1K rules", "requests": n},
                "per_call": {"payloads_inflated_on_device": inflated, "requests_finished_by_host": deferred},
                "decode_plus_verdict": {"value": n / sec2, "ms_per_launch": sec2 * 1e3}})
    return out


def bench_http_host(torch, dev, stream, cl, args, threads):
    """Config 5 through the host entry points: cg_http_pack (CPU, the
    packer: field extraction, program lookup, class coding, tile layout) and
    cg_http_verdicts_host (pinned staging → H2D → http_kernel → D2H →
    request order).  The kernel-only rate is bench.py's line."""
    import oracle
    from cilium_amd import _native as N
    from cilium_amd import synth
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    n = 4_000_000
    rq = synth.http10k_requests(n, info, distinct=200_000)
    t_pack = []
    for _ in range(3):
        t0 = time.perf_counter()
        b = cl.pack_http(**rq)
        t_pack.append(time.perf_counter() - t0)
    got = cl.http_verdicts(b)  # warm
    t_e2e = []
    for _ in range(3):
        t0 = time.perf_counter()
        got = cl.http_verdicts(b)
        t_e2e.append(time.perf_counter() - t0)
    sub = {k: v[:50_000] for k, v in rq.items() if k not in ("hdr_blob", "hdr_off")}
    sub["hdr_off"] = rq["hdr_off"][:50_001]
    sub["hdr_blob"] = rq["hdr_blob"]
    assert np.array_equal(got[:50_000], oracle.HttpOracle(pols).eval(**sub, nthreads=threads)), \
        "host-path verdicts differ from the oracle"
    tp, te = min(t_pack), min(t_e2e)
    batch_bytes = b.used_bytes() + int(b.arena.nbytes)
    hdr_bytes = int(rq["hdr_off"][-1])
    return {"metric": "HTTP host path, config 5: cg_http_pack + cg_http_verdicts_host", "value": n / (tp + te),
            "unit": "verdicts/s", "n_gpus": 1, "higher_is_better": True, "data": "synthetic",
            "pack": {"value": n / tp, "unit": "requests/s",
                     "cores": int(N.lib.cg_http_pack_threads()),
                     "header_MBps": hdr_bytes / tp / 1e6,
                     "ms": tp * 1e3},
            "verdicts_host": {"value": n / te, "unit": "verdicts/s", "ms": te * 1e3,
                              "batch_bytes": batch_bytes, "staged_GBps": batch_bytes / te / 1e9,
                              "pcie_peak_GBps": 63.0,
                              "note": "pinned staging memcpy + H2D + kernel + D2H + request-order scatter"},
            "config": {"workload": "BASELINE config 5 (10K-rule HTTP) requests through the host entry points",
                       "requests": n, "header_bytes": hdr_bytes}}


def bench_http_raw(torch, dev, stream, cl, args, threads):
    """Config 5 requests as raw HTTP/1 heads resident in HBM →
    cg_http_verdicts_raw_dev: the codec step, program lookup, packing and the
    verdicts all on the GPU (kernels_http_raw.hip + http_kernel), one call
    per step (the device-layout sequence, the default, only enqueues; with
    CILIUM_GPU_RAW_LAYOUT=host in the environment the round-3 sequence runs
    instead, which synchronizes its stream for a host layout step)."""
    import oracle  # noqa: F401  (the check below uses the host path)
    from cilium_amd import synth
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_http_parse import _blob, _raw_requests
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    D, reps = 65_536, 1_900
    rq = synth.http10k_requests(D, info, seed=synth.SEED ^ 0x4A1)
    raws = _raw_requests(rq)
    blob, off = _blob(raws)
    args_ = (rq["policy"], rq["ingress"], rq["port"], rq["remote"])
    want = cl.http_verdicts(cl.pack_http_raw(*args_, blob, off))
    tot = int(off[-1])
    d_raw = tile_dev(torch, blob[:tot], reps, dev)
    base = torch.arange(reps, dtype=torch.int64, device=dev).unsqueeze(1) * tot
    d_off = torch.cat([(torch.from_numpy(off[:-1].astype(np.int64)).to(dev).unsqueeze(0) + base).reshape(-1),
                       torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    rep = lambda a, dt: tile_dev(torch, np.asarray(a).astype(dt), reps, dev)
    d_pol, d_ing, d_port, d_rem = rep(args_[0], np.uint32), rep(args_[1], np.uint8), rep(args_[2], np.uint16), \
        rep(args_[3], np.uint32)
    n = D * reps
    d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
    run = lambda: cl.http_verdicts_raw_dev(d_raw, d_off, n, d_pol, d_ing, d_port, d_rem, d_out,
                                           stream=stream.cuda_stream)
    sec = timed(torch, stream, run, args.steps, 1)
    got = d_out.view(reps, D)
    if not os.environ.get("CG_EXP_NOCHECK"):  # set only for measuring-device variants (tools/exp_paths.sh)
        assert bool((got == torch.from_numpy(want).to(dev).unsqueeze(0)).all()), "raw-path verdicts differ from host path"
    bpi = tot / D + 4 + 1 + 2 + 4 + 8 + 1  # head bytes, policy/ingress/port/remote, offset, verdict
    return line("HTTP/1 raw heads → verdicts/s on the GPU (codec step + packing + http_kernel), config 5", n, sec,
                bpi, ("raw_scan+raw_rank+raw_build+http_kernel" if os.environ.get("CILIUM_GPU_RAW_LAYOUT") == "host"
                      else "raw_scan_dl+raw_pad+raw_seal+http_kernel<raw>+raw_walk"), None, "", threads,
                {"config": {"workload": f"BASELINE config 5 requests as raw HTTP/1 heads ({tot / D:.1f} B/head avg), "
                            "10K rules", "requests": n},
                 "request_gbps": n * (tot / D) / sec / 1e9})


def bench_http_fields(torch, dev, stream, cl, args, threads):
    """Config 5 requests as parsed header lists (cg_http_pack's input, the
    header map Envoy's filter sees) → verdicts with the grouping, sorting and
    packing on the GPU (kernels_http_raw.hip list mode + http_kernel):
    * device entry: 124.5M lists resident in HBM, cg_http_verdicts_fields_dev,
      HIP-event timed;
    * host entry: 8M lists in host memory, cg_http_verdicts_fields_host
      (pinned staging on 2 workers, H2D, kernels, D2H), wall clock, against
      the host packer path (cg_http_pack + cg_http_verdicts_host) on the same
      lists."""
    import oracle
    from cilium_amd import synth
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    D, reps = 1 << 20, 119
    rq = synth.http10k_requests_fast(D, info, seed=synth.SEED ^ 0xF1E1D)
    blob, off = rq["hdr_blob"], rq["hdr_off"]
    args_ = (rq["policy"], rq["ingress"], rq["port"], rq["remote"])
    want = cl.http_verdicts(cl.pack_http(*args_, blob, off))
    k = 20_000
    exp = oracle.HttpOracle(pols).eval(*(np.asarray(a)[:k] for a in args_), blob, off[:k + 1], nthreads=threads)
    assert np.array_equal(want[:k], exp), "host-path verdicts differ from the oracle"
    tot = int(off[-1])
    d_blob = tile_dev(torch, np.asarray(blob[:tot]), reps, dev)
    base = torch.arange(reps, dtype=torch.int64, device=dev).unsqueeze(1) * tot
    d_off = torch.cat([(torch.from_numpy(off[:-1].astype(np.int64)).to(dev).unsqueeze(0) + base).reshape(-1),
                       torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    rep = lambda a, dt: tile_dev(torch, np.asarray(a).astype(dt), reps, dev)
    d_pol, d_ing, d_port, d_rem = rep(args_[0], np.uint32), rep(args_[1], np.uint8), rep(args_[2], np.uint16), \
        rep(args_[3], np.uint32)
    n = D * reps
    d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
    run = lambda: cl.http_verdicts_fields_dev(d_blob, d_off, n, d_pol, d_ing, d_port, d_rem, d_out,
                                              stream=stream.cuda_stream)
    sec = timed(torch, stream, run, args.steps, 1)
    assert bool((d_out.view(reps, D) == torch.from_numpy(want).to(dev).unsqueeze(0)).all()), \
        "device list-path verdicts differ from the host path"
    del d_blob, d_off, d_pol, d_ing, d_port, d_rem, d_out
    torch.cuda.empty_cache()
    # host entry on 8M lists (8 distinct 1M pools)
    H = 8 * D
    hq = synth.http10k_requests_fast(H, info, seed=synth.SEED ^ 0x8E1D)
    hargs = (hq["policy"], hq["ingress"], hq["port"], hq["remote"], hq["hdr_blob"], hq["hdr_off"])
    got = cl.http_verdicts_fields(*hargs)  # warm (pinned buffers, workers)
    t_host = []
    for _ in range(3):
        t0 = time.perf_counter()
        got = cl.http_verdicts_fields(*hargs)
        t_host.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    ref = cl.http_verdicts(cl.pack_http(*hargs))
    t_pack_path = time.perf_counter() - t0
    assert np.array_equal(got, ref), "host-entry list-path verdicts differ from the host packer path"
    th = min(t_host)
    hbytes = int(hq["hdr_off"][-1])
    bpi = tot / D + 4 + 1 + 2 + 4 + 8 + 1  # list bytes, policy/ingress/port/remote, offset, verdict
    return line("HTTP header lists → verdicts/s, packing on the GPU (cg_http_verdicts_fields_dev), config 5", n, sec,
                bpi, ("raw_scan(lists)+raw_rank+raw_build+http_kernel" if os.environ.get("CILIUM_GPU_RAW_LAYOUT") == "host"
                      else "raw_scan_dl(lists)+raw_pad+raw_seal+http_kernel<raw>+raw_walk"), None, "", threads,
                {"config": {"workload": f"BASELINE config 5 requests as header lists ({tot / D:.1f} B/list avg), "
                            "10K rules, 1M distinct tiled", "requests": n},
                 "host_entry": {"value": H / th, "unit": "verdicts/s", "ms": th * 1e3, "requests": H,
                                "list_bytes": hbytes, "staged_GBps": (hbytes + 19 * H) / th / 1e9,
                                "note": "cg_http_verdicts_fields_host: lists in host memory, pinned staging on 2 "
                                        "workers, H2D, kernels, D2H (PCIe-inclusive)"},
                 "host_packer_path": {"value": H / t_pack_path, "unit": "verdicts/s", "ms": t_pack_path * 1e3,
                                      "note": "cg_http_pack (CPU) + cg_http_verdicts_host on the same lists"}})


def bench_ipcache(torch, dev, stream, cl, args, threads):
    import oracle
    from cilium_amd import synth
    k, v = synth.ipcache_entries()
    ic = cl.ipcache()
    ic.update(k, v)
    D, reps = 100_000_000, 10
    a4, a6 = synth.ipcache_addresses(D, k)
    g4, g6 = ic.resolve(a4[:1_000_000], a6[:400_000])
    o4, o6 = oracle.ipcache(k, v, a4[:1_000_000], a6[:400_000], nthreads=threads)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6), "ipcache results differ from the oracle"
    d4 = tile_dev(torch, a4, reps, dev)
    d6 = tile_dev(torch, a6, reps, dev)
    n4, n6 = len(a4) * reps, len(a6) * reps
    o4d = torch.empty(n4 * 2, dtype=torch.int32, device=dev)
    o6d = torch.empty(n6 * 2, dtype=torch.int32, device=dev)
    sec = timed(torch, stream, lambda: ic.resolve_dev(d4, n4, o4d, d6, n6, o6d, stream=stream.cuda_stream),
                args.steps, 2)
    bpi = (n4 * 12 + n6 * 24) / (n4 + n6)  # address in + {identity, tunnel} out
    s4, s6 = a4[:5_600_000], a6[:2_400_000]
    cpu = cpu_rate(lambda: oracle.ipcache(k, v, s4, s6, nthreads=threads), 8_000_000, args.cpu_seconds)
    return line("ipcache lookups/s (lookup_ip{4,6}_remote_endpoint → identity, tunnel)", n4 + n6, sec, bpi,
                "ipcache_kernel", cpu,
                f"8M addresses (70% v4) of the same workload per call (incl. the oracle's map build), {threads} threads",
                threads, {"config": {"workload": "SURVEY 8(f) row 1: 512K-entry ipcache (MaxEntries), 1B addresses",
                                     "entries": int(len(k)), "addresses": n4 + n6}})


def r2d2_workload(n: int, seed: int = 0xC111A):
    """64 ports x 8 r2d2 rules (cmd and/or an unanchored file regex; a third
    of the rules restricted to 4 of 64 remote identities); requests half
    crafted to hit a random rule, half random."""
    rng = np.random.default_rng(seed)
    ports, rules_of = [], {}
    for pi in range(64):
        port = 7000 + pi
        rules = []
        for ri in range(8):
            k = pi * 8 + ri
            kind = ri % 4
            rule = {}
            if kind != 3:
                rule["cmd"] = ["READ", "WRITE", "READ"][kind]
            if kind == 0:
                rule["file"] = f"^/svc{k}/[a-z]+"
            elif kind == 1:
                rule["file"] = f"data{k}\\.(csv|json)$"
            elif kind == 3:
                rule["file"] = f"tmp{k}"
            r = {"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": rule}]}}
            if ri % 3 == 0:
                r["remote_policies"] = [int(x) for x in rng.choice(64, 4, replace=False) + 256]
            rules.append(r)
            rules_of[(port, ri)] = (rule, r.get("remote_policies"))
        ports.append({"port": port, "rules": rules})
    pols = [{"name": "r2d2-bench", "ingress_per_port_policies": ports}]
    reqs = []
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", np.uint8)
    for i in range(n):
        pi, ri = int(rng.integers(0, 64)), int(rng.integers(0, 8))
        port = 7000 + pi
        rule, rem = rules_of[(port, ri)]
        word = letters[rng.integers(0, 26, int(rng.integers(3, 12)))].tobytes()
        k = pi * 8 + ri
        if rng.random() < 0.5:
            cmd = rule.get("cmd", "READ").encode()
            f = {0: b"/svc%d/" % k + word, 1: b"x/data%d.json" % k, 2: word, 3: b"a/tmp%d/" % k + word}[ri % 4]
            remote = rem[0] if rem else 256 + int(rng.integers(0, 64))
        else:
            cmd = [b"READ", b"WRITE", b"HALT", b"RESET"][int(rng.integers(0, 4))]
            f = b"/svc%d/" % int(rng.integers(0, 512)) + word
            remote = 256 + int(rng.integers(0, 64))
        reqs.append((port, remote, cmd, f))
    return pols, reqs


def bench_l4ipc(torch, dev, stream, cl, args, threads):
    """Config 2's policy map with each tuple's identity resolved from its
    remote IPv4 address through the 475K-entry ipcache in the same kernel."""
    import oracle
    from cilium_amd import synth
    keys, ports = synth.l4_table()
    pm = cl.policy_map()
    pm.allow_keys(keys, ports)
    ik, iv = synth.ipcache_entries()
    rng = np.random.default_rng(5)
    iv = iv.copy()
    iv[:, 0] = rng.choice(np.append(np.unique(keys["sec_label"]), [0, 999_999]), len(iv))
    ic = cl.ipcache()
    ic.update(ik, iv)
    D, reps = 10_000_000, 10
    a4, _ = synth.ipcache_addresses(int(D / 0.7) + 1, ik)
    a4 = a4[:D]
    tup = synth.l4_tuples(D, keys)
    got = pm.verdicts_via_ipcache(ic, a4[:1_000_000], tup[:1_000_000])
    exp, _, _ = oracle.l4_egress_via_ipcache(keys, ports, ik, iv, a4[:1_000_000], tup[:1_000_000])
    assert np.array_equal(got, exp), "ipcache+L4 verdicts differ from the oracle (policy_can_egress4)"
    d_t = tile_dev(torch, tup, reps, dev)
    d_a = tile_dev(torch, a4, reps, dev)
    n = D * reps
    d_o = torch.empty(n, dtype=torch.int32, device=dev)
    from cilium_amd import _native as N

    def run():
        N.check(N.lib.cg_l4_verdicts_ipcache_dev(cl.h, pm.id, ic.id, d_a.data_ptr(), d_t.data_ptr(), n,
                                                 d_o.data_ptr(), stream.cuda_stream))
    sec = timed(torch, stream, run, args.steps, 2)
    sa, st = a4[:1_000_000], tup[:1_000_000]

    def cpu_leg():
        r4, _ = oracle.ipcache(ik, iv, sa, np.zeros((0, 16), np.uint8), nthreads=threads)
        tt = st.copy()
        tt["identity"] = r4[:, 0]
        oracle.l4(keys, ports, tt, oracle.L4_EGRESS)
    cpu = cpu_rate(cpu_leg, len(st), args.cpu_seconds)
    return line("L4 verdicts/s with ipcache identities (bpf_lxc.c:509-527), config 2 map + 475K-entry ipcache", n,
                sec, 20, "l4_fp_kernel<ipcache>", cpu,
                f"1M tuples of the same workload: oracle ipcache ({threads} threads, incl. its map build) then "
                "oracle.l4 (1 thread)", threads,
                {"config": {"workload": "BASELINE config 2 map, 100M tuples, identities from a 512K-draw ipcache",
                            "tuples": n}})


def bench_proxylib(torch, dev, stream, cl, args, threads):
    from bench import replicate_batch
    from cilium_amd.proxylib import ProxylibPolicy
    from oracle.proxylib_ref import ProxylibOracle
    D, reps = 262_144, 400
    pols, reqs = r2d2_workload(D)
    pl = ProxylibPolicy(cl)
    pl.update(pols)
    pidx = pl.index("r2d2-bench")
    args_ = ([pidx] * D, [1] * D, [r[0] for r in reqs], [r[1] for r in reqs], [r[2] for r in reqs],
             [r[3] for r in reqs])
    b = pl.pack(*args_)
    o = ProxylibOracle(pols)
    chk = 20_000
    got = cl.http_verdicts(b)[:chk]
    exp = [int(o.matches("r2d2-bench", True, r[0], r[1], r[2], r[3])) for r in reqs[:chk]]
    assert got.tolist() == exp, "proxylib verdicts differ from the oracle"
    d_batch, nslots, _, data_bytes = replicate_batch(b, reps, dev, torch)
    d_arena = torch.from_numpy(b.arena).to(dev)
    d_out = torch.zeros(nslots, dtype=torch.uint8, device=dev)
    n = D * reps
    sec = timed(torch, stream, lambda: cl.http_verdicts_dev(d_batch, nslots, d_arena, d_out,
                                                            stream=stream.cuda_stream), args.steps, 2)
    bpi = data_bytes / n + 1
    sample = reqs[:20_000]
    cpu = cpu_rate(lambda: [o.matches("r2d2-bench", True, r[0], r[1], r[2], r[3]) for r in sample], len(sample),
                   args.cpu_seconds)
    return line("proxylib r2d2 verdicts/s (PolicyInstance.Matches + r2d2 rules) on http_kernel", n, sec, bpi,
                "http_kernel", cpu, "20K requests of the same workload, 1 thread (pure-Python oracle)", 1,
                {"config": {"workload": "SURVEY 8(f) row 4: 512 r2d2 rules over 64 ports, 104.9M requests",
                            "requests": n, "allow_fraction": float(np.mean(exp))}})


def _proxylib_fields_bench(torch, dev, stream, cl, pols, name, fields, remotes, ports, want, metric, workload, cpu,
                           cpu_sample, reps):
    """Requests given as their proxylib parser's fields (ProxylibPolicy.
    pack_fields: the escaped values http_kernel walks), replicated to
    `reps` copies of each program group on the device; verdicts of the
    distinct requests equal `want` (the oracle's)."""
    from bench import replicate_batch
    from cilium_amd.proxylib import ProxylibPolicy
    pl = ProxylibPolicy(cl)
    pl.update(pols)
    pidx = pl.index(name)
    D = len(fields)
    b = pl.pack_fields([pidx] * D, [1] * D, ports, remotes, fields)
    got = cl.http_verdicts(b)
    assert got.tolist() == list(want), f"{name}: verdicts differ from the oracle"
    d_batch, nslots, _, data_bytes = replicate_batch(b, reps, dev, torch)
    d_arena = torch.from_numpy(np.concatenate([b.arena.view(np.uint8), np.zeros(16, np.uint8)])).to(dev)
    d_out = torch.zeros(nslots, dtype=torch.uint8, device=dev)
    n = D * reps
    sec = timed(torch, stream, lambda: cl.http_verdicts_dev(d_batch, nslots, d_arena, d_out,
                                                            stream=stream.cuda_stream), 5, 2)
    return line(metric, n, sec, data_bytes / n + 1, "http_kernel", cpu, cpu_sample, 1,
                {"config": {"workload": workload, "requests": n, "allow_fraction": float(np.mean(want))}})


def bench_memcache(torch, dev, stream, cl, args, threads):
    """memcache (proxylib/memcached): 64 ports x 8 rules (a text command set
    with keyExact / keyPrefix / keyRegex, or a binary opcode); requests are
    the parser's MemcacheMeta (command or opcode, keys) as fields.  Oracle:
    oracle/memcache_ref.py Rule.matches (parser.go:46-100), any rule of the
    port (PolicyInstance.Matches)."""
    from oracle.memcache_ref import Meta, Rule
    from cilium_amd.proxylib import memcache_request
    rng = np.random.default_rng(0x3CAC)
    ports, rules_of = [], {}
    for pi in range(64):
        rules = []
        for ri in range(8):
            k = pi * 8 + ri
            rule = [{"command": "get", "keyExact": f"user{k}"}, {"command": "set", "keyPrefix": f"cache{k}/"},
                    {"command": "writeGroup", "keyRegex": f"^sess{k}-[0-9]+$"}, {"command": "delete"}][ri % 4]
            rules.append(rule)
        rules_of[7000 + pi] = [Rule(r) for r in rules]
        ports.append({"port": 7000 + pi, "rules": [{"l7_proto": "memcache", "l7_rules": {"l7_rules": [
            {"rule": r} for r in rules]}}]})
    pols = [{"name": "memcache-bench", "ingress_per_port_policies": ports}]
    D = 131_072
    fields, prt, rem, want = [], [], [], []
    for i in range(D):
        pi = int(rng.integers(0, 64))
        k = pi * 8 + int(rng.integers(0, 8))
        cmd = [b"get", b"gets", b"set", b"add", b"delete", b"incr"][int(rng.integers(0, 6))]
        nk = int(rng.integers(1, 4))
        good = rng.random() < 0.5
        keys = [(b"user%d" % k if cmd in (b"get", b"gets") else b"cache%d/x%d" % (k, j) if cmd in (b"set", b"add")
                 else b"sess%d-%d" % (k, j)) if good else b"k%d" % int(rng.integers(0, 1000)) for j in range(nk)]
        m = Meta(cmd, 0, keys)
        fields.append(memcache_request(cmd, 0, keys))
        prt.append(7000 + pi)
        rem.append(1)
        want.append(int(any(r.matches(m) for r in rules_of[7000 + pi])))
    sample = list(zip(fields[:20_000], prt[:20_000]))

    def cpu_fn():
        for f, p in sample:
            m = Meta(f[0][1][1:], 0, [x for x in bytes(f[1][1]).split(b"\x03\x14") if x])
            any(r.matches(m) for r in rules_of[p])
    cpu = cpu_rate(cpu_fn, len(sample), args.cpu_seconds)
    return _proxylib_fields_bench(torch, dev, stream, cl, pols, "memcache-bench", fields, rem, prt, want,
                                  "proxylib memcache verdicts/s (memcached Rule.Matches) on http_kernel",
                                  "SURVEY 8(f) row 4: 512 memcache rules over 64 ports, requests as MemcacheMeta "
                                  "fields", cpu, "20K requests, 1 thread (pure-Python oracle)", 400)


def bench_cassandra(torch, dev, stream, cl, args, threads):
    """cassandra (proxylib/cassandra): 64 ports x 8 rules (query_action /
    query_table regexes); requests are the parser's paths
    "/opcode/action/table" as fields.  Oracle: oracle/proxylib_ref.py
    (CassandraRule.Matches, cassandraparser.go:73-89)."""
    from oracle.proxylib_ref import ProxylibOracle
    from cilium_amd.proxylib import cassandra_request
    rng = np.random.default_rng(0xCA55)
    ports = []
    for pi in range(64):
        rules = []
        for ri in range(8):
            k = pi * 8 + ri
            rules.append([{"query_action": "select", "query_table": f"ks{k}\\.t[0-9]+"},
                          {"query_action": "insert", "query_table": f"^ks{k}\\."},
                          {"query_table": f"audit{k}$"}, {"query_action": "update"}][ri % 4])
        ports.append({"port": 7000 + pi, "rules": [{"l7_proto": "cassandra", "l7_rules": {"l7_rules": [
            {"rule": r} for r in rules]}}]})
    pols = [{"name": "cassandra-bench", "ingress_per_port_policies": ports}]
    o = ProxylibOracle(pols)
    D = 131_072
    fields, prt, rem, want, paths = [], [], [], [], []
    for i in range(D):
        pi = int(rng.integers(0, 64))
        k = pi * 8 + int(rng.integers(0, 8))
        act = [b"select", b"insert", b"update", b"delete", b"truncate"][int(rng.integers(0, 5))]
        tab = [b"ks%d.t%d" % (k, int(rng.integers(0, 9))), b"ks%d.x" % k, b"audit%d" % k,
               b"other%d.t" % int(rng.integers(0, 999))][int(rng.integers(0, 4))]
        path = b"/query/" + act + b"/" + tab
        paths.append(path)
        fields.append(cassandra_request(path))
        prt.append(7000 + pi)
        rem.append(1)
        want.append(int(o.matches_path("cassandra-bench", True, 7000 + pi, 1, path)))
    sample = list(zip(paths[:20_000], prt[:20_000]))
    cpu = cpu_rate(lambda: [o.matches_path("cassandra-bench", True, p, 1, x) for x, p in sample], len(sample),
                   args.cpu_seconds)
    return _proxylib_fields_bench(torch, dev, stream, cl, pols, "cassandra-bench", fields, rem, prt, want,
                                  "proxylib cassandra verdicts/s (CassandraRule.Matches) on http_kernel",
                                  "SURVEY 8(f) row 4: 512 cassandra rules over 64 ports, requests as "
                                  "/opcode/action/table paths", cpu, "20K requests, 1 thread (pure-Python oracle)",
                                  400)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--paths", default="l4,lpm,kafka,ipcache,proxylib,l4ipc")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--prewarm-seconds", type=float, default=0.3)
    args = ap.parse_args()
    global PREWARM_S
    PREWARM_S = args.prewarm_seconds
    import torch
    from cilium_amd.classifier import Classifier
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    cl = Classifier(device=0)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    fns = {"l4": bench_l4, "lpm": bench_lpm, "kafka": bench_kafka, "ipcache": bench_ipcache,
           "proxylib": bench_proxylib, "l4ipc": bench_l4ipc, "kafkawire": bench_kafka_wire, "httphost": bench_http_host, "httpraw": bench_http_raw,
           "httpfields": bench_http_fields, "memcache": bench_memcache, "cassandra": bench_cassandra,
           "kafkawirez": lambda *a: bench_kafka_wire(*a, codec_frac=0.5)}
    for p in args.paths.split(","):
        print(json.dumps(fns[p](torch, dev, stream, cl, args, threads)), flush=True)
    cl.close()


if __name__ == "__main__":
    main()
