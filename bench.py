"""bench.py — batched HTTP L7 policy verdicts on the 10K-rule set (BASELINE
config 5), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--requests-per-gpu B]

A step is one pass of the verdict kernel over the GPU's resident batch of B
packed requests (default 125M = 1B / 8, so at N = 8 the node processes the
config's 1B requests per step; scaling is weak: per-GPU work is fixed).  The
batch holds --distinct (default 8M) distinct requests, each program group's
tiles repeated to B.  After each step the per-rule and per-program counters
are all-reduced across ranks (RCCL) — the only collective on this path.  The
10K rules are compiled once (rank 0) and every rank imports the same table
image (cg_http_policy_export / _import).

Rank 0 prints one JSON line with throughput, the roofline of the verdict
kernel (HIP events on the kernel's stream), the same kernel on a 262K-distinct
batch, the end-to-end raw path (config 5 as raw HTTP/1 heads resident in HBM
→ cg_http_verdicts_raw_dev: parse, pack and verdicts on the GPU), the host
entry (the distinct requests as header lists in host memory →
cg_http_verdicts_fields_host, PCIe-inclusive) and the CPU oracle (the Envoy-faithful std::regex rule scan) timed on a bounded sample on
the host cores given to this GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "policy verdicts/sec (whole node) + request GB/s, 10K-rule L7 HTTP set"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
OUT_BYTES = 1
CHUNK_TILES = 64        # kChunkTiles (csrc/dev_types.h)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--requests-per-gpu", type=int, default=125_000_000)
    ap.add_argument("--distinct", type=int, default=8_388_608)
    ap.add_argument("--small-distinct", type=int, default=262_144,
                    help="second measurement of the kernel on a batch with this many distinct requests (0: skip)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end raw-heads measurement")
    ap.add_argument("--e2e-layout", default="device", choices=["host", "device"],
                    help="raw path sequence for end_to_end: device (the default: slots, chunk table and header "
                         "on the device, no host round trip) or host (CILIUM_GPU_RAW_LAYOUT=host: the round-3 "
                         "sequence, bucket counts laid out on the host)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--prewarm-seconds", type=float, default=0.5,
                    help="before the --warmup steps, run untimed steps back to back for this long, so the timed "
                         "steps start at the clocks the sustained leg holds (0: skip)")
    ap.add_argument("--sustain-seconds", type=float, default=3.0,
                    help="after the timed steps, run steps back to back for this long and report the sustained "
                         "rate (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--layout", default="tile", choices=["tile", "copy"],
                    help="order of the replicated tiles within a program group (replicate_batch)")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="rehearse the N-rank launch, rendezvous and counter all-reduce on the CPU (gloo, the "
                         "library's host table walker on a small batch): no GPU, and not a measurement")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` run without a launcher: start N rank processes
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT, as
    torch.distributed.run sets them) before this process touches a GPU, and
    return the worst exit code.  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_ranks(args.gpus))
    if args.cpu_rehearsal:
        return rehearse(args)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from cilium_amd import synth
    from cilium_amd.classifier import Classifier

    cl = Classifier(device=dev.index)
    pols, info = synth.http10k_rules()
    t0 = time.time()
    bcast_s = share_policy(cl, pols, dist, rank, dev, torch)
    compile_s = time.time() - t0
    stats = cl.http_policy_stats()

    D = min(args.distinct - args.distinct % 64, args.requests_per_gpu)
    rq = synth.http10k_requests_fast(D, info, seed=synth.SEED ^ (rank * 7919))
    b = cl.pack_http(**rq)
    reps = max(1, -(-args.requests_per_gpu // D))  # ceiling: >= the per-GPU share
    B = reps * D                                  # requests per GPU per step
    d_batch, nslots, tile_map, data_bytes = replicate_batch(b, reps, dev, torch, layout=args.layout)
    d_arena = torch.from_numpy(np.concatenate([b.arena.view(np.uint8), np.zeros(16, np.uint8)])).to(dev)
    d_out = torch.zeros(nslots, dtype=torch.uint8, device=dev)
    n_ctr = cl.allreduce_counter_count()
    d_ctr = torch.zeros(max(n_ctr, 1), dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    kev = []  # (start, end) HIP events around each verdict-kernel launch, on its stream
    aev = []  # (start, end) around each counter all-reduce (N > 1), on the same stream

    def step(timed=False, kev=kev, aev=aev):
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        cl.http_verdicts_dev(d_batch, nslots, d_arena, d_out, stream=stream.cuda_stream)
        if timed:
            e1.record(stream)
            kev.append((e0, e1))
        if dist is not None:
            # the only collective: per-rule hits and per-program allowed/
            # denied counters, summed over ranks (RCCL over xGMI)
            cl.counters_copy_dev(d_ctr, n_ctr, stream=stream.cuda_stream)
            if timed:
                a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a0.record(stream)
            with torch.cuda.stream(stream):
                dist.all_reduce(d_ctr)
            if timed:
                a1.record(stream)
                aev.append((a0, a1))

    # parity spot-check of the resident batch (outside the timed region)
    check = None
    if not args.no_check:
        step()
        torch.cuda.synchronize()
        import oracle
        out_tiles = d_out.view(-1, 64)[torch.from_numpy(tile_map).to(dev)]
        slots = out_tiles.reshape(-1).cpu().numpy()  # the first copy, in b's slot order
        got = np.zeros(D, np.uint8)
        real = b.order < D
        got[b.order[real]] = slots[real]
        exp = oracle.HttpOracle(pols).eval(**rq, nthreads=host_threads())
        check = bool(np.array_equal(got, exp))
        if not check:
            raise SystemExit(f"verdicts differ from the oracle on {int((got != exp).sum())} of {D} requests")

    if args.prewarm_seconds > 0:
        run_for(step, args.prewarm_seconds, dist, dev, torch)
    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t_end = time.perf_counter()
    wall = t_end - t_start
    kernel_ms = sum(a.elapsed_time(z) for a, z in kev) / args.steps
    allreduce_ms = sum(a.elapsed_time(z) for a, z in aev) / args.steps if aev else None
    rank_wall = wall
    wall = max_over_ranks(wall, dist, dev, torch)
    sustained = None
    if args.sustain_seconds > 0:
        sustained = sustain(step, args.sustain_seconds, B * world, dist, dev, torch)
    ranks = gather_rank_stats({"kernel_ms": kernel_ms, "allreduce_ms": allreduce_ms, "broadcast_s": bcast_s,
                               "wall_s": rank_wall}, dist, dev, torch)

    total_req = B * world * args.steps
    value = total_req / wall
    ms_per_step = wall / args.steps * 1e3
    # algorithmic bytes: the packed input the launch consumes (tile data +
    # chunk/tile tables; a tile stores its meta unit and the string units of
    # its longest string) + one verdict byte per request
    per_launch_bytes = data_bytes + B * OUT_BYTES
    achieved = per_launch_bytes / (kernel_ms * 1e-3) / 1e9
    allow_frac = float(d_out.float().sum().item()) / B

    host = None
    if not args.no_e2e:
        host = host_entry_fields(cl, rq, got if check else None)
    del rq
    traffic_bytes, traffic_src = pmc_traffic(B)
    # same unit as `achieved`: HBM bytes per launch over the measured launch time
    traffic = traffic_bytes / (kernel_ms * 1e-3) / 1e9 if traffic_bytes else None
    del d_batch, d_arena
    small = None
    if args.small_distinct and args.small_distinct < D:
        small = kernel_on_batch(cl, info, args.small_distinct, args.requests_per_gpu, rank, dev, torch, stream,
                                args.steps, args.warmup, args.layout)
    e2e = None
    if not args.no_e2e:
        os.environ["CILIUM_GPU_RAW_LAYOUT"] = args.e2e_layout
        e2e = end_to_end(cl, pols, info, min(D, 4_194_304), args.requests_per_gpu, rank, dev, torch, stream,
                         args.steps, min(args.warmup, 2), not args.no_check)
        e2e["layout"] = args.e2e_layout
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(pols, info, args.cpu_seconds)
        cpu["best_cpu_dfa"] = cpu_dfa_line(cl, info, min(args.cpu_seconds, 4.0), cpu["cores"])
    if dist is not None:
        dist.barrier()

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "verdicts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm_seconds": args.prewarm_seconds,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: 10K generated PortRuleHTTP rules over 64 ports / 256 selectors of 1K identities; "
                    f"{D} distinct packed requests (50% rule hits, 50% near misses), each program group's tiles "
                    f"repeated to {B} per GPU",
            "config": {"workload": "BASELINE config 5: 10K-rule L7 HTTP set (method/path/host/header regex union "
                                   "DFA), requests sharded across GPUs",
                       "requests_per_gpu": B, "rules": int(stats["rules"]), "programs": int(stats["programs"]),
                       "dfa_states": int(stats["states"]), "table_bytes": int(stats["table_bytes"]),
                       "compile_s": round(compile_s, 3), "distinct_requests": D,
                       "policy_tables": "compiled once on rank 0, the same image imported by every rank",
                       "packed_bytes_per_request": per_launch_bytes / B,
                       "allreduce_counters": n_ctr, "parallelism": f"dp{world}"},
            "request_gbps": value * per_launch_bytes / B / 1e9,
            "allow_fraction": allow_frac,
            "parity_check": check,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                         "kernel": "http_kernel", "kernel_ms": kernel_ms,
                         "bytes_per_launch": per_launch_bytes, "traffic_bytes_per_launch": traffic_bytes,
                         "traffic_source": traffic_src},
            "sustained": sustained,
            "ranks": ranks,
            "distinct_262k": small,
            "end_to_end": e2e,
            "host_entry": host,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    cl.close()


def host_threads() -> int:
    """Host threads given to this GPU's process: OMP_NUM_THREADS (16 on the
    GPU box: its per-GPU CPU share), else the cores here up to 16."""
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)


def max_over_ranks(sec: float, dist, dev, torch) -> float:
    """The job's time: the slowest rank's timed region (all-reduce MAX)."""
    if dist is None or dist.get_world_size() == 1:
        return sec
    tt = torch.tensor([sec], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def run_for(step, seconds: float, dist, dev, torch, **kw) -> tuple:
    """Steps back to back in bursts of 16 until `seconds` have passed on rank
    0's clock (every rank runs the same number: a step may hold a
    collective).  Returns (steps, wall seconds, max over ranks)."""
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while True:
        for _ in range(16):
            step(**kw)
        n += 16
        torch.cuda.synchronize()
        done = torch.tensor([time.perf_counter() - t0 >= seconds], dtype=torch.int32, device=dev)
        if dist is not None:
            dist.broadcast(done, 0)
        if int(done.item()):
            break
    return n, max_over_ranks(time.perf_counter() - t0, dist, dev, torch)


def sustain(step, seconds: float, per_step: int, dist, dev, torch) -> dict:
    """Steps back to back for `seconds` (the driver's timed region is ~30 ms
    of launches): the sustained rate over the whole run and the mean of the
    per-launch HIP events, so a clock drop past the short window would show
    against the headline."""
    kev, aev = [], []
    n, wall = run_for(step, seconds, dist, dev, torch, timed=True, kev=kev, aev=aev)
    ms = [a.elapsed_time(z) for a, z in kev]
    return {"seconds": wall, "steps": n, "value": per_step * n / wall, "unit": "verdicts/s",
            "kernel_ms_mean": float(np.mean(ms)), "kernel_ms_first16": float(np.mean(ms[:16])),
            "kernel_ms_last16": float(np.mean(ms[-16:])), "kernel_ms_max": float(np.max(ms)),
            "allreduce_ms_mean": float(np.mean([a.elapsed_time(z) for a, z in aev])) if aev else None}


RANK_KEYS = ("kernel_ms", "allreduce_ms", "broadcast_s", "wall_s")


def gather_rank_stats(mine: dict, dist, dev, torch) -> list:
    """Per-rank timings at rank 0 (all_gather of RANK_KEYS; None travels as
    NaN): where an N-GPU run loses against linear scaling — the slowest
    kernel, the counter all-reduce, the table image broadcast."""
    vals = [float("nan") if mine.get(k) is None else float(mine[k]) for k in RANK_KEYS]
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    if dist is None or dist.get_world_size() == 1:
        rows = [t]
    else:
        rows = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(rows, t)
    out = []
    for r, row in enumerate(rows):
        d = {"rank": r}
        for k, v in zip(RANK_KEYS, row.cpu().tolist()):
            d[k] = None if v != v else v
        out.append(d)
    return out


def share_policy(cl, pols, dist, rank, dev, torch) -> float:
    """Compile the rules once (rank 0) and give every rank the same compiled
    table image: broadcast over the process group, imported
    without recompiling.  One rank: compile.  Returns the seconds spent on
    the image's broadcast and import (0 for one rank)."""
    if dist is None or dist.get_world_size() == 1:
        cl.update_http_policy(pols)
        return 0.0
    if rank == 0:
        cl.update_http_policy(pols)
        img = np.frombuffer(cl.export_http_policy(), np.uint8)
        size = torch.tensor([img.size], dtype=torch.int64, device=dev)
    else:
        size = torch.zeros(1, dtype=torch.int64, device=dev)
    dist.barrier()  # rank 0's compile is not part of the broadcast
    t0 = time.perf_counter()
    dist.broadcast(size, 0)
    buf = torch.empty(int(size.item()), dtype=torch.uint8, device=dev)
    if rank == 0:
        buf.copy_(torch.from_numpy(img.copy()))
    dist.broadcast(buf, 0)
    if rank != 0:
        cl.import_http_policy(buf.cpu().numpy().tobytes())
    return time.perf_counter() - t0


def host_entry_fields(cl, rq, ref) -> dict:
    """The Envoy-side entry (envoy/cilium_l7policy.cc:127-182): the same
    distinct requests as header lists in HOST memory through
    cg_http_verdicts_fields_host (staged over PCIe in chunks, grouped, sorted
    and packed on the GPU, verdicts copied back), wall clock; bit-exact
    against the device batch's (oracle-checked) verdicts."""
    args_ = (rq["policy"], rq["ingress"], rq["port"], rq["remote"], rq["hdr_blob"], rq["hdr_off"])
    n = len(rq["policy"])
    got = cl.http_verdicts_fields(*args_)  # warm: pinned buffers, workers
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        got = cl.http_verdicts_fields(*args_)
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    list_bytes = int(rq["hdr_off"][-1])
    return {"metric": "verdicts/s through the host entry: header lists in host memory -> verdicts "
                      "(cg_http_verdicts_fields_host, PCIe-inclusive)",
            "value": n / t, "unit": "verdicts/s", "ms": t * 1e3, "requests": n,
            "staged_GBps": (list_bytes + 19 * n) / t / 1e9,
            "parity_check": None if ref is None else bool(np.array_equal(got, ref))}


def kernel_on_batch(cl, info, distinct, per_gpu, rank, dev, torch, stream, steps, warmup, layout) -> dict:
    """The verdict kernel on a batch of `distinct` requests repeated to
    per_gpu (the round-2 bench layout), HIP events on its stream."""
    from cilium_amd import synth
    D = distinct - distinct % 64
    rq = synth.http10k_requests_fast(D, info, seed=synth.SEED ^ (rank * 7919) ^ 0x262)
    b = cl.pack_http(**rq)
    reps = max(1, -(-per_gpu // D))
    d_batch, nslots, _, data_bytes = replicate_batch(b, reps, dev, torch, layout=layout)
    d_arena = torch.from_numpy(np.concatenate([b.arena.view(np.uint8), np.zeros(16, np.uint8)])).to(dev)
    d_out = torch.zeros(nslots, dtype=torch.uint8, device=dev)
    ev = []
    for k in range(warmup + steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        cl.http_verdicts_dev(d_batch, nslots, d_arena, d_out, stream=stream.cuda_stream)
        e1.record(stream)
        if k >= warmup:
            ev.append((e0, e1))
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(z) for a, z in ev) / steps
    B = reps * D
    return {"distinct_requests": D, "requests": B, "kernel_ms": ms, "value": B / (ms * 1e-3),
            "frac": (data_bytes + B) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}


def end_to_end(cl, pols, info, distinct, per_gpu, rank, dev, torch, stream, steps, warmup, check) -> dict:
    """Config 5 as raw HTTP/1.1 request heads resident in HBM (request line,
    Host, the rule's header), per request its policy / ingress / port /
    remote identity and a u64 offset: cg_http_verdicts_raw_dev parses,
    groups, packs and evaluates them on the GPU and writes verdicts in request
    order.  One call per step; the clock is the host's around all steps
    (the device-layout sequence, the default, only enqueues: the steps queue
    back to back on the stream; --e2e-layout host runs the round-3 sequence,
    which waits on the host for the bucket counts between scan and layout).  Checked
    bit-exact against the oracle (codec step oracle/http1_ref.py, then the
    Envoy-faithful rule scan) on a subsample, and every copy against its
    original."""
    from cilium_amd import synth
    D = distinct - distinct % 64
    rq = synth.http10k_requests_fast(D, info, seed=synth.SEED ^ (rank * 7919) ^ 0xE2E, raw=True)
    reps = max(1, -(-per_gpu // D))
    n = D * reps
    blob, off = rq["raw_blob"], rq["raw_off"]
    tot = int(off[-1])
    d_raw = torch.empty(tot * reps, dtype=torch.uint8, device=dev)
    d_raw[:tot].copy_(torch.from_numpy(blob[:tot]))
    done = 1
    while done < reps:
        k = min(done, reps - done)
        d_raw[done * tot:(done + k) * tot].copy_(d_raw[:k * tot])
        done += k
    base = torch.arange(reps, dtype=torch.int64, device=dev).unsqueeze(1) * tot
    d_off = torch.cat([(torch.from_numpy(off[:-1].astype(np.int64)).to(dev).unsqueeze(0) + base).reshape(-1),
                       torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    rep = lambda a, dt: torch.from_numpy(np.asarray(a).astype(dt)).to(dev).repeat(reps)  # noqa: E731
    d_pol, d_ing = rep(rq["policy"], np.int32), rep(rq["ingress"], np.uint8)
    d_port, d_rem = rep(rq["port"].astype(np.int16), np.int16), rep(rq["remote"].astype(np.int32), np.int32)
    d_out = torch.zeros(n, dtype=torch.uint8, device=dev)

    def run():
        cl.http_verdicts_raw_dev(d_raw, d_off, n, d_pol, d_ing, d_port, d_rem, d_out, stream=stream.cuda_stream)
    for _ in range(warmup):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / steps
    parity = None
    if check:
        import oracle
        from oracle.http1_ref import parse_head
        k = min(D, 20_000)
        lists = [parse_head(bytes(blob[int(off[i]):int(off[i + 1])])) for i in range(k)]
        hb, ho = [], [0]
        for lst in lists:
            one = b"".join(a + b"\0" + v + b"\0" for a, v in (lst or []))
            hb.append(one)
            ho.append(ho[-1] + len(one))
        v = oracle.HttpOracle(pols).eval(rq["policy"][:k], rq["ingress"][:k], rq["port"][:k], rq["remote"][:k],
                                         np.frombuffer(b"".join(hb) or b"\0", np.uint8).copy(),
                                         np.asarray(ho, np.uint64), nthreads=host_threads())
        exp = np.where([x is not None for x in lists], v, 0).astype(np.uint8)
        first = d_out[:D]
        same = bool((d_out.view(reps, D) == first.unsqueeze(0)).all())
        parity = bool(np.array_equal(first[:k].cpu().numpy(), exp)) and same
        if not parity:
            raise SystemExit("end-to-end raw-path verdicts differ from the oracle")
    in_bytes = tot * reps + n * (4 + 1 + 2 + 4 + 8)  # heads, policy, ingress, port, remote, offsets
    per_req = (in_bytes + n) / n
    achieved = (in_bytes + n) / sec / 1e9
    return {"metric": "verdicts/s end to end: raw HTTP/1 heads in HBM -> verdicts in request order "
                      "(cg_http_verdicts_raw_dev: codec step, program lookup, packing, http_kernel)",
            "value": n / sec, "unit": "verdicts/s", "ms_per_step": sec * 1e3, "requests": n,
            "distinct_requests": D, "head_bytes_per_request": tot / D, "request_gbps": tot * reps / sec / 1e9,
            "parity_check": parity,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "bytes_per_request": per_req,
                         "note": "algorithmic bytes = the call's inputs + the verdict; the path is bound by its "
                                 "parse and layout kernels, not by HBM (profiles/r03*_raw_kernel_stats.csv)"}}


def rehearse(args):
    """--cpu-rehearsal: the N>1 control flow of main() without a GPU — gloo
    rendezvous on 127.0.0.1, one shard per rank (bench's per-rank seed), the
    shard classified by the library's host table walker (diagnostics, never a
    verdict path), the per-program allowed/denied counters all-reduced, the
    max-over-ranks wall time, and rank 0's single JSON line.  Its value is
    not a measurement (the line says so)."""
    import torch
    import torch.distributed as dist

    from cilium_amd import synth
    from cilium_amd.classifier import Classifier

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    cl = Classifier(device=-1)
    pols, info = synth.http10k_rules(n_rules=2000, n_ports=16)
    bcast_s = share_policy(cl, pols, dist if world > 1 else None, rank, torch.device("cpu"), torch)
    D = max(64, min(args.requests_per_gpu, args.distinct))
    rq = synth.http10k_requests(D, info, seed=synth.SEED ^ (rank * 7919))
    b = cl.pack_http(**rq)
    nprog = int(cl.http_policy_stats()["programs"])
    ctr = torch.zeros(2 * nprog, dtype=torch.int64)

    kt, at = [], []

    def step():
        t0 = time.perf_counter()
        slot_v = cl.http_eval_host_diag_slots(b)
        ctr.add_(torch.from_numpy(program_counts(b, slot_v, nprog)))
        kt.append(time.perf_counter() - t0)
        if world > 1:
            t = ctr.clone()
            t1 = time.perf_counter()
            dist.all_reduce(t)
            at.append(time.perf_counter() - t1)
            return t
        return ctr

    for _ in range(args.warmup):
        step()
    ctr.zero_()
    kt.clear()
    at.clear()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        total = step()
    if world > 1:
        dist.barrier()
    rank_wall = time.perf_counter() - t0
    wall = max_over_ranks(rank_wall, dist if world > 1 else None, torch.device("cpu"), torch)
    ranks = gather_rank_stats({"kernel_ms": 1e3 * float(np.mean(kt)),
                               "allreduce_ms": 1e3 * float(np.mean(at)) if at else None, "broadcast_s": bcast_s,
                               "wall_s": rank_wall}, dist if world > 1 else None, torch.device("cpu"), torch)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": D * world * args.steps / wall, "unit": "verdicts/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "u8", "data": "synthetic",
                          "config": {"workload": "CPU rehearsal of the N-rank path (host table walker, gloo)",
                                     "requests_per_gpu": D, "parallelism": f"dp{world}"},
                          "rehearsal": True, "ranks": ranks,
                          "allreduced_requests": int(total.sum()), "expected_requests": D * world * args.steps}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()
    cl.close()


def program_counts(b, slot_v: np.ndarray, nprog: int) -> np.ndarray:
    """allowed/denied per program from slot verdicts (what the kernel's
    per-program counters hold after one pass over batch b)."""
    hdr = b.batch[:64]
    nchunks = int(hdr[8:12].view(np.uint32)[0])
    chunks = b.batch[64:64 + 16 * nchunks].view(np.uint32).reshape(nchunks, 4)
    c = np.zeros(2 * nprog, np.int64)
    for prog, first, nt, _ in chunks:
        if prog >= nprog:
            continue
        sl = slice(int(first) * 64, int(first + nt) * 64)
        real = b.order[sl] != 0xFFFFFFFF
        v = slot_v[sl][real].astype(np.int64)
        c[2 * prog] += int(v.sum())
        c[2 * prog + 1] += int((1 - v).sum())
    return c


def batch_parts(batch: np.ndarray):
    """Header fields, chunk table and tile table of a packed batch
    (HttpBatchHeader / HttpChunk / HttpTile, csrc/dev_types.h)."""
    h = batch[:64]
    nchunks = int(h[8:12].view(np.uint32)[0])
    ntiles = int(h[12:16].view(np.uint32)[0])
    toff, ttoff = int(h[16:24].view(np.uint64)[0]), int(h[32:40].view(np.uint64)[0])
    chunks = batch[64:64 + 16 * nchunks].view(np.uint32).reshape(nchunks, 4)
    ttab = batch[ttoff:ttoff + 8 * ntiles].view(np.uint32).reshape(ntiles, 2)
    return ntiles, toff, chunks, ttab


def replicate_batch(b, reps: int, dev, torch, return_groups: bool = False, layout: str = "tile"):
    """Device batch of `reps` copies of packed batch b, laid out as the packer
    lays out a batch of reps x D requests: each program's tiles are
    contiguous and cut into chunks of CHUNK_TILES (http_pack.cc).

    layout "tile" (default): within a program group the packer orders the
    whole batch by string units (then content), so a large batch's tiles
    ascend in units across the group; each of b's tiles is placed `reps`
    times in a row, in b's (ascending) tile order.  layout "copy" (round 1)
    repeats b's whole group `reps` times — an ascending run every D requests,
    which no packer produces for one batch.

    Returns (device batch, nslots, tile_map, data_bytes) where tile_map[t] is
    the tile of the first copy of b's tile t and data_bytes the bytes of the
    packed input (tables + tiles).  With return_groups, also [(first tile in
    b, tiles, first tile of the group)] per program group."""
    ntiles, toff, chunks, ttab = batch_parts(b.batch)
    groups = []  # (prog, first tile, ntiles) of each program group of b
    for prog, first, nt, _ in chunks:
        if groups and groups[-1][0] == prog and groups[-1][1] + groups[-1][2] == first:
            groups[-1][2] += int(nt)
        else:
            groups.append([int(prog), int(first), int(nt)])
    kib = ttab[:, 0].astype(np.int64)  # tile offsets in 512-byte granules (HttpTile.at)
    units_field = ttab[:, 1].astype(np.int64)  # HttpTile.units: units | half-last << 15 | last-unit bytes << 16
    units = units_field & 0x7FFF
    half = (units_field >> 15) & 1
    span = 1 + 2 * units - half        # granules per tile: meta block + 1 KiB units (the last one 512 B when half)
    big, new_tt, placed, pos, kpos = [], [], [], 0, 0
    tile_map = np.zeros(ntiles, np.int64)
    for prog, first, nt in groups:
        run = nt * reps
        for k in range(0, run, CHUNK_TILES):
            big.append((prog, pos + k, min(CHUNK_TILES, run - k), 0))
        g_kib = int(kib[first + nt - 1] + span[first + nt - 1] - kib[first])
        rel = kib[first:first + nt] - kib[first]
        if layout == "copy":
            for r in range(reps):
                new_tt.append(np.stack([kpos + r * g_kib + rel, units_field[first:first + nt]], axis=1))
            tile_map[first:first + nt] = np.arange(pos, pos + nt)
        else:
            sp = span[first:first + nt]
            at0 = kpos + np.concatenate([[0], np.cumsum(sp * reps)[:-1]])  # first copy of each tile
            at = (at0[:, None] + np.arange(reps)[None, :] * sp[:, None]).reshape(-1)
            new_tt.append(np.stack([at, np.repeat(units_field[first:first + nt], reps)], axis=1))
            tile_map[first:first + nt] = pos + np.arange(nt) * reps
        placed.append((first, nt, pos, int(kib[first]), g_kib, kpos))
        pos += run
        kpos += reps * g_kib
    big = np.asarray(big, np.uint32)
    new_tt = np.concatenate(new_tt).astype(np.uint32)
    ttoff = 64 + 16 * len(big)
    hbytes = (ttoff + 8 * pos + 1023) // 1024 * 1024
    total = hbytes + kpos * 512
    hdr = b.batch[:64].copy()
    hdr[8:12] = np.array([len(big)], np.uint32).view(np.uint8)
    hdr[12:16] = np.array([pos], np.uint32).view(np.uint8)
    hdr[16:48] = np.array([hbytes, pos * 64, ttoff, total], np.uint64).view(np.uint8)
    head = np.zeros(hbytes, np.uint8)
    head[:64] = hdr
    head[64:64 + big.nbytes] = big.reshape(-1).view(np.uint8)
    head[ttoff:ttoff + new_tt.nbytes] = new_tt.reshape(-1).view(np.uint8)
    d = torch.empty(total, dtype=torch.uint8, device=dev)
    d[:hbytes].copy_(torch.from_numpy(head))
    data_end = int(kib[-1] + span[-1]) * 512 if ntiles else 0
    src = torch.from_numpy(b.batch[toff:toff + data_end]).to(dev)
    for first, nt, at, k0, g_kib, kp in placed:
        g0, gb = hbytes + kp * 512, g_kib * 512
        if layout == "copy":
            d[g0:g0 + gb].copy_(src[k0 * 512:k0 * 512 + gb])
            done = 1
            while done < reps:  # doubling copies on the device
                k = min(done, reps - done)
                d[g0 + done * gb:g0 + (done + k) * gb].copy_(d[g0:g0 + k * gb])
                done += k
        else:
            # granule gather: each tile's granules `reps` times in a row
            gran = src[k0 * 512:k0 * 512 + gb].view(-1, 512)
            rel = kib[first:first + nt] - kib[first]
            sp = span[first:first + nt]
            idx = np.concatenate([np.tile(np.arange(r0, r0 + s), reps) for r0, s in zip(rel, sp)])
            d[g0:g0 + gb * reps].view(-1, 512).copy_(gran[torch.from_numpy(idx).to(dev)])
    if return_groups:
        return d, pos * 64, tile_map, total - 64, [(first, nt, at) for first, nt, at, _, _, _ in placed]
    return d, pos * 64, tile_map, total - 64


def pmc_traffic(requests_per_launch: int):
    """HBM bytes per launch of the verdict kernel from the newest committed
    PMC summary (profiles/r*_http_pmc.json, written by tools/pmc_summary.py
    from separate rocprofv3 --pmc passes of the same workload: FETCH_SIZE ×2
    gfx950 correction + WRITE_SIZE), scaled to this launch's request count.
    rocprofv3 cannot run inside the timed process, hence a committed file."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_http_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        s = json.load(f)
    per_item = s.get("hbm_bytes_per_item")
    if not per_item:
        return None, None
    return per_item * requests_per_launch, os.path.relpath(files[-1], ROOT)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(pols, info, seconds: float) -> dict:
    """Oracle = Envoy's algorithm (per-request PortNetworkPolicy scan with
    std::regex_match) over a 1M-request sample of the same workload, cycled
    for a bounded time on the host cores given to this GPU (its share of the
    node: OMP_NUM_THREADS on the GPU box); plus the same on one core (SURVEY
    8(d))."""
    import oracle
    from cilium_amd import synth
    threads = host_threads()
    orc = oracle.HttpOracle(pols)
    rq = synth.http10k_requests_fast(1_000_000, info, seed=synth.SEED ^ 0xC0FFEE)

    def rate(nthreads, secs, sub):
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < secs:
            orc.eval(**sub, nthreads=nthreads)
            done += len(sub["policy"])
        return done, time.perf_counter() - t0
    done, el = rate(threads, seconds, rq)
    k = 5_000
    one = {key: v[:k] for key, v in rq.items() if key not in ("hdr_blob", "hdr_off")}
    one["hdr_off"], one["hdr_blob"] = rq["hdr_off"][:k + 1], rq["hdr_blob"]
    d1, e1 = rate(1, min(seconds / 4, 3.0), one)
    nproc = os.cpu_count() or threads
    # BASELINE.md's "all host cores": the box gives this process `threads` of
    # the node's hardware threads (running more would oversubscribe the other
    # GPUs' shares), so the whole-node line scales the measured per-thread
    # rate at `threads` threads to nproc — an extrapolation, stated as one
    all_cores = {"value": done / el / threads * nproc, "unit": "verdicts/s", "cores": nproc,
                 "kind": "extrapolated",
                 "note": f"per-thread rate measured on {threads} threads x {nproc} hardware threads; "
                         f"thread scaling 1 -> {threads} measured at "
                         f"{done / el / (d1 / e1) / threads:.2f} of linear"}
    return {"value": done / el, "unit": "verdicts/s", "cores": threads, "kind": "port", "all_cores": all_cores,
            "cpu_model": cpu_model(), "nproc": os.cpu_count(), "single_core": d1 / e1,
            "cores_note": f"the host threads given to this GPU's process ({threads}: its share of the node's "
                          f"{os.cpu_count()} hardware threads); a node's 8 GPUs' shares run 8 such baselines",
            "sample": f"{done} requests ({done / 1e6:.1f}M: a 1M-request sample of the same 10K-rule workload "
                      f"cycled, {el:.1f} s, {threads} threads, std::regex_match per matcher as Envoy); "
                      f"single core: {d1} requests in {e1:.1f} s"}


def cpu_dfa_line(cl, info, seconds: float, threads: int) -> dict:
    """"Best CPU" line: the engine's own compiled union DFAs
    walked on the host (cg_diag_http_eval_host — the table compilers' CPU
    walker, never a verdict entry point), one packed batch per thread."""
    from concurrent.futures import ThreadPoolExecutor

    from cilium_amd import synth
    per = 65_536
    batches = [cl.pack_http(**synth.http10k_requests_fast(per, info, seed=synth.SEED ^ (0xD0 + t)))
               for t in range(threads)]
    cl.http_eval_host_diag(batches[0])
    t1 = time.perf_counter()
    cl.http_eval_host_diag(batches[0])
    single = per / (time.perf_counter() - t1)
    with ThreadPoolExecutor(threads) as ex:
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            list(ex.map(cl.http_eval_host_diag, batches))
            done += per * threads
        el = time.perf_counter() - t0
    return {"value": done / el, "unit": "verdicts/s", "cores": threads, "single_core": single,
            "sample": f"{done} requests: comb-table DFA walk of the packed batches on the host ({el:.1f} s)"}


if __name__ == "__main__":
    main()
