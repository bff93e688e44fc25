"""The N>1 path on CPU: two ranks over gloo (127.0.0.1), each classifying
its own shard of the 10K-rule workload (per-rank seed as in bench.py) with
the engine's compiled tables (the library's host walker: no GPU here), then
all-reducing the counter vector — per-program allowed/denied and per-rule
first-match hits, the only collective on this path — and
`bench.py --gpus 2` spawning its own ranks (--cpu-rehearsal)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _per_program_counts(cl, b, verdicts_by_slot, nprog):
    """allowed/denied per program from slot verdicts (what the kernel counts)."""
    hdr = b.batch[:64]
    nchunks = int(hdr[8:12].view(np.uint32)[0])
    chunks = b.batch[64:64 + 16 * nchunks].view(np.uint32).reshape(nchunks, 4)
    c = np.zeros(2 * nprog, np.int64)
    for prog, first, nt, _ in chunks:
        if prog >= nprog:
            continue
        sl = slice(int(first) * 64, int(first + nt) * 64)
        real = b.order[sl] != 0xFFFFFFFF
        v = verdicts_by_slot[sl][real]
        c[2 * prog] += int(v.sum())
        c[2 * prog + 1] += int((1 - v).sum())
    return c


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from cilium_amd import synth
        from cilium_amd.classifier import Classifier
        cl = Classifier(device=-1)
        pols, info = synth.http10k_rules(n_rules=2000, n_ports=16)
        cl.update_http_policy(pols)
        rq = synth.http10k_requests(4096, info, seed=synth.SEED ^ (rank * 7919))  # bench.py's shard seed
        b = cl.pack_http(**rq)
        # the engine's tables walked on the host (the GPU kernel's walk); the
        # oracle only checks them
        slot_v = cl.http_eval_host_diag_slots(b).astype(np.int64)
        rules = cl.http_rules_host_diag(b)
        exp = oracle.HttpOracle(pols).eval(**rq)
        assert np.array_equal(cl.http_eval_host_diag(b), exp)
        nprog = cl.http_policy_stats()["programs"]
        hits = np.bincount(rules[rules != 0xFFFFFFFF], minlength=len(cl.http_rule_info())).astype(np.int64)
        mine = np.concatenate([_per_program_counts(cl, b, slot_v, nprog), [0], hits])
        t = torch.from_numpy(mine.copy())
        dist.all_reduce(t)
        gathered = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(mine.copy()))
        ok = bool(torch.equal(t, sum(gathered))) and int(t[:2 * nprog].sum()) == 4096 * world
        ok = ok and int(t[2 * nprog + 1:].sum()) == int(t[0:2 * nprog:2].sum())  # every allow attributed
        q.put((rank, ok, int(t[:2 * nprog].sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_counter_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(ok for _, ok, _ in res), res
    assert all(total == 8192 for _, _, total in res)


@pytest.mark.timeout(300)
def test_bench_spawns_two_ranks_cpu_rehearsal():
    """`bench.py --gpus 2` starts its own two ranks (no launcher), which meet
    over gloo on 127.0.0.1, all-reduce the counters and print ONE line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--cpu-rehearsal",
                        "--steps", "2", "--warmup", "1", "--requests-per-gpu", "2048"],
                       capture_output=True, text=True, timeout=280, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["rehearsal"] is True
    assert d["allreduced_requests"] == d["expected_requests"] == 2048 * 2 * 2
    # per-rank diagnostics (bench.gather_rank_stats): one row per rank, every
    # rank timed its shard, its counter all-reduce and the image broadcast
    assert [r["rank"] for r in d["ranks"]] == [0, 1]
    for r in d["ranks"]:
        assert r["kernel_ms"] > 0 and r["allreduce_ms"] is not None and r["allreduce_ms"] >= 0
        assert r["broadcast_s"] >= 0 and r["wall_s"] > 0
    assert abs(max(r["wall_s"] for r in d["ranks"]) - d["ms_per_step"] * d["steps"] / 1e3) < 1e-6


def _bench_collectives_worker(rank, world, port, q):
    """bench.py's own collectives on gloo: share_policy (rank 0 compiles, the
    image's size and bytes broadcast, the other ranks import it) and
    max_over_ranks (the job time = the slowest rank's)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import hashlib
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        from cilium_amd import synth
        from cilium_amd.classifier import Classifier
        cl = Classifier(device=-1)
        pols, info = synth.http10k_rules(n_rules=1500, n_ports=16)
        bench.share_policy(cl, pols, dist, rank, torch.device("cpu"), torch)
        img = cl.export_http_policy()
        h = torch.tensor(list(hashlib.sha256(img).digest()), dtype=torch.uint8)
        hs = [torch.zeros_like(h) for _ in range(world)]
        dist.all_gather(hs, h)
        same_image = all(torch.equal(x, hs[0]) for x in hs)
        # every rank decides the same sample with its (imported) tables
        rq = synth.http10k_requests(2048, info, seed=99)
        v = torch.from_numpy(cl.http_eval_host_diag(cl.pack_http(**rq)).astype(np.int64))
        vs = [torch.zeros_like(v) for _ in range(world)]
        dist.all_gather(vs, v)
        same_verdicts = all(torch.equal(x, vs[0]) for x in vs)
        wall = bench.max_over_ranks(0.5 + rank, dist, torch.device("cpu"), torch)
        one = bench.max_over_ranks(0.25, None, torch.device("cpu"), torch)
        rows = bench.gather_rank_stats({"kernel_ms": 1.0 + rank, "allreduce_ms": None if rank == 1 else 0.5,
                                        "broadcast_s": 0.1 * rank, "wall_s": 2.0}, dist, torch.device("cpu"), torch)
        rows_ok = rows == [{"rank": r, "kernel_ms": 1.0 + r, "allreduce_ms": None if r == 1 else 0.5,
                            "broadcast_s": 0.1 * r, "wall_s": 2.0} for r in range(world)]
        q.put((rank, same_image and rows_ok, same_verdicts, wall, one))
        cl.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bench_collectives_image_broadcast_and_max_time():
    """Every collective bench.py issues besides the counter all-reduce
    (covered above): the compiled image broadcast, the max-over-ranks time
    and the per-rank timing gather, on 3 gloo ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_bench_collectives_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
    assert [r for r, *_ in res] == [0, 1, 2]
    assert all(img and ver for _, img, ver, _, _ in res), res
    assert all(w == 2.5 and one == 0.25 for *_, w, one in res), res
