"""Profiling driver: the bench's HTTP workload without the oracle / CPU legs,
for rocprofv3 passes (kernel trace, PMC counters).

    python tools/prof_http.py [--requests N] [--iters K] [--digest FILE]

--digest: the SHA-256 of the verdict array after the timed loop is written
to FILE when it does not exist, else compared with it (exit 1 on a
mismatch): the main library's run writes it, kernel variants selected with
CILIUM_AMD_LIB must reproduce it.
"""
import hashlib
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=32_000_000)
    ap.add_argument("--distinct", type=int, default=262_144)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--digest", default=None)
    ap.add_argument("--workload", default="http10k", choices=["http10k", "starwars"])
    args = ap.parse_args()
    import torch

    import bench
    from cilium_amd import synth
    from cilium_amd.classifier import Classifier
    dev = torch.device("cuda", 0)
    cl = Classifier(device=0)
    if args.workload == "http10k":
        pols, info = synth.http10k_rules()
        cl.update_http_policy(pols)
        rq = synth.http10k_requests(args.distinct, info)
    else:
        pols = synth.starwars_policy()
        cl.update_http_policy(pols)
        rq = synth.starwars_requests(args.distinct)
    b = cl.pack_http(**rq)
    reps = max(1, args.requests // args.distinct)
    d_batch, nslots, _, _ = bench.replicate_batch(b, reps, dev, torch)
    d_arena = torch.from_numpy(b.arena).to(dev)
    d_out = torch.zeros(nslots, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.iters):
        cl.http_verdicts_dev(d_batch, nslots, d_arena, d_out)
    cl.sync()
    el = time.perf_counter() - t
    n = reps * args.distinct
    print(f"{args.workload}: {n} requests x {args.iters}: {el / args.iters * 1e3:.3f} ms/iter, "
          f"{n * args.iters / el / 1e9:.3f} G verdicts/s")
    rc = 0
    if args.digest:
        h = hashlib.sha256(d_out.cpu().numpy().tobytes()).hexdigest()
        if os.path.exists(args.digest):
            old = open(args.digest).read().strip()
            rc = 0 if old == h else 1
            print(f"digest {h[:16]} {'matches' if rc == 0 else 'DIFFERS from ' + old[:16]}")
        else:
            with open(args.digest, "w") as f:
                f.write(h + "\n")
            print(f"digest {h[:16]} written")
    cl.close()
    return rc


if __name__ == "__main__":
    sys.exit(main())
