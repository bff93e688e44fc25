"""Kafka wire decode under a profiler: config 4's mix as wire bytes (the
bench_paths.py kafkawire workload), --iters decode launches, nothing else
timed.  python tools/prof_kw.py [--reps 256] [--iters 3]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=256)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import torch
    from bench_paths import kafka_wire_pool, tile_dev
    from cilium_amd import kafka_requests as K
    from cilium_amd import synth
    from cilium_amd.classifier import Classifier
    dev = torch.device("cuda", 0)
    cl = Classifier(device=0)
    pols, info = synth.kafka_policy()
    cl.update_kafka_policy(pols)
    D = 65_536
    pool, rq = kafka_wire_pool(D, info)
    raw, off = K.concat(pool)
    tot, reps = int(off[-1]), a.reps
    d_raw = tile_dev(torch, raw, reps, dev)
    offs = torch.from_numpy(off[:-1].view(np.int64).copy()).to(dev)
    d_off = (offs.unsqueeze(0) + torch.arange(reps, device=dev, dtype=torch.int64).unsqueeze(1) * tot).reshape(-1)
    d_off = torch.cat([d_off, torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    n = D * reps
    d_red = torch.zeros(n, dtype=torch.int16, device=dev)
    d_rem = torch.from_numpy(np.asarray(rq["remote"], np.uint32).view(np.int32)).to(dev).repeat(reps)
    d_reqs = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    cap = tot * reps // 2 + 16
    d_a = torch.empty(cap, dtype=torch.int32, device=dev)
    for _ in range(a.iters):
        cl.kafka_decode_dev(d_raw, d_off, n, d_red, d_rem, d_reqs, d_a, cap, d_st)
    torch.cuda.synchronize()
    print("requests", n, "bytes", tot * reps)
    cl.close()


if __name__ == "__main__":
    main()
