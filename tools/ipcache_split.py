"""ipcache_kernel split by family and by chunk encoding (GPU box).

Times cg_ipcache_resolve_dev on the bench's 512K-entry table (synth) over
100M addresses (70% v4) as bench_paths.py's ipcache line does, then the v4
and v6 addresses alone (2 v4 addresses per lane, the default), then the
mix at 4 per lane and the v4 addresses at 3 and 4 per lane
(CILIUM_GPU_IPC_K); with --encode the builder writes run lines and sparse
maps (CILIUM_GPU_IPC_ENCODE, set before the library loads), the encoding A/B.
One JSON line per leg."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--encode", action="store_true", help="run lines / sparse maps (CILIUM_GPU_IPC_ENCODE)")
    ap.add_argument("--addresses", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    if args.encode:
        os.environ["CILIUM_GPU_IPC_ENCODE"] = "1"
    import numpy as np
    import torch
    from cilium_amd import synth
    from cilium_amd.classifier import Classifier
    from tools.bench_paths import timed
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    cl = Classifier(device=0)
    k, v = synth.ipcache_entries()
    ic = cl.ipcache()
    ic.update(k, v)
    a4, a6 = synth.ipcache_addresses(args.addresses, k)
    d4 = torch.from_numpy(a4.view(np.uint8)).to(dev)
    d6 = torch.from_numpy(a6.reshape(-1)).to(dev)
    n4, n6 = len(a4), len(a6)
    o4 = torch.empty(n4 * 2, dtype=torch.int32, device=dev)
    o6 = torch.empty(n6 * 2, dtype=torch.int32, device=dev)
    legs = [("both", n4, n6, "2"), ("v4", n4, 0, "2"), ("v6", 0, n6, "2"), ("both", n4, n6, "4"), ("v4", n4, 0, "3"),
            ("v4", n4, 0, "4")]
    for leg, m4, m6, k4 in legs:
        os.environ["CILIUM_GPU_IPC_K"] = k4  # read by the launcher on each call
        sec = timed(torch, stream, lambda: ic.resolve_dev(d4, m4, o4, d6, m6, o6, stream=stream.cuda_stream),
                    args.steps, 2)
        print(json.dumps({"leg": leg, "encoding": "encoded" if args.encode else "dense", "v4_per_lane": int(k4),
                          "v4": m4, "v6": m6, "ms": round(sec * 1e3, 3),
                          "G_lookups_per_s": round((m4 + m6) / sec / 1e9, 2)}), flush=True)
    os.environ.pop("CILIUM_GPU_IPC_K")
    cl.close()


if __name__ == "__main__":
    main()
