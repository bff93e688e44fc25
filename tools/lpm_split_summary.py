"""Summarise a tools/gpu_lpm_split.sh run: per-family FETCH bytes and L2
hits/misses per address (FETCH_SIZE KB x 1024 x 2, the gfx950 correction).

    python tools/lpm_split_summary.py gpurun_out/ls2 [kernel]
"""
import collections
import csv
import os
import sys

KERNEL = "lpm"


def per_dispatch(path):
    d = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            d[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
    out = collections.defaultdict(list)
    for (dsp, c), v in sorted(d.items()):
        out[c].append(v)
    return out


def main(root):
    f = per_dispatch(os.path.join(root, "pf", "run_counter_collection.csv"))
    h = per_dispatch(os.path.join(root, "ph", "run_counter_collection.csv"))
    n = {"v4": 70e6, "v6": 30e6}
    for k, fam in enumerate(("v4", "v6")):
        sl = slice(4 * k, 4 * k + 4)
        fetch = sum(f["FETCH_SIZE"][sl]) / 4 * 1024 * 2
        hit = sum(h["TCC_HIT_sum"][sl]) / 4
        miss = sum(h["TCC_MISS_sum"][sl]) / 4
        print(f"{fam}: FETCH {fetch / 1e9:.3f} GB/dispatch = {fetch / n[fam]:.1f} B/addr, "
              f"TCC hit {hit / 1e6:.1f}M miss {miss / 1e6:.1f}M = {miss / n[fam]:.2f} miss/addr")


if __name__ == "__main__":
    if len(sys.argv) > 2:  # kernel name fragment, e.g. ipcache (tools/ipc_split.py: same 70M / 30M split)
        KERNEL = sys.argv[2]
    main(sys.argv[1])
