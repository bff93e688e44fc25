"""Per-kernel PMC sums (per dispatch) of a tools/gpu_raw_ab.sh run.

    python tools/raw_pmc_summary.py gpurun_out/<tag>
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    d = sys.argv[1]
    for f in ("masks", "bytes"):
        p = os.path.join(d, f + ".jsonl")
        if os.path.exists(p):
            lines = open(p).read().strip().splitlines()
            if lines:
                x = json.loads(lines[-1])
                print(f, round(x["value"] / 1e9, 3), "G/s", round(x["ms_per_launch"], 2), "ms")
    for run in sorted(glob.glob(os.path.join(d, "p*", "p*", "run_counter_collection.csv"))):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(run)):
            m = re.search(r"(raw_\w+|http_kernel)", r["Kernel_Name"])
            if m:
                agg[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[m.group(1)].add(r["Dispatch_Id"])
        print(os.path.relpath(run, d))
        for k, v in agg.items():
            print("  ", k, {c: round(x / len(disp[k]) / 1e6, 2) for c, x in v.items()})


if __name__ == "__main__":
    main()
