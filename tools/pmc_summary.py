"""Summarize rocprofv3 PMC passes (tools/gpu_pmc.sh output) for one kernel:
per-dispatch averages of every counter, HBM traffic with the gfx950
FETCH_SIZE correction (MI355X_MICROARCH.md "HBM": FETCH_SIZE reports half of
the bytes of 16-B/lane streaming reads), LDS bank-conflict rate.

    python tools/pmc_summary.py gpurun_out/<tag> [--kernel http_kernel] [--items N] [--out profiles/x.json]
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="http_kernel")
    ap.add_argument("--items", type=int, default=0, help="items (requests) per dispatch")
    ap.add_argument("--algo-bytes", type=float, default=0.0, help="algorithmic bytes per item")
    ap.add_argument("--out", default="")
    ap.add_argument("--last", type=int, default=0, help="only the last N dispatches of the kernel")
    ap.add_argument("--workload", default="", help="what the profiled command ran (recorded in the summary)")
    a = ap.parse_args()
    per = collections.defaultdict(list)
    resources = {}
    for f in sorted(glob.glob(os.path.join(a.dir, "p*", "run_counter_collection.csv"))):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            # "kernel" matches the kernel and its template instances unless
            # it names one ("http_kernel" ⊇ "http_kernel<false>")
            if f"::{a.kernel}(" not in name and ("<" in a.kernel or f"::{a.kernel}<" not in name):
                continue
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            resources = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size",
                                           "VGPR_Count", "SGPR_Count")}
        if a.last:
            keep = set(sorted({int(d) for d, _ in agg}, key=int)[-a.last:])
            agg = {k: v for k, v in agg.items() if int(k[0]) in keep}
        for (_, c), v in agg.items():
            per[c].append(v)
    avg = {c: sum(v) / len(v) for c, v in per.items()}
    out = {"kernel": a.kernel, "counters_per_dispatch": avg, "dispatches": {c: len(v) for c, v in per.items()},
           "resources": resources, "workload": a.workload, "items_per_dispatch": a.items}
    if "FETCH_SIZE" in avg:
        fetch = avg["FETCH_SIZE"] * 1024 * 2  # KB → B, ×2 gfx950 streaming-read correction
        write = avg.get("WRITE_SIZE", 0.0) * 1024
        out["hbm_bytes_per_dispatch"] = fetch + write
        out["fetch_bytes_corrected"] = fetch
        out["write_bytes"] = write
        if a.items:
            out["hbm_bytes_per_item"] = (fetch + write) / a.items
    if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_rate"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
    if "SQ_WAIT_ANY" in avg and avg.get("SQ_WAVE_CYCLES"):
        out["wave_wait_fraction"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
    if a.items and a.algo_bytes:
        out["algorithmic_bytes_per_dispatch"] = a.items * a.algo_bytes
    s = json.dumps(out, indent=1, sort_keys=True)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
