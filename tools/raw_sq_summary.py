"""SQ counter pass (tools/gpu_raw_pmc.sh) → per-kernel JSON summary of the raw
HTTP path kernels: per-dispatch means, VALU instructions per request, wave
wait fraction.

    python tools/raw_sq_summary.py gpurun_out/<tag> --requests N --out profiles/<name>.json
"""
import argparse
import collections
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--requests", type=int, default=124518400)
ap.add_argument("--out", required=True)
a = ap.parse_args()
rows = list(csv.DictReader(open(f"{a.dir}/p1/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
res = {}
for r in rows:
    k = r["Kernel_Name"].replace("void ", "").replace("cg::(anonymous namespace)::", "").split("(")[0]
    if not k.startswith("raw_"):
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
    res[k] = {"VGPR_Count (rocprof units)": r["VGPR_Count"], "Grid_Size": r["Grid_Size"],
              "Workgroup_Size": r["Workgroup_Size"], "LDS_Block_Size": r["LDS_Block_Size"]}
out = {"source": f"rocprofv3 --pmc SQ counters, one pass ({a.dir}); per-dispatch means over the run's dispatches",
       "requests_per_dispatch": a.requests, "kernels": {}}
for k, v in agg.items():
    d = {c: v[c] / cnt[(k, c)] for c in v}
    e = {"counters_per_dispatch": d, "resources": res[k]}
    if d.get("SQ_WAVE_CYCLES"):
        e["wave_wait_fraction"] = d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VALU" in d:
        e["valu_wave_insts_per_64_requests"] = d["SQ_INSTS_VALU"] / a.requests * 64
    out["kernels"][k] = e
json.dump(out, open(a.out, "w"), indent=1)
for k, e in out["kernels"].items():
    print(k, round(e.get("valu_wave_insts_per_64_requests", 0), 1), round(e.get("wave_wait_fraction", 0), 3))
