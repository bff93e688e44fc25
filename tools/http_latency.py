"""Envoy-shaped HTTP verdict latency (tools/http_latency.cc): writes a pool of
config-5 header lists (the 10K-rule set) into a directory, computes the
pool's verdicts through the engine in one batch, checks a subsample against
the oracle (Envoy-faithful rule scan), then runs the C driver, which times
cg_http_ring_verdicts (the persistent ring), cg_http_verdicts_fields_host and
cg_http_pack + cg_http_verdicts_host at batch
sizes 1 … 64K from 1 and 16 threads (one JSON line per point).

    python tools/http_latency.py [--pool N] [--seconds S] [--out DIR]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=1 << 20)
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--entries", default="ring,fields,pack", help="entries to time (ring, fields, pack)")
    args = ap.parse_args()
    import oracle
    from cilium_amd import synth
    from cilium_amd.classifier import Classifier
    pols, info = synth.http10k_rules()
    rq = synth.http10k_requests_fast(args.pool, info, seed=synth.SEED ^ 0x1A7)
    d = args.out or tempfile.mkdtemp(prefix="cg_lat_")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "policy.json"), "w") as f:
        json.dump(pols, f)
    n = len(rq["policy"])
    arrs = {"blob": (rq["hdr_blob"], np.uint8), "off": (rq["hdr_off"], np.uint64), "pol": (rq["policy"], np.uint32),
            "ing": (rq["ingress"], np.uint8), "port": (rq["port"], np.uint16), "rem": (rq["remote"], np.uint32)}
    for k, (a, dt) in arrs.items():
        np.ascontiguousarray(a, dt).tofile(os.path.join(d, k + ".bin"))
    # the pool's verdicts in one batch, a subsample checked against the oracle
    # (the calls of the C driver are checked against these)
    cl = Classifier(device=0)
    cl.update_http_policy(pols)
    args_ = (rq["policy"], rq["ingress"], rq["port"], rq["remote"], rq["hdr_blob"], rq["hdr_off"])
    want = cl.http_verdicts(cl.pack_http(*args_))
    cl.close()
    k = 20_000
    exp = oracle.HttpOracle(pols).eval(*(np.asarray(a)[:k] for a in args_[:4]), rq["hdr_blob"], rq["hdr_off"][:k + 1],
                                       nthreads=16)
    if not np.array_equal(want[:k], exp):
        raise SystemExit("pool verdicts differ from the oracle")
    want.astype(np.uint8).tofile(os.path.join(d, "want.bin"))
    print(json.dumps({"pool": n, "dir": d, "oracle_checked": k, "allow_frac": float(want.mean())}), flush=True)
    exe = os.path.join(ROOT, "tools", "http_latency")
    rc = subprocess.call([exe, d, str(args.seconds), args.entries])
    sys.exit(rc)


if __name__ == "__main__":
    main()
