"""Config 3 prefilter with the IPv4 and IPv6 halves launched separately
(one lpm_kernel dispatch each, 3 repeats), so a rocprofv3 pass attributes
traffic per family.  Measuring driver only.

    python tools/lpm_split.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from cilium_amd import synth
    from cilium_amd.classifier import Classifier
    dev = torch.device("cuda", 0)
    cl = Classifier(device=0)
    pfx = synth.lpm_prefixes()
    pf = cl.prefilter(dyn4=True, dyn6=True, max_lpm=1 << 21)
    pf.insert(0, pfx)
    v4, v6, ep4, ep6 = synth.lpm_addresses(100_000_000, pfx)
    pf.set_endpoints(ep4, ep6)
    d4 = torch.from_numpy(np.ascontiguousarray(v4)).to(dev)
    d6 = torch.from_numpy(np.ascontiguousarray(v6)).to(dev)
    o4 = torch.empty(len(v4), dtype=torch.uint8, device=dev)
    o6 = torch.empty(len(v6), dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream()
    for fam, run in (("v4", lambda: pf.verdicts_dev(d4, len(v4), o4, d6, 0, o6, stream=st.cuda_stream)),
                     ("v6", lambda: pf.verdicts_dev(d4, 0, o4, d6, len(v6), o6, stream=st.cuda_stream))):
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        n = len(v4) if fam == "v4" else len(v6)
        print(fam, n, "G/s", n * 3 / (time.perf_counter() - t0) / 1e9, flush=True)


if __name__ == "__main__":
    main()
