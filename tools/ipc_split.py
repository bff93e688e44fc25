"""ipcache with the IPv4 and IPv6 halves launched
separately (one ipcache_kernel dispatch each, 3 repeats), so a kernel trace
or a rocprofv3 pass attributes time and traffic per family.  Measuring
driver only.  CILIUM_AMD_LIB selects a variant library.

    python tools/ipc_split.py
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
    k, v = synth.ipcache_entries()
    ic = cl.ipcache()
    ic.update(k, v)
    a4, a6 = synth.ipcache_addresses(100_000_000, k)
    d4 = torch.from_numpy(np.ascontiguousarray(a4)).to(dev)
    d6 = torch.from_numpy(np.ascontiguousarray(a6)).to(dev)
    o4 = torch.empty(len(a4) * 2, dtype=torch.int32, device=dev)
    o6 = torch.empty(len(a6) * 2, dtype=torch.int32, device=dev)
    st = torch.cuda.Stream()
    for fam, run in (("v4", lambda: ic.resolve_dev(d4, len(a4), o4, d6, 0, o6, stream=st.cuda_stream)),
                     ("v6", lambda: ic.resolve_dev(d4, 0, o4, d6, len(a6), o6, stream=st.cuda_stream))):
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        n = len(a4) if fam == "v4" else len(a6)
        print(fam, n, "G/s", n * 3 / (time.perf_counter() - t0) / 1e9, flush=True)


if __name__ == "__main__":
    main()
