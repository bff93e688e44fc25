"""Build libciliumgpu.so (HIP kernels + C++ runtime) in-tree for gfx950.

Plain hipcc invocations (no cmake, no JIT cache): every translation unit is
compiled to an object next to the sources' build dir, then linked into
``cilium_amd/libciliumgpu.so``.  Objects are rebuilt when the source or any
header in csrc/ is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE / "_build"
LIB = HERE / "libciliumgpu.so"
ARCH = "gfx950"

SOURCES = ["runtime.cc", "regex.cc", "regex_go.cc", "clsdfa.cc", "comb.cc", "http.cc", "l4.cc", "lpm.cc", "ipcache.cc", "kafka.cc", "http_pack.cc", "capi.cc", "proxylib_shim.cc", "proxylib_memcache.cc", "proxylib_cassandra.cc", "npds_pb.cc", "http_parse.cc", "http_raw.cc", "http_image.cc", "kafka_wire.cc", "ring.cc",
           "kernels.hip", "kernels_http.hip", "kernels_ipcache.hip", "kernels_kafka.hip", "kernels_http_raw.hip"]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _flags(src: str) -> list[str]:
    common = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
              "-Wno-unused-but-set-variable"]
    if src.endswith(".hip"):
        return common + [f"--offload-arch={ARCH}", "-x", "hip", "-munsafe-fp-atomics"]
    # host-only C++ translation units
    return common + ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]


def _newest_header() -> float:
    return max((p.stat().st_mtime for p in list(CSRC.glob("*.h")) +
                [HERE.parent / "include" / "cilium_gpu.h"]), default=0.0)


def _compile(src: str, force: bool) -> Path:
    obj = BUILD / (src + ".o")
    s = CSRC / src
    if not force and obj.exists() and obj.stat().st_mtime >= max(s.stat().st_mtime, _newest_header()):
        return obj
    cmd = [HIPCC, *_flags(src), "-I", str(CSRC), "-I", str(HERE.parent / "include"), "-c", str(s), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> Path:
    BUILD.mkdir(exist_ok=True)
    jobs = min(len(SOURCES), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(LIB),
               "-lpthread", "-lz", "-lhsa-runtime64"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
