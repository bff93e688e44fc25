"""ASan + UBSan build of libciliumgpu.so for the CPU (host) code paths.

Every translation unit of cilium_amd/build.py, compiled by hipcc with the
sanitizers on the host side only (`-Xarch_host -fsanitize=...`: device code
is not instrumented — GPU sanitizers are not available on this pool), linked
into tools/sanitize/_build/libciliumgpu_asan.so.  tools/sanitize/run.sh loads
it through CILIUM_AMD_LIB with the ASan runtime preloaded and runs the CPU
test suite and a bounded fuzz of the parsers that consume untrusted bytes.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
from cilium_amd import build as B  # noqa: E402

OUT = HERE / "_build"
LIB = OUT / "libciliumgpu_asan.so"
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
       "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer"]


def compile_one(src: str) -> Path:
    obj = OUT / (src + ".o")
    flags = [f for f in B._flags(src) if f != "-O3"] + ["-O1", "-g"] + SAN
    cmd = [B.HIPCC, *flags, "-I", str(B.CSRC), "-I", str(ROOT / "include"), "-c", str(B.CSRC / src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def main() -> None:
    OUT.mkdir(exist_ok=True)
    with cf.ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, B.SOURCES))
    cmd = [B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *map(str, objs), "-o", str(LIB), "-lpthread", "-lz",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-shared-libasan"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    print(LIB)


if __name__ == "__main__":
    main()
