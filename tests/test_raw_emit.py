"""The device-layout raw sequence's string emitter (csrc/raw_emit.h TileOut,
used by raw_scan_dl_kernel / raw_defer_dl_kernel) run on the CPU: the header
is host+device, so tests/native/tileout_test.cc builds it with hipcc's host
compiler and checks 20,000 random byte runs — fed as the scan feeds them —
against the plain construction (bytes through the code map, 16-byte units a
tile row apart, zero padding after the string, nothing past the last unit)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tileout_emission_on_host(tmp_path):
    hipcc = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)
    if hipcc is None:
        pytest.skip("no hipcc")
    exe = str(tmp_path / "tileout_test")
    subprocess.run([hipcc, "-x", "hip", "--cuda-host-only", "-O2", "-std=c++17",
                    "-I", os.path.join(ROOT, "cilium_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "tileout_test.cc"), "-o", exe],
                   check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "tileout ok" in r.stdout
