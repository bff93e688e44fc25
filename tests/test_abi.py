"""The C ABI: the library loads, exports every symbol include/cilium_gpu.h
declares, and a host-only handle refuses every verdict call (no CPU
fallback) while still compiling policies."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from cilium_amd import _native as N
from cilium_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "cilium_gpu.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cg_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    names = declared_functions()
    assert len(names) > 40
    lib = C.CDLL(str(N.LIB_PATH))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding declares a signature for each of them
    assert not [n for n in names if n not in N.SIGNATURES]


def test_version_and_errors():
    assert N.lib.cg_version().startswith(b"libciliumgpu gfx950")
    assert N.lib.cg_sync(987654321) == N.CG_INVALID_INSTANCE
    assert b"unknown handle" in N.lib.cg_last_error()


def test_host_handle_refuses_verdicts(host):
    host.update_http_policy(synth.starwars_policy())
    rq = synth.starwars_requests(100)
    b = host.pack_http(**rq)
    with pytest.raises(N.CiliumGPUError) as ei:
        host.http_verdicts(b)
    assert ei.value.code == N.CG_NO_DEVICE
    pm = host.policy_map()
    pm.allow(1, 80, 6, 0, 0)
    from cilium_amd.classifier import L4_TUPLE_DTYPE
    with pytest.raises(N.CiliumGPUError) as ei:
        pm.verdicts(np.zeros(4, L4_TUPLE_DTYPE))
    assert ei.value.code == N.CG_NO_DEVICE
    pf = host.prefilter()
    with pytest.raises(N.CiliumGPUError) as ei:
        pf.verdicts(np.zeros((1, 2), np.uint32), np.zeros((0, 32), np.uint8))
    assert ei.value.code == N.CG_NO_DEVICE


def test_struct_layouts():
    from cilium_amd.classifier import CIDR_DTYPE, KAFKA_REQ_DTYPE, L4_TUPLE_DTYPE, POLICY_KEY_DTYPE
    assert POLICY_KEY_DTYPE.itemsize == 8          # struct policy_key, bpf/lib/common.h:180-186
    assert C.sizeof(N.PolicyEntryC) == 24          # struct policy_entry, common.h:188-193
    assert L4_TUPLE_DTYPE.itemsize == 12
    assert CIDR_DTYPE.itemsize == 20
    assert KAFKA_REQ_DTYPE.itemsize == 64


def test_policy_update_is_all_or_nothing(host):
    host.update_http_policy(synth.starwars_policy())
    before = host.http_policy_stats()
    bad = synth.starwars_policy()
    bad[0]["egress_per_port_policies"][0]["rules"][0]["http_rules"]["http_rules"][0]["headers"][0]["regex_match"] = \
        "(unclosed"
    with pytest.raises(N.CiliumGPUError) as ei:
        host.update_http_policy(bad)
    assert ei.value.code == N.CG_POLICY_REJECTED
    assert host.http_policy_stats() == before  # the previous snapshot keeps serving
    with pytest.raises(N.CiliumGPUError) as ei:
        host.update_http_policy(b"[{]")
    assert ei.value.code == N.CG_POLICY_REJECTED


def test_unsupported_regex_constructs(host):
    """std::regex accepts these and a DFA cannot express them; everything
    else std::regex accepts compiles (\\b, POSIX classes: test_regex_flavours)."""
    for rx in ["(a)\\1", "(?=a)", "(?!x)", "(a)(b)\\2c"]:
        pol = [{"name": "p", "ingress_per_port_policies": [{"port": 80, "rules": [
            {"http_rules": {"http_rules": [{"headers": [{"name": ":path", "regex_match": rx}]}]}}]}]}]
        with pytest.raises(N.CiliumGPUError) as ei:
            host.update_http_policy(pol)
        assert ei.value.code == N.CG_UNSUPPORTED, rx


def test_stale_batch_rejected(host):
    host.update_http_policy(synth.starwars_policy())
    b = host.pack_http(**synth.starwars_requests(10))
    host.update_http_policy(synth.starwars_policy())  # new snapshot
    with pytest.raises(N.CiliumGPUError):
        host.http_eval_host_diag(b)


def test_c_abi_harness(tmp_path):
    """tests/native/abi_harness.c: gcc (C11, -Werror) against
    include/cilium_gpu.h, linked to libciliumgpu.so — static_asserts on the
    BPF-map and record layouts, then the control-plane calls and the host
    table walks on a device = -1 handle (verdict calls: CG_NO_DEVICE)."""
    import shutil
    import subprocess
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    lib = os.path.join(ROOT, "cilium_amd")
    exe = str(tmp_path / "abi_harness")
    subprocess.run([gcc, "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "abi_harness.c"), "-o", exe, "-L", lib, "-lciliumgpu",
                    "-Wl,-rpath," + lib], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_go_binding_names_exist_in_header():
    """go/gpuclassifier (the cgo package; no Go toolchain in this image):
    every C identifier it references is declared by include/cilium_gpu.h (or
    is a cgo builtin), and each struct field it names is a field of that
    struct in the header."""
    import glob
    hdr = open(os.path.join(ROOT, "include", "cilium_gpu.h")).read()
    builtin = {"CString", "GoString", "free", "CBytes", "size_t", "int", "char", "uint8_t", "uint16_t",
               "uint32_t", "uint64_t", "int16_t", "int32_t", "int64_t"}
    names = set()
    for f in glob.glob(os.path.join(ROOT, "go", "gpuclassifier", "*.go")):
        src = open(f).read()
        names |= set(re.findall(r"\bC\.([A-Za-z_][A-Za-z0-9_]*)", src))
        for struct, body in re.findall(r"C\.(cg_[a-z_0-9]+)\{([^}]*)\}", src):
            m = re.search(r"typedef struct \{([^}]*)\}\s*" + struct + ";", hdr)
            assert m, struct
            for field in re.findall(r"(\w+):", body):
                assert re.search(r"\b" + field + r"\b", m.group(1)), (struct, field)
    missing = [n for n in sorted(names) if n not in builtin and not re.search(r"\b" + n + r"\b", hdr)]
    assert not missing, missing
    assert len(names) > 40
