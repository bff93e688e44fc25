"""ctypes binding of libciliumgpu.so (include/cilium_gpu.h).

The library is the product: every verdict runs in its HIP kernels.  If the
shared object is missing this module raises at import time — there is no
Python or CPU fallback for any verdict path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

# CILIUM_AMD_LIB: load another build of the same library (kernel experiments)
LIB_PATH = Path(os.environ.get("CILIUM_AMD_LIB") or Path(__file__).resolve().parent / "libciliumgpu.so")

# cg_result (include/cilium_gpu.h)
CG_OK = 0
CG_POLICY_DROP = 1
CG_PARSER_ERROR = 2
CG_UNKNOWN_PARSER = 3
CG_UNKNOWN_CONNECTION = 4
CG_INVALID_ADDRESS = 5
CG_INVALID_INSTANCE = 6
CG_UNKNOWN_ERROR = 7
CG_INVALID_ARGUMENT = 16
CG_NO_DEVICE = 17
CG_DEVICE_ERROR = 18
CG_POLICY_REJECTED = 19
CG_REVISION_MISMATCH = 20
CG_MAP_FULL = 21
CG_NOT_FOUND = 22
CG_NO_MAP = 23
CG_UNSUPPORTED = 24

CG_REGEX_ECMA, CG_REGEX_GO = 0, 1

CG_L4_F_INGRESS = 0x01
CG_L4_F_FRAGMENT = 0x02
CG_L4_F_CB_POLICY = 0x04
CG_L4_CAN_ACCESS, CG_L4_INGRESS, CG_L4_EGRESS, CG_L4_IGNORE_DROP = 0, 1, 2, 0x100
CG_DROP_POLICY = -133
CG_DROP_FRAG_NOSUPPORT = -157

CG_PF_DYN4, CG_PF_DYN6, CG_PF_FIX4, CG_PF_FIX6 = 1, 2, 4, 8
CG_XDP_DROP, CG_XDP_PASS = 1, 2
CG_WORLD_ID = 2

CG_CTR_HTTP_PROGRAMS, CG_CTR_KAFKA, CG_CTR_PREFILTER, CG_CTR_HTTP_RULES, CG_CTR_HTTP_ALLREDUCE = 0, 1, 2, 3, 4
CG_HTTP_RULE_NO_HTTP, CG_HTTP_RULE_SCOPE_ALLOW = 0xFFFFFFFF, 0xFFFFFFFE

CG_HTTP_TILE = 64
CG_HTTP_UNITS = 9

CG_KAFKA_MAX_TOPICS = 12
CG_KAFKA_K_NIL, CG_KAFKA_K_TYPED, CG_KAFKA_K_CONSUMER_METADATA = 0, 1, 2
CG_KAFKA_UNKNOWN_STR = 0xFFFFFFFF
CG_KAFKA_TOPICS_IN_ARENA = 255
CG_KAFKA_DECODE_OK, CG_KAFKA_DECODE_ERROR = 0, 1
CG_KAFKA_V_DENY, CG_KAFKA_V_ALLOW, CG_KAFKA_V_CLOSE = 0, 1, 2


class CiliumGPUError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code
        self.msg = msg


class KV(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p)]


class PolicyKeyC(C.Structure):
    _pack_ = 1
    _fields_ = [("sec_label", C.c_uint32), ("dport", C.c_uint16), ("protocol", C.c_uint8), ("egress", C.c_uint8)]


class PolicyEntryC(C.Structure):
    _fields_ = [("proxy_port", C.c_uint16), ("pad", C.c_uint16 * 3), ("packets", C.c_uint64),
                ("bytes", C.c_uint64)]


class CidrC(C.Structure):
    _fields_ = [("family", C.c_uint8), ("prefixlen", C.c_uint8), ("pad", C.c_uint8 * 2), ("addr", C.c_uint8 * 16)]


# Exported symbols and their signatures: (restype, argtypes)
_u64, _u32, _sz, _p, _i64 = C.c_uint64, C.c_uint32, C.c_size_t, C.c_void_p, C.c_int64
SIGNATURES = {
    "cg_open": (_u64, [C.POINTER(KV), _sz, C.c_uint8]),
    "cg_close": (None, [_u64]),
    "cg_last_error": (C.c_char_p, []),
    "cg_version": (C.c_char_p, []),
    "cg_sync": (C.c_int, [_u64]),
    "cg_policymap_create": (C.c_int, [_u64, _u32, C.POINTER(_u32)]),
    "cg_policymap_destroy": (C.c_int, [_u64, _u32]),
    "cg_policymap_allow": (C.c_int, [_u64, _u32, _p, _p, _sz]),
    "cg_policymap_delete": (C.c_int, [_u64, _u32, _p, _sz]),
    "cg_policymap_lookup": (C.c_int, [_u64, _u32, _p, _p]),
    "cg_policymap_dump": (C.c_int, [_u64, _u32, _p, _p, _sz, C.POINTER(_sz)]),
    "cg_policymap_flush": (C.c_int, [_u64, _u32]),
    "cg_l4_verdicts_dev": (C.c_int, [_u64, _u32, _p, _sz, _p, _p]),
    "cg_l4_verdicts_host": (C.c_int, [_u64, _u32, _p, _sz, _p]),
    "cg_l4_policy_verdicts_dev": (C.c_int, [_u64, _u32, _u32, _p, _sz, _p, _p]),
    "cg_l4_policy_verdicts_host": (C.c_int, [_u64, _u32, _u32, _p, _sz, _p]),
    "cg_prefilter_create": (C.c_int, [_u64, _u32, _u32, _u32, C.POINTER(_u32)]),
    "cg_prefilter_destroy": (C.c_int, [_u64, _u32]),
    "cg_prefilter_insert": (C.c_int, [_u64, _u32, _i64, _p, _sz, C.POINTER(_i64)]),
    "cg_prefilter_delete": (C.c_int, [_u64, _u32, _i64, _p, _sz, C.POINTER(_i64)]),
    "cg_prefilter_dump": (C.c_int, [_u64, _u32, _p, _sz, C.POINTER(_sz), C.POINTER(_i64)]),
    "cg_prefilter_set_endpoints": (C.c_int, [_u64, _u32, _p, _sz, _p, _sz]),
    "cg_prefilter_verdicts_dev": (C.c_int, [_u64, _u32, _p, _sz, _p, _p, _sz, _p, _p]),
    "cg_prefilter_verdicts_host": (C.c_int, [_u64, _u32, _p, _sz, _p, _p, _sz, _p]),
    "cg_ipcache_create": (C.c_int, [_u64, _u32, C.POINTER(_u32)]),
    "cg_ipcache_destroy": (C.c_int, [_u64, _u32]),
    "cg_ipcache_update": (C.c_int, [_u64, _u32, _p, _p, _sz]),
    "cg_ipcache_delete": (C.c_int, [_u64, _u32, _p, _sz]),
    "cg_ipcache_lookup": (C.c_int, [_u64, _u32, _p, _p]),
    "cg_ipcache_dump": (C.c_int, [_u64, _u32, _p, _p, _sz, C.POINTER(_sz)]),
    "cg_ipcache_resolve_dev": (C.c_int, [_u64, _u32, _p, _sz, _p, _p, _sz, _p, _p]),
    "cg_ipcache_resolve_host": (C.c_int, [_u64, _u32, _p, _sz, _p, _p, _sz, _p]),
    "cg_proxylib_stats": (C.c_int, [_u64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "cg_kafka_decode_stats": (C.c_int, [_u64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "cg_kafka_inflate_stats": (C.c_int, [_u64, C.POINTER(C.c_uint64)]),
    "cg_proxylib_set_batching": (C.c_int, [_u64, _u32, _u32]),
    "cg_proxylib_policy_update": (C.c_int, [_u64, C.c_char_p, _sz]),
    "cg_proxylib_policy_update_npds": (C.c_int, [_u64, C.c_char_p, _sz]),
    "cg_l4_verdicts_ipcache_dev": (C.c_int, [_u64, _u32, _u32, _p, _p, _sz, _p, _p]),
    "cg_l4_verdicts_ipcache_host": (C.c_int, [_u64, _u32, _u32, _p, _p, _sz, _p]),
    "cg_l4_verdicts_ipcache6_dev": (C.c_int, [_u64, _u32, _u32, _p, _p, _sz, _p, _p]),
    "cg_l4_verdicts_ipcache6_host": (C.c_int, [_u64, _u32, _u32, _p, _p, _sz, _p]),
    "cg_http_policy_update": (C.c_int, [_u64, C.c_char_p, _sz]),
    "cg_http_policy_update_npds": (C.c_int, [_u64, C.c_char_p, _sz]),
    "cg_http_pack_threads": (_u32, []),
    "cg_http_policy_export": (C.c_int, [_u64, C.c_void_p, _sz, C.POINTER(_sz)]),
    "cg_http_policy_import": (C.c_int, [_u64, C.c_char_p, _sz]),
    "cg_http_policy_index": (C.c_int, [_u64, C.c_char_p, C.POINTER(_u32)]),
    "cg_http_policy_stats": (C.c_int, [_u64, C.POINTER(_u64), _sz]),
    "cg_http_rule_info_get": (C.c_int, [_u64, _p, _sz, C.POINTER(_sz)]),
    "cg_http_batch_bytes": (_sz, [_u64, _sz]),
    "cg_http_batch_slots": (_sz, [_u64, _sz]),
    "cg_http_pack": (C.c_int, [_u64, _sz, _p, _p, _p, _p, _p, _p, _p, _sz, _p, C.POINTER(_sz), _p, _sz,
                               C.POINTER(_sz)]),
    "cg_http_parse_heads": (C.c_int, [_p, _p, _sz, _p, _sz, _p, C.POINTER(_sz), _p]),
    "cg_http_verdicts_dev": (C.c_int, [_u64, _p, _sz, _p, _p, _p]),
    "cg_http_verdicts_host": (C.c_int, [_u64, _p, _sz, _p, _sz, _p, _sz, _p]),
    "cg_http_verdicts_rules_host": (C.c_int, [_u64, _p, _sz, _p, _sz, _p, _sz, _p, _p]),
    "cg_http_verdicts_rules_dev": (C.c_int, [_u64, _p, _sz, _p, _p, _p, _p]),
    "cg_http_verdicts_raw_dev": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p, _p, _p, _p]),
    "cg_http_verdicts_raw_host": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p, _p, _p]),
    "cg_http_verdicts_fields_dev": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p, _p, _p, _p]),
    "cg_http_verdicts_fields_host": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p, _p, _p]),
    "cg_http_ring_open": (C.c_int, [_u64, C.c_uint32, C.c_uint32]),
    "cg_http_ring_verdicts": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p, _p, _p]),
    "cg_http_ring_stats": (C.c_int, [_u64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "cg_http_ring_close": (C.c_int, [_u64]),
    "cg_kafka_policy_update": (C.c_int, [_u64, C.c_char_p, _sz]),
    "cg_kafka_policy_index": (C.c_int, [_u64, C.c_char_p, C.POINTER(_u32)]),
    "cg_kafka_intern": (C.c_int, [_u64, _u32, C.c_char_p, _sz, C.POINTER(_u32)]),
    "cg_kafka_verdicts_dev": (C.c_int, [_u64, _p, _sz, _p, _p, _p]),
    "cg_kafka_verdicts_split_dev": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p]),
    "cg_kafka_verdicts_host": (C.c_int, [_u64, _p, _sz, _p, _sz, _p]),
    "cg_kafka_decode_host": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p, _p, _sz, C.POINTER(_sz), _p]),
    "cg_kafka_decode_dev": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p, _p, _sz, C.POINTER(_sz), _p, _p]),
    "cg_kafka_verdicts_raw_host": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p]),
    "cg_diag_kafka_decode_host": (C.c_int, [_u64, _p, _p, _sz, _p, _p, _p, _p, _sz, C.POINTER(_sz), _p]),
    "cg_read_counters": (C.c_int, [_u64, _u32, _u32, _p, _sz, C.POINTER(_sz)]),
    "cg_counters_device_ptr": (C.c_int, [_u64, _u32, _u32, C.POINTER(_p), C.POINTER(_sz)]),
    "cg_counters_copy_dev": (C.c_int, [_u64, _u32, _u32, _p, _sz, _p]),
    "cg_reset_counters": (C.c_int, [_u64]),
    "cg_diag_regex_match": (C.c_int, [C.c_char_p, _sz, _p, _sz, _u32, C.POINTER(C.c_uint8)]),
    "cg_regex_validate": (C.c_int, [C.c_char_p, _sz, _u32]),
    "cg_diag_http_eval_host": (C.c_int, [_u64, _p, _sz, _p, _sz, _p, _sz, _p]),
    "cg_diag_http_rules_host": (C.c_int, [_u64, _p, _sz, _p, _sz, _p, _sz, _p]),
    "cg_diag_kafka_eval_host": (C.c_int, [_u64, _p, _sz, _p, _sz, _p]),
    "cg_diag_l4_eval_host": (C.c_int, [_u64, _u32, _p, _sz, _p]),
    "cg_diag_ipcache_eval_host": (C.c_int, [_u64, _u32, _p, _sz, _p, _p, _sz, _p]),
    "cg_diag_prefilter_eval_host": (C.c_int, [_u64, _u32, _p, _sz, _p, _p, _sz, _p]),
}


def _load() -> C.CDLL:
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -m cilium_amd.build` "
                          "(there is no CPU fallback for the verdict paths)")
    lib = C.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | getattr(os, "RTLD_GLOBAL", 0))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc: int) -> None:
    if rc != CG_OK:
        raise CiliumGPUError(rc, lib.cg_last_error().decode(errors="replace"))


def regex_validate(pattern, flavour: int = CG_REGEX_GO) -> None:
    """cg_regex_validate: raises CiliumGPUError(CG_POLICY_REJECTED) with
    the parser's message when `pattern` is not valid in `flavour`."""
    b = pattern.encode("utf-8", "surrogateescape") if isinstance(pattern, str) else bytes(pattern)
    check(lib.cg_regex_validate(b, len(b), flavour))


def ptr(a) -> int | None:
    """Address of a numpy array / torch tensor / None."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data
