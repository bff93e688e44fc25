"""CPU oracle — TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg, as the checker or the timed CPU baseline; never by the
product (``cilium_amd``).  ``liboracle.so`` (oracle.cc) restates the
reference algorithms in C++ with libstdc++ std::regex (Envoy's engine);
``ref_py`` restates them in pure Python for small cases and fixture
generation.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"


def build() -> Path:
    import subprocess
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def _load():
    if not LIB_PATH.exists():
        build()
    lib = C.CDLL(str(LIB_PATH))
    p, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
    lib.or_last_error.restype = C.c_char_p
    lib.or_l4.argtypes = [p, p, sz, p, sz, p, p, p]
    lib.or_l4_mode.argtypes = [p, p, sz, p, sz, p, p, p, u32]
    lib.or_prefilter.argtypes = [u32, p, sz, p, sz, p, sz, p, sz, p, p, sz, p, C.c_int]
    lib.or_ipcache.argtypes = [p, p, sz, p, sz, p, p, sz, p, C.c_int]
    lib.or_http_load.restype = p
    lib.or_http_load.argtypes = [C.c_char_p, sz]
    lib.or_http_free.argtypes = [p]
    lib.or_http_eval.argtypes = [p, sz, p, p, p, p, p, p, p, C.c_int]
    lib.or_http_eval_attr.argtypes = [p, sz, p, p, p, p, p, p, p, p, C.c_int]
    lib.or_regex_match.argtypes = [C.c_char_p, sz, p, sz, C.c_int]
    lib.or_kafka_load.restype = p
    lib.or_kafka_load.argtypes = [C.c_char_p, sz]
    lib.or_kafka_free.argtypes = [p]
    lib.or_kafka_eval.argtypes = [p, sz, p, p, p, p, p, p, p, p, p, C.c_int]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


# ------------------------------------------------------------------ L4 ----
L4_CAN_ACCESS, L4_INGRESS, L4_EGRESS, L4_IGNORE_DROP = 0, 1, 2, 0x100


def l4(keys: np.ndarray, ports_be: np.ndarray, tuples: np.ndarray, mode: int = L4_CAN_ACCESS):
    """__policy_can_access over tuples (or a wrapper of it, see or_l4_mode);
    returns (verdicts, packets, bytes per key)."""
    keys = np.ascontiguousarray(keys)
    ports_be = np.ascontiguousarray(ports_be, np.uint16)
    tuples = np.ascontiguousarray(tuples)
    out = np.zeros(max(len(tuples), 1), np.int32)
    pk = np.zeros(max(len(keys), 1), np.uint64)
    by = np.zeros(max(len(keys), 1), np.uint64)
    lib().or_l4_mode(_ptr(keys), _ptr(ports_be), len(keys), _ptr(tuples), len(tuples), _ptr(out), _ptr(pk),
                     _ptr(by), mode)
    return out[:len(tuples)], pk[:len(keys)], by[:len(keys)]


def l4_egress_via_ipcache(keys, ports_be, ik, iv, remote, tuples):
    """The egress flow of bpf_lxc.c:509-527 (v4 remote: u32 network order)
    / :205-220 (v6 remote: (n, 16) u8): the remote identity from the ipcache
    oracle, then policy_can_egress.  Returns (verdicts, packets, bytes)."""
    t = np.array(tuples, copy=True)
    if remote.dtype == np.uint8:
        _, o6 = ipcache(ik, iv, np.zeros(0, np.uint32), remote.reshape(-1, 16))
        t["identity"] = o6[:, 0]
    else:
        o4, _ = ipcache(ik, iv, remote, np.zeros((0, 16), np.uint8))
        t["identity"] = o4[:, 0]
    return l4(keys, ports_be, t, L4_EGRESS)


# ----------------------------------------------------------------- LPM ----
def prefilter(config: int, cidrs: np.ndarray, ep4: np.ndarray, ep6: np.ndarray, v4: np.ndarray, v6: np.ndarray,
              nthreads: int = 1):
    cidrs = np.ascontiguousarray(cidrs)
    ep4 = np.ascontiguousarray(ep4, np.uint32)
    ep6 = np.ascontiguousarray(ep6, np.uint8).reshape(-1)
    v4 = np.ascontiguousarray(v4, np.uint32).reshape(-1)
    v6 = np.ascontiguousarray(v6, np.uint8).reshape(-1)
    n4, n6 = len(v4) // 2, len(v6) // 32
    o4 = np.zeros(max(n4, 1), np.uint8)
    o6 = np.zeros(max(n6, 1), np.uint8)
    lib().or_prefilter(config, _ptr(cidrs), len(cidrs), _ptr(ep4), len(ep4), _ptr(ep6), len(ep6) // 16,
                       _ptr(v4), n4, _ptr(o4), _ptr(v6), n6, _ptr(o6), nthreads)
    return o4[:n4], o6[:n6]


# ------------------------------------------------------------- ipcache ----
def ipcache(keys: np.ndarray, vals: np.ndarray, v4: np.ndarray, v6: np.ndarray, nthreads: int = 1):
    """lookup_ip{4,6}_remote_endpoint + the bpf_lxc.c:509-518 resolution.

    keys: CIDR_DTYPE records; vals: (n, 2) u32 {sec_label, tunnel_endpoint};
    v4: u32 network-order addresses; v6: (n6, 16) u8.  Returns (n4, 2) and
    (n6, 2) u32 {identity, tunnel_endpoint}."""
    keys = np.ascontiguousarray(keys)
    vals = np.ascontiguousarray(vals, np.uint32).reshape(-1, 2)
    v4 = np.ascontiguousarray(v4, np.uint32).reshape(-1)
    v6 = np.ascontiguousarray(v6, np.uint8).reshape(-1)
    n4, n6 = len(v4), len(v6) // 16
    o4 = np.zeros((max(n4, 1), 2), np.uint32)
    o6 = np.zeros((max(n6, 1), 2), np.uint32)
    lib().or_ipcache(_ptr(keys), _ptr(vals), len(keys), _ptr(v4), n4, _ptr(o4), _ptr(v6), n6, _ptr(o6), nthreads)
    return o4[:n4], o6[:n6]


# ---------------------------------------------------------------- HTTP ----
def _blob(b: bytes) -> bytes:
    return str(len(b)).encode() + b" " + b


def http_policy_text(policies: list[dict]) -> bytes:
    """NPDS dicts → the oracle's length-prefixed text format."""
    from cilium_amd.policy import matcher_kind  # pure-Python helper, no native code
    out = []
    for p in policies:
        out.append(b"policy " + _blob(p["name"].encode()))
        for d, key in ((1, "ingress_per_port_policies"), (0, "egress_per_port_policies")):
            out.append(b"dir %d" % d)
            for pp in p.get(key) or []:
                proto = pp.get("protocol", "TCP")
                tcp = 1 if proto in ("TCP", 0) else 0
                out.append(b"port %d %d" % (int(pp.get("port", 0)), tcp))
                for r in pp.get("rules") or []:
                    remotes = [int(x) for x in r.get("remote_policies") or []]
                    hr = r.get("http_rules")
                    has_http = 1 if hr is not None else 0
                    out.append(b"rule %d %d" % (has_http, len(remotes)) +
                               b"".join(b" %d" % x for x in remotes))
                    for rule in (hr or {}).get("http_rules") or []:
                        hs = rule.get("headers") or []
                        out.append(b"http %d" % len(hs))
                        for m in hs:
                            kind, val = matcher_kind(m)
                            out.append(b"hdr " + kind.encode() + b" " + _blob(m["name"].encode()) + b" " +
                                       _blob(val.encode()))
    return b"\n".join(out) + b"\n"


class HttpOracle:
    def __init__(self, policies: list[dict]):
        txt = http_policy_text(policies)
        self.h = lib().or_http_load(txt, len(txt))
        if not self.h:
            raise ValueError("oracle rejected policy: " + lib().or_last_error().decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_http_free(self.h)

    def eval(self, policy, ingress, port, remote, hdr_blob, hdr_off, nthreads: int = 1) -> np.ndarray:
        n = len(policy)
        policy = np.ascontiguousarray(policy, np.uint32)
        ingress = np.ascontiguousarray(ingress, np.uint8)
        port = np.ascontiguousarray(port, np.uint16)
        remote = np.ascontiguousarray(remote, np.uint32)
        hdr_blob = np.ascontiguousarray(hdr_blob, np.uint8)
        if len(hdr_blob) == 0:
            hdr_blob = np.zeros(1, np.uint8)
        hdr_off = np.ascontiguousarray(hdr_off, np.uint64)
        out = np.zeros(max(n, 1), np.uint8)
        lib().or_http_eval(self.h, n, _ptr(policy), _ptr(ingress), _ptr(port), _ptr(remote), _ptr(hdr_blob),
                           _ptr(hdr_off), _ptr(out), nthreads)
        return out[:n]

    def eval_attr(self, policy, ingress, port, remote, hdr_blob, hdr_off, nthreads: int = 1):
        """Verdicts plus, per request, the rule that allowed it in Envoy's
        evaluation order: (n, 4) u32 {program port, scope, rule, http_rule},
        program port 0xFFFFFFFF when no rule allowed it (oracle.cc Attr)."""
        n = len(policy)
        policy = np.ascontiguousarray(policy, np.uint32)
        ingress = np.ascontiguousarray(ingress, np.uint8)
        port = np.ascontiguousarray(port, np.uint16)
        remote = np.ascontiguousarray(remote, np.uint32)
        hdr_blob = np.ascontiguousarray(hdr_blob, np.uint8)
        if len(hdr_blob) == 0:
            hdr_blob = np.zeros(1, np.uint8)
        hdr_off = np.ascontiguousarray(hdr_off, np.uint64)
        out = np.zeros(max(n, 1), np.uint8)
        attr = np.zeros((max(n, 1), 4), np.uint32)
        lib().or_http_eval_attr(self.h, n, _ptr(policy), _ptr(ingress), _ptr(port), _ptr(remote), _ptr(hdr_blob),
                                _ptr(hdr_off), _ptr(out), _ptr(attr), nthreads)
        return out[:n], attr[:n]


def regex_match(re: bytes, s: bytes, search: bool = False) -> int:
    """std::regex_match / regex_search (ECMAScript): 1, 0, or -1 for an invalid regex."""
    buf = np.frombuffer(s, np.uint8) if s else np.zeros(1, np.uint8)
    return lib().or_regex_match(re, len(re), _ptr(buf), len(s), 1 if search else 0)


# --------------------------------------------------------------- Kafka ----
def kafka_policy_text(redirects: list[dict]) -> bytes:
    out = []
    for rd in redirects:
        out.append(b"redirect " + _blob(rd["name"].encode()))
        for s in rd.get("selectors", []):
            ids = s.get("identities")
            wild = ids is None
            ids = ids or []
            out.append(b"sel %d %d" % (1 if wild else 0, len(ids)) + b"".join(b" %d" % int(x) for x in ids))
            for r in s.get("rules", []):
                if hasattr(r, "to_json"):
                    r = r.to_json()
                out.append(b"krule " + b" ".join(_blob(r.get(k, "").encode())
                                                for k in ("role", "apiKey", "apiVersion", "clientID", "topic")))
    return b"\n".join(out) + b"\n"


class KafkaOracle:
    def __init__(self, redirects: list[dict]):
        txt = kafka_policy_text(redirects)
        self.h = lib().or_kafka_load(txt, len(txt))
        if not self.h:
            raise ValueError("oracle rejected Kafka policy: " + lib().or_last_error().decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_kafka_free(self.h)

    def eval(self, redirect, remote, api_key, api_version, kind, client_id, topics, nthreads: int = 1):
        n = len(redirect)
        parts, off = [], [0]
        for i in range(n):
            b = client_id[i] + b"\0" + b"".join(t + b"\0" for t in topics[i])
            parts.append(b)
            off.append(off[-1] + len(b))
        blob = np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy()
        args = [np.ascontiguousarray(redirect, np.uint32), np.ascontiguousarray(remote, np.uint32),
                np.ascontiguousarray(api_key, np.int16), np.ascontiguousarray(api_version, np.int16),
                np.ascontiguousarray(kind, np.uint8)]
        off = np.asarray(off, np.uint64)
        nt = np.asarray([len(t) for t in topics], np.uint32)
        out = np.zeros(max(n, 1), np.uint8)
        lib().or_kafka_eval(self.h, n, *[_ptr(a) for a in args], _ptr(blob), _ptr(off), _ptr(nt), _ptr(out),
                            nthreads)
        return out[:n]
