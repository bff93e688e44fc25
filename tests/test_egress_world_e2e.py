"""test/runtime/Policies.go:1087-1190 ("Tests Egress To World") end to end
(tests/golden/egress_world_kat.json) under PolicyEnforcement=always
(ComputePolicyEnforcement, pkg/endpoint/policy.go:616-639): the destination
through the ipcache, app1's egress map (policy_can_egress), and for a pod
destination that pod's ingress map (policy_can_access_ingress).  CPU: the
oracle and the compiled tables' host walks; GPU: the fused ipcache →
l4_fp_kernel path and the ingress kernel.
"""
import ipaddress

import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import resolve as R
from cilium_amd.classifier import IPCache, L4_TUPLE_DTYPE
from cilium_amd.policy import htons
from kat_util import load
from test_policy_merge import _keys_ports

KAT = load("egress_world_kat.json")
PODS = KAT["pods"]
IDS = {n: 300 + i for i, n in enumerate(PODS)}
CACHE = {IDS[n]: {f"container:id.{n}": ""} for n in PODS}
CACHE.update({R.RESERVED_HOST: {"reserved:host": ""}, R.RESERVED_WORLD: {"reserved:world": ""}})


def _ipcache():
    return (IPCache._keys([f"{KAT['addrs'][n]}/32" for n in PODS]),
            np.array([[IDS[n], 0] for n in PODS], np.uint32))


def _probes(suite):
    """(remote address, egress tuple, ingress tuple or None, expect)"""
    repo = R.Repository([R.Rule.from_json(r) for r in suite["policy"]],
                        R.PolicyConfig(always_allow_localhost=False, enforcement=KAT["enforcement"]))
    maps = {n: _keys_ports(R.endpoint_policy_map_state(repo, CACHE[IDS[n]], CACHE)) for n in PODS}
    out = []
    for dst, proto, dport, want in suite["asserts"]:
        a = np.array([int.from_bytes(ipaddress.ip_address(KAT["addrs"][dst]).packed, "little")], np.uint32)
        eg = np.zeros(1, L4_TUPLE_DTYPE)
        eg[0] = (0, htons(dport), proto, 0, 100)
        ing = None
        if dst in IDS:
            ing = np.zeros(1, L4_TUPLE_DTYPE)
            ing[0] = (IDS["app1"], htons(dport), proto, N.CG_L4_F_INGRESS, 100)
        out.append((dst, a, eg, ing, bool(want)))
    return maps, out


def _check(suite, egress_fn, ingress_fn):
    maps, probes = _probes(suite)
    bad = []
    for dst, a, eg, ing, want in probes:
        ok = int(egress_fn(maps["app1"], a, eg)) >= 0
        if ok and ing is not None:
            ok = int(ingress_fn(maps[dst], ing)) >= 0
        if ok != want:
            bad.append(dst)
    assert not bad, bad


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_egress_world_oracle(suite):
    ik, iv = _ipcache()
    _check(suite, lambda kp, a, t: oracle.l4_egress_via_ipcache(*kp, ik, iv, a, t)[0][0],
           lambda kp, t: oracle.l4(*kp, t, oracle.L4_INGRESS)[0][0])


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_egress_world_host_tables(host, suite):
    ic = host.ipcache()
    ic.update(*_ipcache())

    def walk(kp, t):
        pm = host.policy_map()
        pm.allow_keys(*kp)
        v = pm.eval_host_diag(t)[0]
        pm.destroy()
        return v

    def egress(kp, a, t):
        t = t.copy()
        t["identity"] = ic.eval_host_diag(a, np.zeros((0, 16), np.uint8))[0][:, 0]
        return walk(kp, t)
    _check(suite, egress, walk)


@pytest.mark.gpu
@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_gpu_egress_world(gpu, suite):
    ic = gpu.ipcache()
    ic.update(*_ipcache())

    def egress(kp, a, t):
        pm = gpu.policy_map()
        pm.allow_keys(*kp)
        v = pm.verdicts_via_ipcache(ic, a, t)[0]
        pm.destroy()
        return v

    def ingress(kp, t):
        pm = gpu.policy_map()
        pm.allow_keys(*kp)
        v = pm.verdicts(t, mode=N.CG_L4_INGRESS)[0]
        pm.destroy()
        return v
    _check(suite, egress, ingress)
    ic.destroy()


def test_policy_enforcement_modes():
    """Policies.go:99-240: whether the id.app endpoint has policy enforcement
    on (any direction) per daemon mode, without and with sample_policy.json."""
    m = KAT["enforcement_modes"]
    lbl = {"container:id.app": ""}
    for mode, (without, with_policy) in m["enabled"].items():
        for rules, want in (([], without), (m["policy"], with_policy)):
            repo = R.Repository([R.Rule.from_json(r) for r in rules], R.PolicyConfig(enforcement=mode))
            assert any(R.compute_policy_enforcement(repo, lbl)) == want, (mode, bool(rules))
    # an endpoint still labelled reserved:init is enforced in default mode
    assert R.compute_policy_enforcement(R.Repository(), {"reserved:init": ""}) == (True, True)
