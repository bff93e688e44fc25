"""test/runtime/Policies.go:1087-1190 ("Tests Egress To World"), :99-240
(enforcement modes) and :1395-1552 (reserved:init policies) end to end
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
    """Pods by their /32s, the node by its address (the host identity)."""
    return (IPCache._keys([f"{KAT['addrs'][n]}/32" for n in PODS] + [f"{KAT['host_ip']}/32"]),
            np.array([[IDS[n], 0] for n in PODS] + [[R.RESERVED_HOST, 0]], np.uint32))


def _probes(suite):
    """(remote address, egress tuple, ingress tuple or None, expect)"""
    repo = R.Repository([R.Rule.from_json(r) for r in suite["policy"]],
                        R.PolicyConfig(always_allow_localhost=False,
                                       enforcement=suite.get("enforcement", KAT["enforcement"])))
    maps = {n: _keys_ports(R.endpoint_policy_map_state(repo, CACHE[IDS[n]], CACHE)) for n in PODS}
    out = []
    for dst, proto, dport, want in suite["asserts"]:
        a = np.array([int.from_bytes(ipaddress.ip_address(KAT["addrs"][dst]).packed, "little")], np.uint32)
        eg = np.zeros(1, L4_TUPLE_DTYPE)
        eg[0] = (0, htons(dport), proto, 0, 100)
        ing = None
        if dst in IDS:
            ing = np.zeros(1, L4_TUPLE_DTYPE)
            ing[0] = (IDS["app1"], htons(dport), proto, N.CG_L4_F_INGRESS, 100)  # (the host has no map)
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


def _init_case(with_policy: bool):
    """Policies.go:1395-1552 under enforcement always: (endpoint, direction,
    tuple, remote address or None, expect) — ingress from the host identity,
    egress to the host address through the ipcache."""
    c = KAT["init"]
    ids = {"init": R.RESERVED_INIT, "somelabel": 400}
    cache = {ids[n]: lbl for n, lbl in c["endpoints"].items()}
    cache.update({R.RESERVED_HOST: {"reserved:host": ""}, R.RESERVED_WORLD: {"reserved:world": ""}})
    repo = R.Repository([R.Rule.from_json(r) for r in (c["policy"] if with_policy else [])],
                        R.PolicyConfig(always_allow_localhost=False, enforcement="always"))
    maps = {n: _keys_ports(R.endpoint_policy_map_state(repo, c["endpoints"][n], cache)) for n in ids}
    host_a = np.array([int.from_bytes(ipaddress.ip_address(c["host_ip"]).packed, "little")], np.uint32)
    ik = IPCache._keys([f"{c['host_ip']}/32"])
    iv = np.array([[R.RESERVED_HOST, 0]], np.uint32)
    out = []
    for ep, d, no_pol, pol in c["asserts"]:
        t = np.zeros(1, L4_TUPLE_DTYPE)
        if d == "ingress":
            t[0] = (R.RESERVED_HOST, 0, 1, N.CG_L4_F_INGRESS, 84)
        else:
            t[0] = (0, 0, 1, 0, 84)
        out.append((ep, d, t, maps[ep], pol if with_policy else no_pol))
    return out, ik, iv, host_a


@pytest.mark.parametrize("with_policy", [False, True])
def test_init_policy_oracle(with_policy):
    probes, ik, iv, host_a = _init_case(with_policy)
    for ep, d, t, kp, want in probes:
        v = (oracle.l4(*kp, t, oracle.L4_INGRESS)[0][0] if d == "ingress" else
             oracle.l4_egress_via_ipcache(*kp, ik, iv, host_a, t)[0][0])
        assert (int(v) >= 0) == want, (ep, d, int(v))


@pytest.mark.gpu
@pytest.mark.parametrize("with_policy", [False, True])
def test_gpu_init_policy(gpu, with_policy):
    probes, ik, iv, host_a = _init_case(with_policy)
    ic = gpu.ipcache()
    ic.update(ik, iv)
    for ep, d, t, kp, want in probes:
        pm = gpu.policy_map()
        pm.allow_keys(*kp)
        v = pm.verdicts(t, mode=N.CG_L4_INGRESS)[0] if d == "ingress" else pm.verdicts_via_ipcache(ic, host_a, t)[0]
        pm.destroy()
        assert (int(v) >= 0) == want, (ep, d, int(v))
    ic.destroy()
