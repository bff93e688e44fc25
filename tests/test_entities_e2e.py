"""test/k8sT/Policies.go:162-215,674-733 ("Validate to-entities policies") end
to end (tests/golden/entities_kat.json): each CNP → Repository → the client
pod's egress map state, and every probe's destination address → ipcache →
identity → policy_can_egress, as bpf_lxc.c:509-527 chains them
(lookup_ip4_remote_endpoint, then the L4 verdict; a miss is WORLD).  CPU: the
oracle's fused restatement and the compiled tables' host walks; GPU: the fused
l4_fp_kernel<4> ipcache path.
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

KAT = load("entities_kat.json")
PODS = list(KAT["pods"])
IDS = {n: 300 + i for i, n in enumerate(PODS)}
CACHE = {IDS[n]: KAT["pods"][n] for n in PODS}
CACHE.update({R.RESERVED_HOST: {"reserved:host": ""}, R.RESERVED_WORLD: {"reserved:world": ""}})


def _a4(ip: str) -> int:
    return int.from_bytes(ipaddress.ip_address(ip).packed, "little")  # iphdr.daddr as loaded


def _ipcache():
    cidrs = [f"{KAT['addrs'][n]}/32" for n in PODS] + [f"{KAT['node']}/32"]
    vals = [[IDS[n], 0] for n in PODS] + [[R.RESERVED_HOST, 0]]
    return IPCache._keys(cidrs), np.array(vals, np.uint32)


def _case(suite):
    # Kubernetes mode: allow-localhost "auto" resolves to "always" (daemon.go:1144-1147)
    repo = R.Repository([R.Rule.from_json(r) for r in suite["policy"]], R.PolicyConfig(always_allow_localhost=True))
    for n in ("app1", "app2", "app3"):  # validatePolicyEnforcementStatus(Egress)
        assert repo.get_rules_matching(KAT["pods"][n]) == (False, True), n
    maps = {c: _keys_ports(R.endpoint_policy_map_state(repo, KAT["pods"][c], CACHE)) for c in ("app2", "app3")}
    out = []
    for c, dst, proto, dport, want in suite["asserts"]:
        t = np.zeros(1, L4_TUPLE_DTYPE)
        t[0] = (0, htons(dport), proto, 0, 100)  # identity from the ipcache; egress
        out.append((c, np.array([_a4(KAT["addrs"][dst])], np.uint32), t, bool(want), dst))
    return maps, out


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_entities_oracle(suite):
    maps, probes = _case(suite)
    ik, iv = _ipcache()
    bad = []
    for c, remote, t, want, dst in probes:
        v, _, _ = oracle.l4_egress_via_ipcache(*maps[c], ik, iv, remote, t)
        if (int(v[0]) >= 0) != want:
            bad.append((c, dst, int(v[0])))
    assert not bad, bad


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_entities_host_tables(host, suite):
    maps, probes = _case(suite)
    ic = host.ipcache()
    ic.update(*_ipcache())
    bad = []
    for c, remote, t, want, dst in probes:
        ident, _ = ic.eval_host_diag(remote, np.zeros((0, 16), np.uint8))
        t2 = t.copy()
        t2["identity"] = ident[:, 0]
        pm = host.policy_map()
        pm.allow_keys(*maps[c])
        v = int(pm.eval_host_diag(t2)[0])
        pm.destroy()
        if (v >= 0) != want:
            bad.append((c, dst, v))
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_gpu_entities(gpu, suite):
    maps, probes = _case(suite)
    ic = gpu.ipcache()
    ic.update(*_ipcache())
    bad = []
    for c, remote, t, want, dst in probes:
        pm = gpu.policy_map()
        pm.allow_keys(*maps[c])
        v = int(pm.verdicts_via_ipcache(ic, remote, t)[0])
        pm.destroy()
        if (v >= 0) != want:
            bad.append((c, dst, v))
    ic.destroy()
    assert not bad, bad
