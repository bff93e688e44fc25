"""test/runtime/Policies.go:495-560 ("L7 Checks"), :637-697 ("L3-Dependent
L7 Egress", with its proxy statistics) and test/k8sT/Policies.go:249-343 (the
CNP L3/L4 and L7 policies on demo.yaml's pods) end to end
(tests/golden/policies_l7_kat.json): the policy files → Repository → per
endpoint policy map state (L4 redirects to proxy ports) and NPDS → every
curl / ping assertion as the datapath and the proxy decide it:

- client side (not for the host, which has no endpoint): policy_can_egress
  at the client's map, remote = server; a redirect sends the request through
  the client's egress NPDS (port 80, remote = server);
- server side: policy_can_access_ingress at the server's map, remote =
  client; a redirect sends it through the server's ingress NPDS.

A probe succeeds when every step allows it.  The CPU test runs the chain
through the oracle and the compiled tables' host walks; the GPU test through
l4_fp_kernel and http_kernel.
"""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import resolve as R
from cilium_amd.classifier import L4_TUPLE_DTYPE
from cilium_amd.policy import htons
from kat_util import load
from test_policy_merge import _keys_ports

KAT = load("policies_l7_kat.json")
# one proxy port per (ingress, protocol, port) redirect (proxy.go allocates them)
PROXY = {(True, "TCP", 80): 15001, (False, "TCP", 80): 15002, (True, "TCP", 8080): 15003,
         (False, "TCP", 8080): 15004}
PATHS = {"public": b"/public", "private": b"/private"}


def _names(suite):
    return suite.get("containers", KAT["containers"])


def _world(suite):
    names = _names(suite)
    ids = {n: 256 + i for i, n in enumerate(names)}
    ids["host"] = R.RESERVED_HOST
    cache = {R.RESERVED_HOST: {"reserved:host": ""}, R.RESERVED_WORLD: {"reserved:world": ""}}
    for n in names:
        cache[ids[n]] = suite["labels"][n] if "labels" in suite else {f"container:id.{n}": ""}
    return ids, cache


def _endpoints(suite):
    """Per container: (policy map keys, proxy ports) and its NPDS, in the
    suite's container order (the NPDS list index is the policy index)."""
    ids, cache = _world(suite)
    repo = R.Repository([R.Rule.from_json(r) for r in suite["policy"]],
                        R.PolicyConfig(always_allow_localhost=suite.get("allow_localhost", KAT["allow_localhost"])))
    maps, npds = {}, []
    for n in _names(suite):
        lbl = cache[ids[n]]
        ing_on, eg_on = repo.get_rules_matching(lbl)
        l4 = R.L4Policy(Ingress=repo.resolve_l4_ingress_policy(lbl) if ing_on else {},
                        Egress=repo.resolve_l4_egress_policy(lbl) if eg_on else {})
        maps[n] = _keys_ports(R.endpoint_policy_map_state(repo, lbl, cache, PROXY))
        npds.append(R.get_network_policy(f"ep-{n}", ids[n], l4, ing_on, eg_on, cache))
    return ids, maps, npds


def _probes(suite):
    out = []
    for cli, srv, kind, expect in suite["asserts"]:
        for k in (["ping", "public", "private"] if kind == "all" else [kind]):
            out.append((cli, srv, k, expect))
    return out


def _tuple(remote, kind, ingress):
    t = np.zeros(1, L4_TUPLE_DTYPE)
    proto, dport = (1, 0) if kind == "ping" else (6, 80)
    t[0] = (remote, htons(dport), proto, N.CG_L4_F_INGRESS if ingress else 0, 100)
    return t


def _request(pol, ingress, remote, kind):
    blob = b":method\0GET\0:path\0" + PATHS[kind] + b"\0:authority\0server\0"
    return dict(policy=np.array([pol], np.uint32), ingress=np.array([ingress], np.uint8),
                port=np.array([80], np.uint16), remote=np.array([remote], np.uint32),
                hdr_blob=np.frombuffer(blob, np.uint8).copy(), hdr_off=np.array([0, len(blob)], np.uint64))


def _connectivity(suite, l4_fn, http_fn):
    """l4_fn(name, tuples, mode) → i32 verdicts at endpoint `name`'s map;
    http_fn(request dict) → u8 verdicts under the suite's NPDS list."""
    ids, _, _ = _endpoints(suite)
    idx = {n: i for i, n in enumerate(_names(suite))}
    stats = suite.get("proxy_stats")
    seen = {"received": 0, "denied": 0}

    def proxy(ep, ingress, remote, kind):  # one request through `ep`'s proxy
        allowed = bool(http_fn(_request(idx[ep], ingress, remote, kind))[0])
        if stats and ep == stats["endpoint"] and ingress == (stats["direction"] == "ingress"):
            seen["received"] += stats["twins"]  # http and http6 send one request each
            seen["denied"] += 0 if allowed else stats["twins"]
        return allowed
    got = []
    for cli, srv, kind, _ in _probes(suite):
        ok = True
        if cli != "host":  # the client's egress (bpf_lxc.c:527 policy_can_egress)
            v = int(l4_fn(cli, _tuple(ids[srv], kind, False), oracle.L4_EGRESS)[0])
            ok = v >= 0 and (v == 0 or kind == "ping" or proxy(cli, 0, ids[srv], kind))
        if ok:  # the server's ingress (bpf_lxc.c:948 policy_can_access_ingress)
            v = int(l4_fn(srv, _tuple(ids[cli], kind, True), oracle.L4_INGRESS)[0])
            ok = v >= 0 and (v == 0 or kind == "ping" or proxy(srv, 1, ids[cli], kind))
        got.append(ok)
    want = [p[3] for p in _probes(suite)]
    bad = [(p[0], p[1], p[2]) for p, g, w in zip(_probes(suite), got, want) if g != w]
    if stats:  # checkProxyStatistics (Policies.go:659-696)
        fwd = seen["received"] - seen["denied"]
        if (seen["received"], seen["denied"], fwd) != (stats["received"], stats["denied"], stats["forwarded"]):
            bad.append(("proxy statistics", seen, fwd))
    return bad


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_policies_l7_oracle(suite):
    _, maps, npds = _endpoints(suite)
    orc = oracle.HttpOracle(npds)
    bad = _connectivity(suite, lambda n, t, mode: oracle.l4(*maps[n], t, mode)[0], lambda rq: orc.eval(**rq))
    assert not bad, bad


@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_policies_l7_host_tables(host, suite):
    _, maps, npds = _endpoints(suite)
    host.update_http_policy(npds)
    pms = {}
    for n, (k, p) in maps.items():
        pms[n] = host.policy_map()
        pms[n].allow_keys(k, p)
    bad = _connectivity(suite, lambda n, t, mode: pms[n].eval_host_diag(t),
                        lambda rq: host.http_eval_host_diag(host.pack_http(**rq)))
    for pm in pms.values():
        pm.destroy()
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("suite", KAT["suites"], ids=lambda s: s["name"])
def test_gpu_policies_l7(gpu, suite):
    _, maps, npds = _endpoints(suite)
    gpu.update_http_policy(npds)
    pms = {}
    for n, (k, p) in maps.items():
        pms[n] = gpu.policy_map()
        pms[n].allow_keys(k, p)
    modes = {oracle.L4_EGRESS: N.CG_L4_EGRESS, oracle.L4_INGRESS: N.CG_L4_INGRESS}
    bad = _connectivity(suite, lambda n, t, mode: pms[n].verdicts(t, mode=modes[mode]),
                        lambda rq: gpu.http_verdicts(gpu.pack_http(**rq)))
    for pm in pms.values():
        pm.destroy()
    assert not bad, bad
