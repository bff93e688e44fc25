"""Policy repository resolution pinned to the
reference's own assertions:

- the 12-case merge table of pkg/policy/l4Filter_test.go:40-66 (mergeL4Port,
  wildcardL3L4Rule, CreateL4IngressFilter's localhost override): every
  sub-case's resolved L4Filter, error or nil (tests/golden/l4_merge_kat.json);
- the L7 outcome the table's Notes column states, through the whole chain
  policy → Repository.ResolveL4IngressPolicy → NPDS (getNetworkPolicy) →
  http_kernel, and the L4 half → policy map keys → l4_fp_kernel;
- test/runtime/Policies.go:380-443 (Policies-l3-policy.json,
  Policies-l4-policy.json): every connectivity assertion as policy → per
  endpoint policy map state (ComputePolicyEnforcement, resolveL4Policy,
  L3 / L4 / localhost entries) → egress verdict at the client's map AND
  ingress verdict at the server's map (tests/golden/policies_e2e_kat.json).

The CPU tests walk the compiled tables on the host and check the oracle; the
`gpu` tests run the same chains through the kernels.
"""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import resolve as R
from cilium_amd.classifier import L4_TUPLE_DTYPE
from cilium_amd.policy import L7Rules, PortRuleHTTP, PortRuleKafka, htons
from kat_util import load

MERGE = load("l4_merge_kat.json")
E2E = load("policies_e2e_kat.json")
PROXY_PORT = 15001


def _rules(case):
    return [R.Rule.from_json(r) for r in case["rules"]]


def _resolve(case):
    cfg = R.PolicyConfig(always_allow_localhost=bool(case.get("allow_localhost")))
    egress = case.get("dir") == "egress"
    if case["level"] == "repo":
        repo = R.Repository(_rules(case), cfg)
        return repo.resolve_l4_egress_policy(case["from"]) if egress else repo.resolve_l4_ingress_policy(case["to"])
    res = R.L4Policy()
    found = None
    for r in _rules(case):
        r.sanitize()
        if egress:
            found = R.resolve_rule_l4_egress(r, case["from"], (), res) or found
        else:
            found = R.resolve_rule_l4_ingress(r, case["to"], (), res, cfg) or found
    if found is None:
        return None
    return found.Egress if egress else found.Ingress


def _l7(entry) -> L7Rules:
    if entry.get("empty"):
        return L7Rules()
    http = [PortRuleHTTP(Path=h.get("path", ""), Method=h.get("method", "")) for h in entry["http"]] \
        if "http" in entry else None
    kafka = [PortRuleKafka(Topic=k.get("topic", "")) for k in entry["kafka"]] if "kafka" in entry else None
    return L7Rules(HTTP=http, Kafka=kafka)


@pytest.mark.parametrize("case", MERGE["cases"], ids=lambda c: c["case"])
def test_merge_table(case):
    if case.get("error"):
        with pytest.raises(R.PolicyMergeError):
            _resolve(case)
    else:
        got = _resolve(case)
        assert got is not None
        for key, want in (case.get("expect") or {}).items():
            f = got[key]
            assert (f.Port, f.Protocol, f.U8Proto, f.Ingress) == (want["port"], want["protocol"], want["u8proto"],
                                                                 want["ingress"])
            assert f.Endpoints == [R.selector_from_json(s) for s in want["endpoints"]]
            assert f.L7Parser == want["parser"]
            exp = {R.selector_from_json(e["sel"]): _l7(e) for e in want["l7"]}
            assert dict(f.L7RulesPerEp) == exp
            assert len(f.DerivedFromRules) == want["derived"]
        assert set(got) == set(case.get("expect") or case["check"])
        for key, want in (case.get("check") or {}).items():
            f = got[key]
            assert f.Port == want["port"] and f.Ingress == want["ingress"]
            assert R.selects_all(f.Endpoints) == want["selects_all"]
            assert f.L7Parser == want["parser"] and len(f.L7RulesPerEp) == want["l7_len"]
    if case.get("foo_nil"):
        # the rule does not select an endpoint labelled "foo": nothing resolved
        other = dict(case, to={"foo": ""}, level="rule")
        other.pop("error", None)
        assert _resolve(other) is None


# ------------------------------------------------- chains to the kernels ----
L7_IDS = {"a": 100, "c": 101, "b": 102, "host": R.RESERVED_HOST}
L7_CACHE = {100: {"id": "a"}, 101: {"id": "c"}, 102: {"id": "b"}, R.RESERVED_HOST: {"reserved:host": ""}}


def _l7_chain(case):
    """Repository resolution for the endpoint id=a, the NPDS it yields, and
    its policy map state (redirects on port 80 to PROXY_PORT)."""
    cfg = R.PolicyConfig(always_allow_localhost=bool(case.get("allow_localhost")))
    repo = R.Repository(_rules(case), cfg)
    l4map = repo.resolve_l4_ingress_policy(case["to"])
    npds = R.get_network_policy("ep-a", 100, R.L4Policy(Ingress=l4map), True, False, L7_CACHE)
    state = R.endpoint_policy_map_state(repo, case["to"], L7_CACHE, {(True, "TCP", 80): PROXY_PORT})
    return npds, state


def _l7_requests(srcs):
    names, methods, blob, off = [], [], b"", [0]
    for src in srcs:
        for m in ("GET", "POST"):
            b = b":method\0" + m.encode() + b"\0:path\0/\0"
            blob += b
            off.append(len(blob))
            names.append(src)
            methods.append(m)
    n = len(names)
    rq = dict(policy=np.zeros(n, np.uint32), ingress=np.ones(n, np.uint8), port=np.full(n, 80, np.uint16),
              remote=np.array([L7_IDS[s] for s in names], np.uint32),
              hdr_blob=np.frombuffer(blob, np.uint8).copy(), hdr_off=np.array(off, np.uint64))
    return rq, names


def _expected_l7(case, names):
    allow = case["l7_outcome"]["allow"]
    out = []
    for i, s in enumerate(names):
        out.append(allow[s][i % 2])
    return np.array(out, np.uint8)


def _tuples_ingress(srcs, port=80, proto=6):
    t = np.zeros(len(srcs), L4_TUPLE_DTYPE)
    t["identity"] = [L7_IDS[s] for s in srcs]
    t["dport"] = htons(port)
    t["proto"] = proto
    t["flags"] = N.CG_L4_F_INGRESS
    t["len"] = 100
    return t


def _keys_ports(state):
    from cilium_amd.classifier import POLICY_KEY_DTYPE
    keys = np.zeros(len(state), POLICY_KEY_DTYPE)
    ports = np.zeros(len(state), np.uint16)
    for i, (k, p) in enumerate(sorted(state.items(), key=lambda kv: (kv[0].Identity, kv[0].DestPort,
                                                                       kv[0].Nexthdr, kv[0].TrafficDirection))):
        keys[i] = (k.Identity, htons(k.DestPort), k.Nexthdr, k.TrafficDirection)
        ports[i] = htons(p)
    return keys, ports


L7_CASES = [c for c in MERGE["cases"] if "l7_outcome" in c]


def _check_l7_case(cl, case):
    npds, state = _l7_chain(case)
    srcs = [s for s in ("a", "c", "b", "host") if s in case["l7_outcome"]["allow"]]
    rq, names = _l7_requests(srcs)
    want = _expected_l7(case, names)
    cl.update_http_policy([npds])
    assert np.array_equal(oracle.HttpOracle([npds]).eval(**rq), want)
    # L4: the sources with any allowed request reach the proxy port, the rest drop
    keys, ports = _keys_ports(state)
    t = _tuples_ingress(srcs)
    # __policy_can_access returns the entry's proxy_port as stored (network order)
    exp_l4 = np.array([htons(PROXY_PORT) if any(case["l7_outcome"]["allow"][s]) else -133 for s in srcs], np.int32)
    assert np.array_equal(oracle.l4(keys, ports, t)[0], exp_l4)
    return rq, want, keys, ports, t, exp_l4


@pytest.mark.parametrize("case", L7_CASES, ids=lambda c: c["case"])
def test_merge_l7_outcomes_host(host, case):
    rq, want, keys, ports, t, exp_l4 = _check_l7_case(host, case)
    assert np.array_equal(host.http_eval_host_diag(host.pack_http(**rq)), want)
    pm = host.policy_map()
    pm.allow_keys(keys, ports)
    assert np.array_equal(pm.eval_host_diag(t), exp_l4)


@pytest.mark.gpu
@pytest.mark.parametrize("case", L7_CASES, ids=lambda c: c["case"])
def test_gpu_merge_l7_outcomes(gpu, case):
    rq, want, keys, ports, t, exp_l4 = _check_l7_case(gpu, case)
    assert np.array_equal(gpu.http_verdicts(gpu.pack_http(**rq)), want)
    pm = gpu.policy_map()
    pm.allow_keys(keys, ports)
    assert np.array_equal(pm.verdicts(t), exp_l4)
    pm.destroy()


# ------------------------------------------------ Policies.go runtime e2e ----
def _e2e_world():
    names = E2E["containers"]
    ids = {n: 256 + i for i, n in enumerate(names)}
    cache = {R.RESERVED_HOST: {"reserved:host": ""}, R.RESERVED_WORLD: {"reserved:world": ""}}
    for n in names:
        cache[ids[n]] = {f"container:id.{n}": ""}
    return ids, cache


def _e2e_cases(suite):
    """(client, server, proto, dport, expect) per connectivity probe; `all`
    expands to ping + http."""
    out = []
    for cli, srv, kind, expect in suite["asserts"]:
        kinds = ["ping", "http"] if kind == "all" else [kind]
        for k in kinds:
            proto, dport = (1, 0) if k == "ping" else (6, 80)
            out.append((cli, srv, proto, dport, expect, k))
    return out


def _e2e_maps(suite):
    ids, cache = _e2e_world()
    # the runtime daemon's allow-localhost "auto" is "policy" outside
    # Kubernetes (daemon.go:1144-1147, option/config.go:298-309)
    repo = R.Repository([R.Rule.from_json(r) for r in suite["policy"]], R.PolicyConfig(always_allow_localhost=False))
    states = {n: R.endpoint_policy_map_state(repo, cache[ids[n]], cache) for n in ids}
    return ids, states


def _e2e_tuples(cases, ids):
    eg = np.zeros(len(cases), L4_TUPLE_DTYPE)  # at the client's map: remote = server
    ing = np.zeros(len(cases), L4_TUPLE_DTYPE)  # at the server's map: remote = client
    for i, (cli, srv, proto, dport, _, _) in enumerate(cases):
        eg[i] = (ids[srv], htons(dport), proto, 0, 100)
        ing[i] = (ids[cli], htons(dport), proto, N.CG_L4_F_INGRESS, 100)
    return eg, ing


def _connectivity(suite, verdict_fn):
    """verdict_fn(name, keys, ports, tuples, mode) → int32 verdicts."""
    ids, states = _e2e_maps(suite)
    cases = _e2e_cases(suite)
    eg, ing = _e2e_tuples(cases, ids)
    got = []
    for i, (cli, srv, _, _, _, _) in enumerate(cases):
        kc, pc = _keys_ports(states[cli])
        ks, ps = _keys_ports(states[srv])
        v_eg = verdict_fn(cli, kc, pc, eg[i:i + 1], oracle.L4_EGRESS)[0]
        v_in = verdict_fn(srv, ks, ps, ing[i:i + 1], oracle.L4_INGRESS)[0]
        got.append(bool(v_eg >= 0 and v_in >= 0))
    want = [c[4] for c in cases]
    bad = [(c[0], c[1], c[5], g) for c, g, w in zip(cases, got, want) if g != w]
    return bad


@pytest.mark.parametrize("suite", E2E["suites"], ids=lambda s: s["name"])
def test_policies_e2e_oracle(suite):
    """The chain through the oracle's __policy_can_access wrappers."""
    bad = _connectivity(suite, lambda n, k, p, t, mode: oracle.l4(k, p, t, mode)[0])
    assert not bad, bad


@pytest.mark.parametrize("suite", E2E["suites"], ids=lambda s: s["name"])
def test_policies_e2e_host_tables(host, suite):
    """The engine's compiled tables (host walk of __policy_can_access: the
    tuple's CG_L4_F_INGRESS flag selects the direction)."""
    def fn(name, k, p, t, mode):
        pm = host.policy_map()
        pm.allow_keys(k, p)
        v = pm.eval_host_diag(t)
        pm.destroy()
        return v
    bad = _connectivity(suite, fn)
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("suite", E2E["suites"], ids=lambda s: s["name"])
def test_gpu_policies_e2e(gpu, suite):
    """Every endpoint's map synced by syncPolicyMap onto the device, each probe
    through l4_fp_kernel as policy_can_egress at the client and
    policy_can_access_ingress at the server."""
    ids, states = _e2e_maps(suite)
    maps = {}
    for n, st in states.items():
        pm = gpu.policy_map()
        R.sync_policy_map(pm, st)
        maps[n] = pm
    cases = _e2e_cases(suite)
    eg, ing = _e2e_tuples(cases, ids)
    got = []
    for i, (cli, srv, _, _, _, _) in enumerate(cases):
        v_eg = maps[cli].verdicts(eg[i:i + 1], mode=N.CG_L4_EGRESS)[0]
        v_in = maps[srv].verdicts(ing[i:i + 1], mode=N.CG_L4_INGRESS)[0]
        got.append(bool(v_eg >= 0 and v_in >= 0))
    want = [c[4] for c in cases]
    for pm in maps.values():
        pm.destroy()
    assert got == want, [(c[0], c[1], c[5]) for c, g, w in zip(cases, got, want) if g != w]
