"""GPU parity: every verdict kernel against the CPU oracle on identical
seeded inputs (bit-exact), through the C ABI."""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import synth
from cilium_amd.classifier import CIDR_DTYPE, L4_TUPLE_DTYPE, PolicyMap
from cilium_amd.policy import PolicyKey, htons

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ L4 ----
def _l4_map(cl, keys, ports):
    pm = cl.policy_map()
    pm.allow_keys(keys, ports)
    return pm


def test_l4_config2_table_parity(gpu):
    keys, ports = synth.l4_table()
    pm = _l4_map(gpu, keys, ports)
    tuples = synth.l4_tuples(2_000_000, keys)
    got = pm.verdicts(tuples)
    exp, pk, by = oracle.l4(keys, ports, tuples)
    assert np.array_equal(got, exp)
    dump = {(k.Identity, k.DestPort, k.Nexthdr, k.TrafficDirection): e for k, e in pm.dump_to_slice()}
    gpk = np.array([dump[(int(k["sec_label"]), int(k["dport"]), int(k["protocol"]), int(k["egress"]))].Packets
                    for k in keys], np.uint64)
    gby = np.array([dump[(int(k["sec_label"]), int(k["dport"]), int(k["protocol"]), int(k["egress"]))].Bytes
                    for k in keys], np.uint64)
    assert np.array_equal(gpk, pk)
    assert np.array_equal(gby, by)
    # verdict classes all exercised
    assert (exp > 0).any() and (exp == 0).any() and (exp == -133).any() and (exp == -157).any()


def test_l4_branch_table(gpu):
    """Each branch of __policy_can_access (policy.h:61-109)."""
    pm = gpu.policy_map()
    pm.allow(100, 80, 6, 0, 10001)        # L4 ingress, proxied
    pm.allow(100, 0, 0, 0, 7777)          # L3 ingress: proxy port ignored
    pm.allow(0, 53, 17, 1, 0)             # any identity, egress UDP/53
    pm.allow(200, 443, 6, 1, 0)           # L4 egress, not proxied
    t = np.zeros(9, L4_TUPLE_DTYPE)
    rows = [
        (100, htons(80), 6, 1, 100),      # L4 hit → proxy_port as stored (be16)
        (100, htons(81), 6, 1, 100),      # L3 fallback → 0
        (100, htons(80), 6, 1 | 2, 100),  # fragment skips L4 → L3 hit → 0
        (101, htons(53), 17, 0, 60),      # egress any-identity → 0
        (101, htons(53), 17, 1, 60),      # ingress: no entry → DROP_POLICY
        (101, htons(53), 17, 2, 60),      # egress fragment → DROP_FRAG_NOSUPPORT
        (101, htons(54), 17, 4, 60),      # cb_policy → allow
        (200, htons(443), 6, 0, 1500),    # egress L4 hit
        (200, htons(443), 6, 1, 1500),    # ingress miss → drop
    ]
    for i, r in enumerate(rows):
        t[i] = r
    got = pm.verdicts(t)
    assert got.tolist() == [htons(10001), 0, 0, 0, -133, -157, 0, 0, -133]
    keys = np.zeros(4, dtype=[("sec_label", "<u4"), ("dport", "<u2"), ("protocol", "u1"), ("egress", "u1")])
    e = pm.lookup(PolicyKey(100, 0, 0, 0))
    assert e.Packets == 2 and e.Bytes == 200
    assert pm.lookup(PolicyKey(100, htons(80), 6, 0)).Packets == 1
    assert pm.lookup(PolicyKey(0, htons(53), 17, 1)).Packets == 1
    # update path: delete the L3 entry → the fallback now drops
    pm.delete(100, 0, 0, 0)
    got = pm.verdicts(t[1:2])
    assert got.tolist() == [-133]
    pm.flush()
    assert pm.dump_to_slice() == []
    assert pm.verdicts(t).tolist() == [-133, -133, -157, -133, -133, -157, 0, -133, -133]
    del keys


# Expected results of the wrappers for the branch-table rows above
# (bpf/lib/policy.h:126-163): ingress forces CT_INGRESS and keeps the
# fragment flag; egress forces CT_EGRESS and is_fragment = false; both
# collapse negatives to DROP_POLICY (or TC_ACT_OK under IGNORE_DROP).
WRAPPER_ROWS = [
    (100, 80, 6, 1, 100), (100, 81, 6, 1, 100), (100, 80, 6, 1 | 2, 100), (101, 53, 17, 0, 60),
    (101, 53, 17, 1, 60), (101, 53, 17, 2, 60), (101, 54, 17, 4, 60), (200, 443, 6, 0, 1500),
    (200, 443, 6, 1, 1500), (100, 80, 6, 0, 100), (200, 443, 6, 2, 1500), (7, 9, 6, 2, 40),
]
WRAPPER_EXPECT = {
    N.CG_L4_INGRESS: [10001, 0, 0, -133, -133, -133, 0, -133, -133, 10001, -133, -133],
    N.CG_L4_EGRESS: [-133, -133, -133, 0, 0, 0, 0, 0, 0, -133, 0, -133],
    N.CG_L4_INGRESS | N.CG_L4_IGNORE_DROP: [10001, 0, 0, 0, 0, 0, 0, 0, 0, 10001, 0, 0],
    N.CG_L4_EGRESS | N.CG_L4_IGNORE_DROP: [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0],
}


def wrapper_case():
    keys = np.zeros(4, dtype=[("sec_label", "<u4"), ("dport", "<u2"), ("protocol", "u1"), ("egress", "u1")])
    keys[:] = [(100, htons(80), 6, 0), (100, 0, 0, 0), (0, htons(53), 17, 1), (200, htons(443), 6, 1)]
    ports = np.array([htons(10001), htons(7777), 0, 0], np.uint16)
    t = np.zeros(len(WRAPPER_ROWS), L4_TUPLE_DTYPE)
    for i, (ident, port, proto, flags, ln) in enumerate(WRAPPER_ROWS):
        t[i] = (ident, htons(port), proto, flags, ln)
    return keys, ports, t


@pytest.mark.parametrize("mode", sorted(WRAPPER_EXPECT))
def test_l4_wrappers_branch_table(gpu, mode):
    keys, ports, t = wrapper_case()
    pm = _l4_map(gpu, keys, ports)
    got = pm.verdicts(t, mode)
    exp = [htons(v) if v > 0 else v for v in WRAPPER_EXPECT[mode]]
    assert got.tolist() == exp
    o, pk, by = oracle.l4(keys, ports, t, mode)
    assert o.tolist() == exp
    dump = {(k.Identity, k.DestPort, k.Nexthdr, k.TrafficDirection): e for k, e in pm.dump_to_slice()}
    for i, k in enumerate(keys):
        e = dump[(int(k["sec_label"]), int(k["dport"]), int(k["protocol"]), int(k["egress"]))]
        assert (e.Packets, e.Bytes) == (int(pk[i]), int(by[i]))
    pm.destroy()


@pytest.mark.parametrize("mode", [N.CG_L4_INGRESS, N.CG_L4_EGRESS, N.CG_L4_INGRESS | N.CG_L4_IGNORE_DROP])
def test_l4_wrappers_config2(gpu, mode):
    """policy_can_access_ingress / policy_can_egress over the config-2 map
    and 2M tuples with mixed direction/fragment flags: verdicts and counters."""
    keys, ports = synth.l4_table()
    pm = _l4_map(gpu, keys, ports)
    tuples = synth.l4_tuples(2_000_000, keys, seed=mode)
    got = pm.verdicts(tuples, mode)
    exp, pk, by = oracle.l4(keys, ports, tuples, mode)
    assert np.array_equal(got, exp)
    assert not (exp == -157).any()
    dump = {(k.Identity, k.DestPort, k.Nexthdr, k.TrafficDirection): e for k, e in pm.dump_to_slice()}
    gpk = np.array([dump[(int(k["sec_label"]), int(k["dport"]), int(k["protocol"]), int(k["egress"]))].Packets
                    for k in keys], np.uint64)
    assert np.array_equal(gpk, pk)
    pm.destroy()


def test_l4_empty_and_ragged(gpu):
    keys, ports = synth.l4_table(n_entries=1000, n_ids=500)
    pm = _l4_map(gpu, keys, ports)
    assert len(pm.verdicts(np.zeros(0, L4_TUPLE_DTYPE))) == 0
    for n in (1, 63, 1025, 65537):
        tuples = synth.l4_tuples(n, keys, n_ids=500, seed=n)
        got = pm.verdicts(tuples)
        exp, _, _ = oracle.l4(keys, ports, tuples)
        assert np.array_equal(got, exp), n


def test_l4_large_map_and_long_lengths(gpu):
    """A 65,536-entry map (fingerprints and counters no longer fit LDS: the
    global-memory kernel) and packet lengths >= 64 KiB (the LDS counter's
    byte field is bypassed), verdicts and counters against the oracle."""
    keys, ports = synth.l4_table(n_entries=20000, n_ids=20000)
    for max_entries in (65536, 20000):
        pm = gpu.policy_map(max_entries=max_entries)
        pm.allow_keys(keys, ports)
        tuples = synth.l4_tuples(300_000, keys, n_ids=20000, seed=max_entries)
        tuples["len"][::7] = 70000 + np.arange(len(tuples[::7])) % 1000
        got = pm.verdicts(tuples)
        exp, pk, by = oracle.l4(keys, ports, tuples)
        assert np.array_equal(got, exp)
        dump = {(k.Identity, k.DestPort, k.Nexthdr, k.TrafficDirection): e for k, e in pm.dump_to_slice()}
        for i in range(0, len(keys), 97):
            k = keys[i]
            e = dump[(int(k["sec_label"]), int(k["dport"]), int(k["protocol"]), int(k["egress"]))]
            assert (e.Packets, e.Bytes) == (int(pk[i]), int(by[i]))


def test_l4_map_full(gpu):
    pm = gpu.policy_map(max_entries=4)
    for i in range(4):
        pm.allow(i + 1, 80, 6, 0, 0)
    with pytest.raises(N.CiliumGPUError) as ei:
        pm.allow(9, 80, 6, 0, 0)
    assert ei.value.code == N.CG_MAP_FULL
    pm.allow(1, 80, 6, 0, 5)  # update of an existing key is fine


# ----------------------------------------------------------------- LPM ----
@pytest.mark.parametrize("dyn", [True, False])
def test_prefilter_parity(gpu, dyn):
    pfx = synth.lpm_prefixes(70_000, 30_000, seed=7)
    if not dyn:
        pfx = pfx[((pfx["family"] == 4) & (pfx["prefixlen"] == 32)) | ((pfx["family"] == 6) & (pfx["prefixlen"] == 128))]
    pf = gpu.prefilter(dyn4=dyn, dyn6=dyn, max_lpm=1 << 20)
    pf.insert(0, pfx)
    v4, v6, ep4, ep6 = synth.lpm_addresses(1_000_000, pfx if len(pfx) else synth.lpm_prefixes(10, 10), seed=3)
    pf.set_endpoints(ep4, ep6)
    g4, g6 = pf.verdicts(v4, v6)
    o4, o6 = oracle.prefilter(pf.config, pfx, ep4, ep6, v4, v6, nthreads=8)
    assert np.array_equal(g4, o4)
    assert np.array_equal(g6, o6)
    assert (o4 == 1).any() and (o4 == 2).any() and (o6 == 1).any() and (o6 == 2).any()


@pytest.mark.parametrize("seed", range(2))
def test_prefilter_dense_partials(gpu, seed):
    """Rank over many partial /24 blocks, crowded IPv6 buckets (binary
    search), all-zero endpoint addresses (cases of the CPU differential)."""
    from test_cpu_differential import dense_prefilter_case
    pfx, v4, v6, ep4, ep6 = dense_prefilter_case(seed, n=400_000)
    pf = gpu.prefilter(dyn4=True, dyn6=True, max_lpm=1 << 20)
    pf.insert(0, pfx)
    pf.set_endpoints(ep4, ep6)
    g4, g6 = pf.verdicts(v4, v6)
    o4, o6 = oracle.prefilter(pf.config, pfx, ep4, ep6, v4, v6, nthreads=8)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6)


@pytest.mark.parametrize("seed", range(2))
def test_prefilter_v6_bucket_codes(gpu, seed):
    """Whole-bucket, edge-aligned and first/last-bucket IPv6 prefixes with
    addresses on and beside every interval edge (bucket codes 0/1/2)."""
    from test_cpu_differential import v6_bucket_case
    pfx, v4, v6, ep4, ep6 = v6_bucket_case(seed)
    pf = gpu.prefilter(dyn4=True, dyn6=True, max_lpm=1 << 20)
    pf.insert(0, pfx)
    pf.set_endpoints(ep4, ep6)
    g4, g6 = pf.verdicts(v4, v6)
    o4, o6 = oracle.prefilter(pf.config, pfx, ep4, ep6, v4, v6)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6)


def test_prefilter_edges(gpu):
    pf = gpu.prefilter(dyn4=True, dyn6=True)
    pf.insert(0, ["0.0.0.0/1", "10.0.0.0/8", "192.168.1.128/25", "::/1", "2001:db8::/32", "fe80::1/128"])
    v4 = np.array([[0x01000000, 0], [0x0100000A, 0], [0x80A8C0 | (200 << 24), 0], [0x7FA8C0 | (200 << 24), 0]],
                  np.uint32)  # 0.0.0.1, 10.0.0.1, 192.168.1.200 (covered), 192.168.127.200
    v6 = np.zeros((3, 32), np.uint8)
    v6[0, 0] = 0x20; v6[0, 1] = 0x01; v6[0, 2] = 0x0d; v6[0, 3] = 0xb8
    v6[1, 0] = 0xfe; v6[1, 1] = 0x80; v6[1, 15] = 1
    v6[2, 0] = 0xfe; v6[2, 1] = 0x80; v6[2, 15] = 2
    g4, g6 = pf.verdicts(v4, v6)
    o4, o6 = oracle.prefilter(pf.config, pf.cidrs(pf.dump()[0]), np.zeros(0, np.uint32), np.zeros((0, 16)), v4, v6)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6)
    assert g6.tolist() == [1, 1, 1]  # ::/1 covers everything below 8000::
    e4, e6 = pf.verdicts(np.zeros((0, 2), np.uint32), np.zeros((0, 32), np.uint8))
    assert len(e4) == 0 and len(e6) == 0


# ---------------------------------------------------------------- HTTP ----
def _http_check(cl, pols, rq):
    cl.update_http_policy(pols)
    b = cl.pack_http(**rq)
    n = len(rq["policy"])
    got = cl.http_verdicts(b)
    exp = oracle.HttpOracle(pols).eval(**rq, nthreads=8)
    assert np.array_equal(got, exp)
    return got


def test_http_starwars_parity(gpu):
    got = _http_check(gpu, synth.starwars_policy(), synth.starwars_requests(200_000))
    assert got.any() and not got.all()


def test_http_10k_parity(gpu):
    pols, info = synth.http10k_rules()
    got = _http_check(gpu, pols, synth.http10k_requests(300_000, info, distinct=100_000))
    assert 0.3 < got.mean() < 0.95


@pytest.mark.parametrize("ids", ["dense", "spread"])
@pytest.mark.parametrize("seed", range(6))
def test_http_random_policies(gpu, seed, ids):
    """Random policies (header matchers of every kind, ports, remotes) on the
    GPU: both class-mode and byte-mode programs, and both remote lookups
    (the direct identity array for a dense span, the bucket table for a
    spread one)."""
    import random
    from test_cpu_differential import ID_SETS, _rand_policy, _rand_requests
    rng = random.Random(100 + seed)
    pols = _rand_policy(rng, ids=ID_SETS[ids])
    rq = _rand_requests(rng, 3000, len(pols), ids=ID_SETS[ids])
    try:
        orc = oracle.HttpOracle(pols)
    except ValueError:
        return
    gpu.update_http_policy(pols)
    assert np.array_equal(gpu.http_verdicts(gpu.pack_http(**rq)), orc.eval(**rq))


@pytest.mark.parametrize("seed", range(4))
def test_http_all_matcher_forms(gpu, seed):
    """prefix / suffix / range / invert_match / empty exact on the GPU
    against the oracle's matchHeaders restatement."""
    from test_cpu_differential import all_matcher_case
    pols, rq, _ = all_matcher_case(seed, 4000)
    gpu.update_http_policy(pols)
    assert np.array_equal(gpu.http_verdicts(gpu.pack_http(**rq)), oracle.HttpOracle(pols).eval(**rq))


def test_http_many_byte_classes(gpu):
    """A program over more than 64 byte classes keeps byte-indexed comb rows
    (the class-code packing needs a class code in one byte): 90 exact paths
    of distinct characters, requests hitting and missing them."""
    chars = [chr(c) for c in range(0x21, 0x7B) if chr(c) not in "\\"][:90]
    rules = [{"headers": [{"name": ":path", "exact_match": "/" + c + c}]} for c in chars]
    pols = [{"name": "many", "policy": 0, "ingress_per_port_policies": [
        {"port": 80, "protocol": "TCP", "rules": [{"remote_policies": [], "http_rules": {"http_rules": rules}}]}]}]
    rng = np.random.default_rng(3)
    reqs = []
    for i in range(4000):
        c, d = chars[int(rng.integers(0, len(chars)))], chars[int(rng.integers(0, len(chars)))]
        reqs.append([(":path", "/" + c + (c if i % 2 else d)), (":method", "GET")])
    parts, off = [], [0]
    for hs in reqs:
        b = b"".join(k.encode() + b"\0" + v.encode() + b"\0" for k, v in hs)
        parts.append(b)
        off.append(off[-1] + len(b))
    n = len(reqs)
    rq = dict(policy=np.zeros(n, np.uint32), ingress=np.ones(n, np.uint8), port=np.full(n, 80, np.uint16),
              remote=np.arange(n, dtype=np.uint32) % 7, hdr_blob=np.frombuffer(b"".join(parts), np.uint8).copy(),
              hdr_off=np.array(off, np.uint64))
    got = _http_check(gpu, pols, rq)
    assert got.any() and not got.all()


def test_http_overflow_records(gpu):
    pols = synth.starwars_policy()
    rq = synth.starwars_requests(3000, seed=11)
    # make every third request longer than the 128-byte slot
    reqs = []
    blob, off = rq["hdr_blob"].tobytes(), rq["hdr_off"]
    for i in range(len(off) - 1):
        b = blob[off[i]:off[i + 1]]
        if i % 3 == 0:
            b = b.replace(b":path\0/v1/", b":path\0/v1/" + b"z" * (130 + i % 200), 1)
        reqs.append(b)
    rq["hdr_blob"] = np.frombuffer(b"".join(reqs), np.uint8).copy()
    rq["hdr_off"] = np.concatenate([[0], np.cumsum([len(b) for b in reqs])]).astype(np.uint64)
    _http_check(gpu, pols, rq)


def test_http_counters(gpu):
    pols = synth.starwars_policy()
    rq = synth.starwars_requests(10_000, seed=5)
    gpu.update_http_policy(pols)
    b = gpu.pack_http(**rq)
    got = gpu.http_verdicts(b)
    c = gpu.read_counters(0)
    # every request maps to a program (port 80) or to "no policy for port" (8080)
    on80 = rq["port"] == 80
    assert int(c[0::2].sum()) == int(got[on80].sum())
    assert int(c[1::2].sum()) == int((1 - got[on80]).sum())


# --------------------------------------------------------------- Kafka ----
def test_kafka_parity(gpu):
    pols, info = synth.kafka_policy()
    gpu.update_kafka_policy(pols)
    rq = synth.kafka_requests(200_000, info)
    reqs, arena = gpu.pack_kafka(**rq)
    got = gpu.kafka_verdicts(reqs, arena)
    exp = oracle.KafkaOracle(pols).eval(**rq, nthreads=8)
    assert np.array_equal(got, exp)
    assert 0.05 < got.mean() < 0.99
    # per-redirect counters: one redirect, every request counted once
    c = gpu.read_counters(1)
    assert int(c[0]) == int(got.sum()) and int(c[1]) == len(got) - int(got.sum())


def test_kafka_edge_parity(gpu):
    """Summary bits, exception rules, topic lists and unknown keys/kinds on
    the device, against the oracle (cases of test_kafka_edge_rules)."""
    import random

    from test_cpu_differential import _kafka_edge_policy
    for seed in range(6):
        rng = random.Random(seed)
        pols, topics, clients = _kafka_edge_policy(rng)
        gpu.update_kafka_policy(pols)
        n = 5000
        rq = dict(redirect=[rng.choice([0, 0, 1, 2]) for _ in range(n)],
                  remote=[rng.choice([0, 7, 8, 9, 10, 11]) for _ in range(n)],
                  api_key=[rng.choice([0, 1, 3, 10, 12, 18, 37, -1, 40, 63, 64, 1000]) for _ in range(n)],
                  api_version=[rng.choice([0, 1, 5, 63, 64, 100, -1, 32767, -32768]) for _ in range(n)],
                  kind=[rng.choice([0, 1, 2, 3]) for _ in range(n)],
                  client_id=[rng.choice(clients + ["zz"]).encode() for _ in range(n)],
                  topics=[[rng.choice(topics + ["nope"]).encode() for _ in range(rng.choice([0, 0, 1, 2, 3, 14]))]
                          for _ in range(n)])
        reqs, arena = gpu.pack_kafka(**rq)
        got = gpu.kafka_verdicts(reqs, arena)
        assert np.array_equal(got, oracle.KafkaOracle(pols).eval(**rq)), f"seed {seed}"


@pytest.mark.gpu
def test_gpu_kafka_split_layout(gpu):
    """cg_kafka_verdicts_split_dev: the same verdicts and per-redirect
    counters as the 64-byte records (and the oracle), with heads and topic
    tails in separate arrays — overflow-arena topic lists included."""
    import torch
    pols, info = synth.kafka_policy(n_rules=400, n_topics=60, n_clients=12, seed=5)
    gpu.update_kafka_policy(pols)
    rq = synth.kafka_requests(300_000, info, seed=6)
    reqs, arena = gpu.pack_kafka(**rq)
    exp = oracle.KafkaOracle(pols).eval(**rq, nthreads=16)
    n = len(reqs)
    raw = reqs.view(np.uint8).reshape(n, 64)
    dev = torch.device("cuda", 0)
    d_heads = torch.from_numpy(np.ascontiguousarray(raw[:, :16])).to(dev)
    d_topics = torch.from_numpy(np.ascontiguousarray(raw[:, 16:])).to(dev)
    d_arena = torch.from_numpy(arena if len(arena) else np.zeros(1, np.uint32)).to(dev)
    d_out = torch.full((n,), 9, dtype=torch.uint8, device=dev)
    gpu.reset_counters()
    s = torch.cuda.current_stream().cuda_stream
    gpu.kafka_verdicts_split_dev(d_heads, d_topics, n, d_arena, d_out, stream=s)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy(), exp)
    c_split = gpu.read_counters(1).copy()
    gpu.reset_counters()
    d_reqs = torch.from_numpy(raw.copy()).to(dev)
    gpu.kafka_verdicts_dev(d_reqs, n, d_arena, d_out, stream=s)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy(), exp)
    assert np.array_equal(gpu.read_counters(1), c_split)
