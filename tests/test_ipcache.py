"""ipcache: IP → security identity.

Reference: cilium_ipcache (bpf/lib/maps.h:135-159), lookup_ip{4,6}_remote_endpoint
(bpf/lib/eps.h:48-115) and the callers' resolution (bpf_lxc.c:509-518: a hit
with sec_label != 0 gives {sec_label, tunnel_endpoint}, else WORLD_ID), map ops
of pkg/maps/ipcache/ipcache.go:36-130.

The reference has no unit test of the LPM lookup itself (pkg/maps/ipcache has
no _test.go); the KAT below is written from the branch structure of those
lines.  The agent-side tests of pkg/ipcache (ipcache_test.go TestIPCache,
TestKeyToIPNet) are replayed at the end of this file as the map ops and
lookups they imply — they pin host keys, update/delete and prefix parsing
against the reference's own cases, but no longest-prefix choice between
overlapping CIDRs (partially pinned).  The oracle is oracle.cc `or_ipcache` (the
LPM_LOOKUP_FN probe order, eps.h:86-108); the product's tables are checked
against it on the CPU (host walker of the same tables) and on the GPU.
"""
import ipaddress

import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import synth

WORLD = N.CG_WORLD_ID
TUN = 0x0101010A  # 10.1.1.1 stored as bytes

KAT_ENTRIES = [
    ("10.0.0.0/8", 100, 0),
    ("10.1.0.0/16", 200, 0),
    ("10.1.2.0/24", 0, 0),          # sec_label 0: shadows the /16, resolves to WORLD
    ("10.1.2.3/32", 300, TUN),
    ("192.168.0.0/31", 400, TUN),
    ("255.255.255.255/32", 500, 0),
    ("fd00::/8", 1100, 0),
    ("fd00:1::/64", 1200, 0),
    ("fd00:1::/96", 0, 0),
    ("fd00:1::5/128", 1300, TUN),
    ("::/0", 1400, 0),               # v6 default route
    ("ffff:ffff:ffff:ffff:ffff:ffff:ffff:ffff/128", 1500, 0),
]
KAT_V4 = [
    ("10.1.2.3", (300, TUN)), ("10.1.2.4", (WORLD, 0)), ("10.1.3.1", (200, 0)), ("10.2.0.0", (100, 0)),
    ("10.255.255.255", (100, 0)), ("11.0.0.1", (WORLD, 0)), ("0.0.0.0", (WORLD, 0)),
    ("192.168.0.1", (400, TUN)), ("192.168.0.2", (WORLD, 0)), ("255.255.255.255", (500, 0)),
    ("255.255.255.254", (WORLD, 0)),
]
KAT_V6 = [
    ("fd00:1::5", (1300, TUN)), ("fd00:1::6", (WORLD, 0)), ("fd00:1::1:0:0", (1200, 0)),
    ("fd00:2::1", (1100, 0)), ("fe80::1", (1400, 0)), ("::", (1400, 0)),
    ("ffff:ffff:ffff:ffff:ffff:ffff:ffff:ffff", (1500, 0)), ("ffff:ffff:ffff:ffff:ffff:ffff:ffff:fffe", (1400, 0)),
]


def _kat_arrays():
    v4 = np.array([int.from_bytes(ipaddress.ip_address(a).packed, "little") for a, _ in KAT_V4], np.uint32)
    v6 = np.array([list(ipaddress.ip_address(a).packed) for a, _ in KAT_V6], np.uint8)
    e4 = np.array([x for _, x in KAT_V4], np.uint32)
    e6 = np.array([x for _, x in KAT_V6], np.uint32)
    return v4, v6, e4, e6


def _kat_map(cl):
    ic = cl.ipcache()
    ic.update([c for c, _, _ in KAT_ENTRIES], [[i, t] for _, i, t in KAT_ENTRIES])
    return ic


def _kat_keys():
    from cilium_amd.classifier import IPCache
    k = IPCache._keys([c for c, _, _ in KAT_ENTRIES])
    v = np.array([[i, t] for _, i, t in KAT_ENTRIES], np.uint32)
    return k, v


# ------------------------------------------------------------------ CPU ----
def test_oracle_kat():
    k, v = _kat_keys()
    v4, v6, e4, e6 = _kat_arrays()
    o4, o6 = oracle.ipcache(k, v, v4, v6)
    assert np.array_equal(o4, e4)
    assert np.array_equal(o6, e6)


def test_tables_kat(host):
    ic = _kat_map(host)
    v4, v6, e4, e6 = _kat_arrays()
    g4, g6 = ic.eval_host_diag(v4, v6)
    assert np.array_equal(g4, e4)
    assert np.array_equal(g6, e6)


def test_map_ops(host):
    ic = host.ipcache(max_entries=4)
    ic.upsert("10.0.0.0/8", 7)
    ic.upsert("10.0.0.1/8", 8)  # same key after masking: overwritten (BPF_ANY)
    assert ic.lookup("10.0.0.0/8") == (8, 0)
    assert ic.lookup("10.0.0.0/9") is None
    ic.update(["1.2.3.4/32", "fd00::/8"], [[9, 1], [10, 0]])
    with pytest.raises(N.CiliumGPUError) as ei:  # 3 + 2 new > 4: nothing applied
        ic.update(["2.0.0.0/8", "3.0.0.0/8"], [[1, 0], [2, 0]])
    assert ei.value.code == N.CG_MAP_FULL
    assert len(ic.dump()) == 3
    with pytest.raises(N.CiliumGPUError) as ei:  # one absent key: nothing deleted
        ic.delete(["1.2.3.4/32", "9.9.9.9/32"])
    assert ei.value.code == N.CG_NOT_FOUND
    ic.delete(["1.2.3.4/32"])
    assert ic.dump() == [("10.0.0.0/8", 8, 0), ("fd00::/8", 10, 0)]
    # delete + re-resolve rebuilds the tables
    g4, _ = ic.eval_host_diag(np.array([int.from_bytes(bytes([1, 2, 3, 4]), "little")], np.uint32),
                              np.zeros((0, 16), np.uint8))
    assert g4.tolist() == [[WORLD, 0]]


def test_empty_map(host):
    ic = host.ipcache()
    v4 = np.arange(1000, dtype=np.uint32) * 4294967
    v6 = np.random.default_rng(1).integers(0, 256, (100, 16), dtype=np.uint8)
    g4, g6 = ic.eval_host_diag(v4, v6)
    assert (g4 == [WORLD, 0]).all() and (g6 == [WORLD, 0]).all()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tables_random_vs_oracle(host, seed):
    rng = np.random.default_rng(seed)
    k, v = synth.ipcache_entries(int(rng.integers(2000, 40000)), n_nodes=int(rng.integers(4, 300)), seed=seed)
    a4, a6 = synth.ipcache_addresses(200_000, k, seed=seed)
    ic = host.ipcache()
    ic.update(k, v)
    g4, g6 = ic.eval_host_diag(a4, a6)
    o4, o6 = oracle.ipcache(k, v, a4, a6, nthreads=4)
    assert np.array_equal(g4, o4)
    assert np.array_equal(g6, o6)


def test_tables_nested_dense(host):
    """Deeply nested prefixes on one path (every length 0..32 / 0..128 over the
    same address, alternating zero identities) plus their neighbours."""
    from cilium_amd.classifier import CIDR_DTYPE
    rng = np.random.default_rng(7)
    base4 = bytes([172, 16, 99, 201])
    base6 = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    keys, vals = [], []
    for plen in range(33):
        keys.append(str(ipaddress.ip_network((base4, plen), strict=False)))
        vals.append([0 if plen % 5 == 3 else 1000 + plen, plen])
    for plen in range(129):
        keys.append(str(ipaddress.ip_network((base6, plen), strict=False)))
        vals.append([0 if plen % 7 == 2 else 5000 + plen, plen])
    ic = host.ipcache()
    ic.update(keys, vals)
    from cilium_amd.classifier import IPCache
    k = IPCache._keys(keys)
    b4 = int.from_bytes(base4, "big")
    a4 = np.array([(b4 ^ (1 << s)) for s in range(32)] + [b4], np.uint32).astype(">u4").view("<u4")
    b6 = int.from_bytes(base6, "big")
    a6 = np.array([list(((b6 ^ (1 << s)) % (1 << 128)).to_bytes(16, "big")) for s in range(128)] + [list(base6)],
                  np.uint8)
    g4, g6 = ic.eval_host_diag(a4, a6)
    o4, o6 = oracle.ipcache(k, np.array(vals, np.uint32), a4, a6)
    assert np.array_equal(g4, o4)
    assert np.array_equal(g6, o6)
    assert CIDR_DTYPE.itemsize == 20


def v4_chunk_kinds_case():
    """IPv4 chunks in every encoding (dev_types.h ipc_chunk_get): dense /32-
    and /24-level chunks (every entry distinct), sparse maps whose set keys
    sit on the 56-key map word edges, run lines of exactly 7 runs and sparse
    ones of 8, with every address of those /24s probed."""
    keys, vals, probe = [], [], []

    def add(net, ident, tun=0):
        keys.append(net)
        vals.append([ident, tun])

    for k in range(256):  # 10.9.9.0/24: 256 distinct /32s (dense /32 chunk)
        add(f"10.9.9.{k}/32", 7000 + k, k)
    for k in range(256):  # 10.8.0.0/16: 256 distinct /24s (dense /24 chunk)
        add(f"10.8.{k}.0/24", 8000 + k)
    edges = [0, 1, 54, 55, 56, 57, 111, 112, 113, 167, 168, 223, 224, 225, 254, 255]
    for k in edges:  # sparse /32 chunk over a /24 background
        add(f"10.7.7.{k}/32", 9000 + k, 1)
    add("10.7.7.0/24", 9999)
    for k in edges:  # sparse /24 chunk (/24s of one /16, alternating zero identities)
        add(f"10.6.{k}.0/24", 0 if k % 3 == 0 else 6000 + k)
    add("10.6.0.0/16", 6999)
    for n, net in ((7, "10.5.5"), (8, "10.4.4")):  # 7 runs (a run line), 8 runs (sparse)
        for r in range((n + 1) // 2):
            add(f"{net}.{40 * r + 7}/32", 5000 + 10 * n + r)
    for p in ("10.9.9", "10.7.7", "10.5.5", "10.4.4"):
        probe += [f"{p}.{k}" for k in range(256)]
    probe += [f"10.8.{k}.{(k * 37) & 255}" for k in range(256)] + [f"10.6.{k}.9" for k in range(256)]
    a4 = np.array([int.from_bytes(ipaddress.ip_address(a).packed, "little") for a in probe], np.uint32)
    return keys, np.array(vals, np.uint32), a4


def exact_shadow_case():
    """Full-length entries (the exact tables) against shorter prefixes around
    them: a /32 or /128 with identity 0 shadows its covering prefix (WORLD),
    a /32 beside a /31, the first and last addresses of a family, a /16
    holding only /32s, and a v6 bucket whose only entries are /128s."""
    ents = [("10.20.0.0/16", 700, 0), ("10.20.5.7/32", 0, 0), ("10.20.5.8/32", 701, 3),
            ("10.20.5.9/31", 702, 0), ("10.20.5.10/32", 703, 0), ("0.0.0.0/32", 704, 0),
            ("255.255.255.255/32", 705, 0), ("10.21.1.1/32", 706, 0), ("10.21.200.3/32", 707, 0),
            ("fd10::/32", 800, 0), ("fd10::7/128", 0, 0), ("fd10::8/128", 801, 5), ("fd10::9/127", 802, 0),
            ("::/128", 803, 0), ("ffff:ffff:ffff:ffff:ffff:ffff:ffff:ffff/128", 804, 0),
            ("fd77:1:2:3::1/128", 805, 0), ("fd77:1:2:3::2/128", 806, 0)]
    a4 = ["10.20.5.%d" % k for k in range(4, 14)] + ["0.0.0.0", "0.0.0.1", "255.255.255.255", "255.255.255.254",
                                                    "10.21.1.1", "10.21.1.2", "10.21.200.3", "10.21.0.0"]
    a6 = ["fd10::%x" % k for k in range(4, 14)] + ["::", "::1", "ffff:ffff:ffff:ffff:ffff:ffff:ffff:ffff",
                                                 "fd77:1:2:3::1", "fd77:1:2:3::2", "fd77:1:2:3::3", "fd77:1:2::"]
    keys = [c for c, _, _ in ents]
    vals = np.array([[i, t] for _, i, t in ents], np.uint32)
    v4 = np.array([int.from_bytes(ipaddress.ip_address(x).packed, "little") for x in a4], np.uint32)
    v6 = np.array([list(ipaddress.ip_address(x).packed) for x in a6], np.uint8)
    return keys, vals, v4, v6


def _check_exact_shadow(cl, lookup):
    from cilium_amd.classifier import IPCache
    keys, vals, v4, v6 = exact_shadow_case()
    ic = cl.ipcache()
    ic.update(keys, vals)
    g4, g6 = lookup(ic, v4, v6)
    o4, o6 = oracle.ipcache(IPCache._keys(keys), vals, v4, v6)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6)
    assert o4[3].tolist() == [WORLD, 0] and o4[4].tolist() == [701, 3]  # 10.20.5.7 (identity 0), .8
    assert o6[3].tolist() == [WORLD, 0] and o6[4].tolist() == [801, 5]


def test_tables_exact_shadow(host):
    _check_exact_shadow(host, lambda ic, a4, a6: ic.eval_host_diag(a4, a6))


def _check_chunk_kinds(cl, lookup):
    from cilium_amd.classifier import IPCache
    keys, vals, a4 = v4_chunk_kinds_case()
    ic = cl.ipcache()
    ic.update(keys, vals)
    a6 = np.zeros((0, 16), np.uint8)
    g4, _ = lookup(ic, a4, a6)
    o4, _ = oracle.ipcache(IPCache._keys(keys), vals, a4, a6)
    assert np.array_equal(g4, o4)
    assert len(np.unique(o4[:, 0])) > 500


@pytest.mark.parametrize("encode", [False, True])
def test_tables_v4_chunk_kinds(host, monkeypatch, encode):
    if encode:  # run lines and sparse maps (ipcache.cc; dense chunks by default)
        monkeypatch.setenv("CILIUM_GPU_IPC_ENCODE", "1")
    _check_chunk_kinds(host, lambda ic, a4, a6: ic.eval_host_diag(a4, a6))


def v6_bucket_case(seed: int):
    """IPv6 top-bits buckets of every kind: spanned by one WORLD run (bit
    clear), spanned by one non-WORLD run (short prefixes), a few runs, and
    crowded ones (a node /64 of pods: the 64-way crowd line; and ~800
    runs: a plain binary search), with the first
    and last buckets taken, and addresses on and beside every run edge."""
    import random
    rnd = random.Random(200 + seed)
    nets = []
    for _ in range(40):  # whole buckets, some with identity 0
        nets.append((rnd.getrandbits(128), rnd.randrange(6, 20)))
    crowd = rnd.getrandbits(16) << 112  # 400 prefixes under one /16
    for _ in range(400):
        nets.append((crowd | rnd.getrandbits(112), rnd.randrange(40, 129)))
    for _ in range(400):
        nets.append((rnd.getrandbits(128), rnd.randrange(24, 129)))
    pods = rnd.getrandbits(64) << 64  # a node /64 of 40 pods: a crowded bucket (8..255 runs)
    nets += [(pods | rnd.getrandbits(64), 128) for _ in range(40)]
    near = pods | (rnd.getrandbits(8) << 56)  # and 30 pods sharing 72 bits (a narrow window)
    nets += [(near | rnd.getrandbits(56), 128) for _ in range(30)]
    nets += [(0, 24), ((1 << 128) - 1, 128), (((1 << 16) - 1) << 112, 16)]
    keys, vals, edges = [], [], []
    for a, plen in nets:
        net = ipaddress.IPv6Network((a, plen), strict=False)
        keys.append(str(net))
        vals.append([0 if len(vals) % 9 == 4 else 3000 + len(vals), len(vals)])
        lo, hi = int(net.network_address), int(net.broadcast_address)
        edges += [lo, hi, (lo - 1) % (1 << 128), (hi + 1) % (1 << 128)]
    addrs = edges + [rnd.getrandbits(128) for _ in range(2000)] + \
        [crowd | rnd.getrandbits(112) for _ in range(2000)] + \
        [pods | rnd.getrandbits(64) for _ in range(1000)] + [near | rnd.getrandbits(56) for _ in range(1000)]
    a6 = np.array([list(x.to_bytes(16, "big")) for x in addrs], np.uint8)
    return keys, np.array(vals, np.uint32), a6


@pytest.mark.parametrize("seed", range(2))
def test_tables_v6_buckets(host, seed):
    from cilium_amd.classifier import IPCache
    keys, vals, a6 = v6_bucket_case(seed)
    ic = host.ipcache()
    ic.update(keys, vals)
    a4 = np.zeros(1, np.uint32)
    g4, g6 = ic.eval_host_diag(a4, a6)
    o4, o6 = oracle.ipcache(IPCache._keys(keys), vals, a4, a6)
    assert np.array_equal(g6, o6)
    assert 0.05 < (o6[:, 0] == WORLD).mean() < 0.95


def test_host_handle_refuses_resolve(host):
    ic = host.ipcache()
    with pytest.raises(N.CiliumGPUError) as ei:
        ic.resolve(np.zeros(4, np.uint32), np.zeros((0, 16), np.uint8))
    assert ei.value.code == N.CG_NO_DEVICE


# ------------------------------------------------------------------ GPU ----
@pytest.mark.gpu
def test_gpu_exact_shadow(gpu):
    _check_exact_shadow(gpu, lambda ic, a4, a6: ic.resolve(a4, a6))


@pytest.mark.gpu
@pytest.mark.parametrize("encode", [False, True])
def test_gpu_v4_chunk_kinds(gpu, monkeypatch, encode):
    if encode:
        monkeypatch.setenv("CILIUM_GPU_IPC_ENCODE", "1")
    _check_chunk_kinds(gpu, lambda ic, a4, a6: ic.resolve(a4, a6))


@pytest.mark.gpu
def test_gpu_encoded_tables_random_vs_oracle(gpu, monkeypatch):
    """The encoded v4 chunks on the random workload of test_gpu_random."""
    monkeypatch.setenv("CILIUM_GPU_IPC_ENCODE", "1")
    k, v = synth.ipcache_entries(30000, n_nodes=200, seed=9)
    a4, a6 = synth.ipcache_addresses(300_000, k, seed=9)
    ic = gpu.ipcache()
    ic.update(k, v)
    g4, g6 = ic.resolve(a4, a6)
    o4, o6 = oracle.ipcache(k, v, a4, a6, nthreads=8)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6)


@pytest.mark.gpu
def test_gpu_kat(gpu):
    ic = _kat_map(gpu)
    v4, v6, e4, e6 = _kat_arrays()
    g4, g6 = ic.resolve(v4, v6)
    assert np.array_equal(g4, e4)
    assert np.array_equal(g6, e6)


@pytest.mark.gpu
def test_gpu_parity_full_map(gpu):
    k, v = synth.ipcache_entries()
    a4, a6 = synth.ipcache_addresses(2_000_000, k)
    ic = gpu.ipcache()
    ic.update(k, v)
    g4, g6 = ic.resolve(a4, a6)
    o4, o6 = oracle.ipcache(k, v, a4, a6, nthreads=16)
    assert np.array_equal(g4, o4)
    assert np.array_equal(g6, o6)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(2))
def test_gpu_v6_buckets(gpu, seed):
    from cilium_amd.classifier import IPCache
    keys, vals, a6 = v6_bucket_case(seed)
    ic = gpu.ipcache()
    ic.update(keys, vals)
    a4 = np.zeros(1, np.uint32)
    g4, g6 = ic.resolve(a4, a6)
    o4, o6 = oracle.ipcache(IPCache._keys(keys), vals, a4, a6)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6)


@pytest.mark.gpu
def test_gpu_empty_ragged_and_update(gpu):
    k, v = synth.ipcache_entries(20_000, n_nodes=64, seed=5)
    ic = gpu.ipcache()
    g4, g6 = ic.resolve(np.zeros(0, np.uint32), np.zeros((0, 16), np.uint8))
    assert g4.shape == (0, 2) and g6.shape == (0, 2)
    g4, g6 = ic.resolve(np.arange(7, dtype=np.uint32), np.zeros((3, 16), np.uint8))  # empty map
    assert (g4 == [WORLD, 0]).all() and (g6 == [WORLD, 0]).all()
    ic.update(k, v)
    for n in (1, 3, 255, 1025, 100_003):
        a4, a6 = synth.ipcache_addresses(n, k, seed=n)
        g4, g6 = ic.resolve(a4, a6)
        o4, o6 = oracle.ipcache(k, v, a4, a6)
        assert np.array_equal(g4, o4) and np.array_equal(g6, o6), n
    # delete half the entries: the next resolve rebuilds the device tables
    ic.delete(k[::2])
    a4, a6 = synth.ipcache_addresses(100_000, k, seed=9)
    g4, g6 = ic.resolve(a4, a6)
    o4, o6 = oracle.ipcache(k[1::2], v[1::2], a4, a6)
    assert np.array_equal(g4, o4) and np.array_equal(g6, o6)


# ----------------------- ipcache → L4 egress (bpf_lxc.c:509-527 v4, :205-220 v6)
def _ipc_l4_case(n_entries: int, n: int, seed: int, family: int = 4):
    """Tuples whose flags include ingress and fragment bits: the egress flow
    must ignore both (policy_can_egress4/6 pass CT_EGRESS and is_fragment
    false, bpf/lib/policy.h:150-177)."""
    keys, ports = synth.l4_table(n_entries=n_entries, n_ids=1024, seed=seed)
    ids = np.unique(keys["sec_label"])
    ik, iv = synth.ipcache_entries(20_000, n_nodes=64, seed=seed)
    rng = np.random.default_rng(seed)
    iv = iv.copy()
    iv[:, 0] = rng.choice(np.append(ids, [0, 2, 999_999]), len(iv))
    a4, a6 = synth.ipcache_addresses(n, ik, seed=seed)
    remote = a4 if family == 4 else np.ascontiguousarray(a6, np.uint8).reshape(-1, 16)
    tuples = synth.l4_tuples(len(remote), keys, n_ids=1024, seed=seed)
    tuples["flags"] |= rng.choice(np.array([0, 1, 2, 3], np.uint8), len(tuples), p=[0.4, 0.4, 0.1, 0.1])
    exp, pk, by = oracle.l4_egress_via_ipcache(keys, ports, ik, iv, remote, tuples)
    return keys, ports, ik, iv, remote, tuples, exp, pk, by


@pytest.mark.gpu
@pytest.mark.parametrize("family", [4, 6])
@pytest.mark.parametrize("n_entries", [2048, 65536])  # LDS-fingerprint kernel and the global one
def test_gpu_l4_via_ipcache(gpu, n_entries, family):
    keys, ports, ik, iv, remote, tuples, exp, pk, by = _ipc_l4_case(n_entries, 300_000, 7, family)
    pm = gpu.policy_map(max_entries=max(n_entries, 16384))
    pm.allow_keys(keys, ports)
    ic = gpu.ipcache()
    ic.update(ik, iv)
    got = pm.verdicts_via_ipcache(ic, remote, tuples)
    assert np.array_equal(got, exp)
    # egress wrapper: only DROP_POLICY, never DROP_FRAG_NOSUPPORT
    assert (exp == 0).any() and (exp == -133).any() and not (exp == -157).any()
    dump = {(k.Identity, k.DestPort, k.Nexthdr, k.TrafficDirection): e for k, e in pm.dump_to_slice()}
    for i in range(0, len(keys), 61):
        k = keys[i]
        e = dump[(int(k["sec_label"]), int(k["dport"]), int(k["protocol"]), int(k["egress"]))]
        assert (e.Packets, e.Bytes) == (int(pk[i]), int(by[i]))


# ------------- replay of the reference's own ipcache tests (pkg/ipcache) ----
# TestIPCache (pkg/ipcache/ipcache_test.go:37-176) drives the agent-side cache,
# whose listener turns each effective change into one BPF map op
# (pkg/datapath/ipcache/listener.go:97-119: Upsert → Map.Update of the host
# /32 or /128 key, Delete → Map.Delete).  The steps below are that test's
# sequence reduced to the map ops it produces — calls the agent drops make no
# op: Delete of an absent IP (ipcache.go:347-350), a Kubernetes-source upsert
# over a kvstore entry (ipcache.go:233-236, test line 63) and an upsert of the
# same identity (ipcache.go:240-242, test line 69) — and each LookupByIP /
# LookupByPrefix assertion becomes an expected datapath resolve / exact-key
# lookup (test file line in the comment).
REF_IPCACHE_STEPS = [
    ("upsert", "10.0.0.15", 68), ("expect", "10.0.0.15", 68),              # :48-59
    ("delete", "10.0.0.15"), ("expect", "10.0.0.15", None),                # :78-86
    ("upsert", "10.0.0.15", 68), ("upsert", "10.0.0.15", 69),              # :88-97
    ("expect", "10.0.0.15", 69),
    ("delete", "10.0.0.15"),                                               # :110
    ("upsert", "192.168.0.1", 5), ("expect", "192.168.0.1", 5),            # :117-127
    ("upsert", "20.3.75.3", 67), ("expect", "20.3.75.3", 67),
    ("upsert", "27.2.2.2", 29), ("expect", "27.2.2.2", 29),
    ("upsert", "127.0.0.1", 29), ("expect", "127.0.0.1", 29),
    ("expect", "127.0.0.1", 29),                                           # 5th upsert: same identity, no op
    ("delete", "27.2.2.2"), ("expect", "27.2.2.2", None),                  # :137
    ("expect", "127.0.0.1", 29), ("prefix", "127.0.0.1/32", 29),           # :147-153
    ("delete", "127.0.0.1"), ("prefix", "127.0.0.1/32", None),             # :155-161
    ("delete", "192.168.0.1"), ("expect", "192.168.0.1", None),            # :164-171
    ("delete", "20.3.75.3"), ("expect", "20.3.75.3", None),
]
# TestKeyToIPNet (ipcache_test.go:178-243): the kvstore keys' IP part and the
# net.ParseCIDR result it must equal; host keys are full-length prefixes.
REF_KEY_NETS = [("f00d::a00:0:0:c164", "f00d::a00:0:0:c164/128", True),
                ("f00d::a00:0:0:0/64", "f00d::a00:0:0:0/64", False),
                ("10.0.114.197", "10.0.114.197/32", True),
                ("10.0.114.0/24", "10.0.114.0/24", False)]
REF_KEY_BAD = ["10.abfd.114.197", "192.0.2.3/54"]  # ipcache_test.go:231, :238


def _host_key(ip: str) -> str:
    a = ipaddress.ip_address(ip)
    return f"{ip}/{a.max_prefixlen}"


def _addr_arrays(ips):
    v4 = [ip for ip in ips if ipaddress.ip_address(ip).version == 4]
    v6 = [ip for ip in ips if ipaddress.ip_address(ip).version == 6]
    a4 = np.array([int.from_bytes(ipaddress.ip_address(a).packed, "little") for a in v4], np.uint32)
    a6 = np.array([list(ipaddress.ip_address(a).packed) for a in v6], np.uint8).reshape(-1, 16)
    return v4, v6, a4, a6


def _replay_ref_steps(cl, resolve):
    ic = cl.ipcache()
    checked = 0
    for step in REF_IPCACHE_STEPS:
        op, ip = step[0], step[1]
        if op == "upsert":
            ic.upsert(_host_key(ip), step[2])
        elif op == "delete":
            ic.delete([_host_key(ip)])
        elif op == "prefix":
            got = ic.lookup(ip)
            assert (got[0] if got else None) == step[2], step
            checked += 1
        else:
            _, _, a4, a6 = _addr_arrays([ip])
            g4, g6 = resolve(ic, a4, a6)
            g = (g4 if len(a4) else g6)[0]
            assert tuple(g.tolist()) == ((step[2], 0) if step[2] is not None else (WORLD, 0)), step
            checked += 1
    assert ic.dump() == []  # the test ends with both caches empty (:173-174)
    return checked


def _key_net_case(cl, resolve):
    for bad in REF_KEY_BAD:
        with pytest.raises(ValueError):
            IPCacheKeys([bad])
    ic = cl.ipcache()
    keys = [k for k, _, _ in REF_KEY_NETS]
    ic.update(keys, [[1000 + i, 0] for i in range(len(keys))])
    assert sorted(c for c, _, _ in ic.dump()) == sorted(str(ipaddress.ip_network(n, strict=False)) for _, n, _ in REF_KEY_NETS)
    for i, (k, net, host) in enumerate(REF_KEY_NETS):
        assert ic.lookup(net) == (1000 + i, 0)
        nw = ipaddress.ip_network(net, strict=False)  # net.ParseCIDR masks: f00d::a00:0:0:0/64 is f00d::/64
        assert (nw.prefixlen == nw.max_prefixlen) == host
    # the host key shadows its /64 or /24; the rest of the prefix resolves to it
    ips = ["f00d::a00:0:0:c164", "f00d::a00:0:0:c165", "f00d::a00:ffff:ffff:ffff", "f00d::ffff:0:0:0", "f00d:0:0:1::",
           "10.0.114.197", "10.0.114.196", "10.0.114.255", "10.0.115.197"]
    want = {"f00d::a00:0:0:c164": 1000, "f00d::a00:0:0:c165": 1001, "f00d::a00:ffff:ffff:ffff": 1001,
            "f00d::ffff:0:0:0": 1001, "f00d:0:0:1::": WORLD, "10.0.114.197": 1002, "10.0.114.196": 1003, "10.0.114.255": 1003,
            "10.0.115.197": WORLD}
    v4, v6, a4, a6 = _addr_arrays(ips)
    g4, g6 = resolve(ic, a4, a6)
    got = dict(zip(v4 + v6, [int(x) for x in g4[:, 0]] + [int(x) for x in g6[:, 0]]))
    assert got == want


def IPCacheKeys(keys):
    from cilium_amd.classifier import IPCache
    return IPCache._keys(keys)


def test_ref_ipcache_replay_host(host):
    assert _replay_ref_steps(host, lambda ic, a4, a6: ic.eval_host_diag(a4, a6)) == 14


def test_ref_key_to_ipnet_host(host):
    _key_net_case(host, lambda ic, a4, a6: ic.eval_host_diag(a4, a6))


@pytest.mark.gpu
def test_gpu_ref_ipcache_replay(gpu):
    assert _replay_ref_steps(gpu, lambda ic, a4, a6: ic.resolve(a4, a6)) == 14


@pytest.mark.gpu
def test_gpu_ref_key_to_ipnet(gpu):
    _key_net_case(gpu, lambda ic, a4, a6: ic.resolve(a4, a6))


def test_destroy(host):
    ic = host.ipcache()
    ic.upsert("10.0.0.0/8", 5)
    ic.destroy()
    with pytest.raises(N.CiliumGPUError) as ei:
        ic.upsert("10.0.0.0/8", 5)
    assert ei.value.code == N.CG_NOT_FOUND
    pf = host.prefilter()
    pf.destroy()
    pm = host.policy_map()
    pm.destroy()
