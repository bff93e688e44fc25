"""Control-plane semantics mirrored from the reference (no GPU needed):
PreFilter revisions / map selection / undo (pkg/datapath/prefilter/prefilter.go)
and PolicyMap Allow / Delete / Dump / Flush (pkg/maps/policymap)."""
import ipaddress

import numpy as np
import pytest

from cilium_amd import _native as N
from cilium_amd.policy import PolicyKey, htons


class PyPreFilter:
    """Pure-Python restatement of PreFilter (prefilter.go:57-203) — the checker."""

    def __init__(self, dyn4, dyn6, fix4, fix6, max_lpm=65536, max_hash=20 << 20):
        self.revision = 1
        self.en = {"v4dyn": dyn4, "v4fix": fix4, "v6dyn": dyn6, "v6fix": fix4}  # :237 quirk
        self.maps = {k: set() for k in self.en}
        self.cap = {"v4dyn": max_lpm, "v6dyn": max_lpm, "v4fix": max_hash, "v6fix": max_hash}

    @staticmethod
    def select(net):
        ones, bits = net.prefixlen, net.max_prefixlen
        return ("v4" if bits == 32 else "v6") + ("fix" if ones == bits else "dyn")

    def insert(self, rev, cidrs):
        if rev != 0 and rev != self.revision:
            return N.CG_REVISION_MISMATCH
        undo = []
        for c in cidrs:
            net = ipaddress.ip_network(c, strict=False)
            w = self.select(net)
            if not self.en[w]:
                err = N.CG_NO_MAP
                break
            if net in self.maps[w]:
                undo.append((w, net))  # updated in place, still undone on failure (:141-158)
                continue
            if len(self.maps[w]) >= self.cap[w]:
                err = N.CG_MAP_FULL
                break
            self.maps[w].add(net)
            undo.append((w, net))
        else:
            self.revision += 1
            return N.CG_OK
        for w, net in undo:
            self.maps[w].discard(net)
        return err

    def delete(self, rev, cidrs):
        if rev != 0 and rev != self.revision:
            return N.CG_REVISION_MISMATCH
        nets = []
        for c in cidrs:
            net = ipaddress.ip_network(c, strict=False)
            w = self.select(net)
            if not self.en[w]:
                return N.CG_NO_MAP
            if net not in self.maps[w]:
                return N.CG_NOT_FOUND
            nets.append((w, net))
        for w, net in nets:
            self.maps[w].discard(net)
        self.revision += 1
        return N.CG_OK

    def dump(self):
        return sorted(str(n) for m in self.maps.values() for n in m)


def _call(fn, *a):
    try:
        fn(*a)
        return N.CG_OK
    except N.CiliumGPUError as e:
        return e.code


@pytest.mark.parametrize("cfg", [(False, False, True, True), (True, True, True, True), (True, False, False, True)])
def test_prefilter_control_plane(host, cfg):
    import random
    rng = random.Random(sum(cfg))
    pf = host.prefilter(*cfg, max_lpm=6, max_hash=8)
    ref = PyPreFilter(*cfg, max_lpm=6, max_hash=8)
    pool = ["10.0.0.0/8", "10.1.2.3/32", "192.168.0.0/16", "192.168.1.1", "2001:db8::/32", "2001:db8::1/128",
            "fe80::/10", "172.16.0.0/12", "1.2.3.4/32", "1.2.3.5/32", "10.1.2.3/8", "::/0", "0.0.0.0/0"]
    for step in range(200):
        op = rng.random()
        cidrs = rng.sample(pool, rng.randint(1, 3))
        rev = rng.choice([0, ref.revision, ref.revision - 1])
        if op < 0.6:
            exp = ref.insert(rev, cidrs)
            got = _call(pf.insert, rev, cidrs)
        else:
            exp = ref.delete(rev, cidrs)
            got = _call(pf.delete, rev, cidrs)
        assert got == exp, (step, cidrs, rev)
        d, r = pf.dump()
        assert r == ref.revision
        assert sorted(d) == ref.dump()


def test_prefilter_revision_and_errors(host):
    pf = host.prefilter()  # NewPreFilter default: fix4/fix6 only (prefilter.go:284-289)
    assert pf.dump() == ([], 1)
    with pytest.raises(N.CiliumGPUError) as ei:
        pf.insert(0, ["10.0.0.0/8"])  # dyn maps disabled
    assert ei.value.code == N.CG_NO_MAP
    assert pf.insert(1, ["10.0.0.1/32"]) == 2
    with pytest.raises(N.CiliumGPUError) as ei:
        pf.insert(1, ["10.0.0.2/32"])  # "Latest revision is 2 not 1"
    assert ei.value.code == N.CG_REVISION_MISMATCH
    assert pf.delete(0, ["10.0.0.1/32"]) == 3


def test_policymap_control_plane(host):
    pm = host.policy_map(max_entries=8)
    pm.allow(100, 80, 6, 0, 10000)
    pm.allow(100, 80, 6, 0, 10001)  # update in place
    pm.allow(0, 53, 17, 1, 0)
    assert pm.exists(100, 80, 6, 0) and not pm.exists(100, 81, 6, 0)
    e = pm.lookup(PolicyKey(100, htons(80), 6, 0))
    assert e.ProxyPort == htons(10001)
    dump = pm.dump_to_slice()
    assert {k for k, _ in dump} == {PolicyKey(100, htons(80), 6, 0), PolicyKey(0, htons(53), 17, 1)}
    with pytest.raises(N.CiliumGPUError) as ei:
        pm.delete(7, 7, 6, 0)
    assert ei.value.code == N.CG_NOT_FOUND
    pm.delete(100, 80, 6, 0)
    assert not pm.exists(100, 80, 6, 0)
    pm.flush()
    assert pm.dump_to_slice() == []
    with pytest.raises(N.CiliumGPUError):
        pm.allow_keys(np.array([(0xFFFFFFFF, 0xFFFF, 0xFF, 0xFF)], dtype=[("sec_label", "<u4"), ("dport", "<u2"),
                                                                             ("protocol", "u1"), ("egress", "u1")]),
                      np.zeros(1, np.uint16))


def test_policy_entries_dump_less():
    """policymap_test.go:31-143 TestPolicyEntriesDump_Less, case for case
    (Ingress = 0, Egress = 1: policymap.go TrafficDirection)."""
    from cilium_amd.classifier import PolicyEntriesDump, PolicyEntry
    e = PolicyEntry(0, 0, 0)

    def dump(*keys):
        return PolicyEntriesDump((PolicyKey(*k), e) for k in keys)
    cases = [("same element", dump((0, 0, 0, 0)), 0, 0, False),
             ("identity smaller", dump((0, 0, 0, 0), (1, 0, 0, 0)), 0, 1, True),
             ("direction smaller", dump((0, 0, 0, 0), (1, 0, 0, 1)), 0, 1, True),
             ("identity bigger", dump((1, 0, 0, 1), (0, 0, 0, 1)), 0, 1, False)]
    for name, p, i, j, want in cases:
        assert p.less(i, j) == want, name


def test_policymap_dump_sorted(host):
    pm = host.policy_map(max_entries=16)
    for ident, d in [(7, 1), (3, 0), (9, 0), (1, 1), (5, 0)]:
        pm.allow(ident, 80, 6, d, 0)
    s = pm.dump_to_slice().sorted()
    assert [(k.TrafficDirection, k.Identity) for k, _ in s] == [(0, 3), (0, 5), (0, 9), (1, 1), (1, 7)]
    assert all(not s.less(j, i) for i in range(len(s)) for j in range(i + 1, len(s)))


def test_http_policy_image_roundtrip():
    """cg_http_policy_export / _import: the compiled 10K-rule tables moved to
    another handle give identical verdicts (host walk), keep the policy index
    and rule info, and a damaged or truncated image is rejected with the
    previous snapshot still serving."""
    import numpy as np

    from cilium_amd import _native as N
    from cilium_amd import synth
    from cilium_amd.classifier import Classifier
    pols, info = synth.http10k_rules(n_rules=3000, n_ports=16)
    a, b = Classifier(device=-1), Classifier(device=-1)
    a.update_http_policy(pols)
    img = a.export_http_policy()
    b.import_http_policy(img)
    rq = synth.http10k_requests(20_000, info, seed=3)
    va = a.http_eval_host_diag(a.pack_http(**rq))
    vb = b.http_eval_host_diag(b.pack_http(**rq))
    assert np.array_equal(va, vb) and 0 < va.sum() < len(va)
    assert b.http_policy_index("ep-10k") == a.http_policy_index("ep-10k")
    assert np.array_equal(a.http_rule_info(), b.http_rule_info())
    assert a.http_policy_stats() == b.http_policy_stats()
    assert b.export_http_policy() == img  # the epoch is not part of the image
    bad = bytearray(img)
    bad[len(bad) // 2] ^= 1
    for blob in (bytes(bad), img[:-9], b"", img[:8]):
        rc = N.lib.cg_http_policy_import(b.h, blob, len(blob))
        assert rc == N.CG_POLICY_REJECTED
    assert np.array_equal(b.http_eval_host_diag(b.pack_http(**rq)), va)
    a.close()
    b.close()


def _fnv64(b: bytes) -> int:
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def _reseal(body: bytes) -> bytes:
    """An image body with a valid trailing FNV-64 (http_image.cc): FNV is no
    MAC, so the structural checks are what stands between a crafted image and
    the kernels."""
    return body + _fnv64(body).to_bytes(8, "little")


def test_http_policy_image_structural_corruption():
    """Images whose checksum is recomputed after damaging a word: every one is
    either rejected (CG_POLICY_REJECTED, the previous snapshot serving) or
    imported and then walked by the host verdict path without reading outside
    its tables (the walker runs under the ASan build in tools/sanitize)."""
    import numpy as np

    from cilium_amd import _native as N
    from cilium_amd import synth
    from cilium_amd.classifier import Classifier
    a, b = Classifier(device=-1), Classifier(device=-1)
    a.update_http_policy(synth.starwars_policy())
    img = a.export_http_policy()
    rq = synth.starwars_requests(300, seed=4)
    good = a.http_eval_host_diag(a.pack_http(**rq))
    body = bytearray(img[:-8])
    rng = np.random.default_rng(7)
    rejected = accepted = 0
    for k in range(600):
        bad = bytearray(body)
        for _ in range(int(rng.integers(1, 3))):
            i = int(rng.integers(8, len(bad) - 4)) & ~3  # a word past magic and version
            v = int.from_bytes(bad[i:i + 4], "little")
            v = [v ^ (1 << int(rng.integers(0, 32))), 0xFFFFFFFF, 0, v + 1, v + 0x10000, int(rng.integers(0, 2**32))][
                int(rng.integers(0, 6))] & 0xFFFFFFFF
            bad[i:i + 4] = v.to_bytes(4, "little")
        blob = _reseal(bytes(bad))
        rc = N.lib.cg_http_policy_import(b.h, blob, len(blob))
        if rc == N.CG_OK:
            accepted += 1
            try:
                b.http_eval_host_diag(b.pack_http(**rq))
            except N.CiliumGPUError:
                pass
        else:
            assert rc == N.CG_POLICY_REJECTED
            rejected += 1
    assert rejected > 100 and accepted > 50, (rejected, accepted)
    b.import_http_policy(img)
    assert np.array_equal(b.http_eval_host_diag(b.pack_http(**rq)), good)
    a.close()
    b.close()
