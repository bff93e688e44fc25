"""NPDS protobuf ingestion:
cg_http_policy_update_npds / cg_proxylib_policy_update_npds take the wire form
Envoy's and proxylib's NPDS clients receive — a serialized DiscoveryResponse of
Any-wrapped cilium.NetworkPolicy (envoy/cilium/npds.proto:31-182).  Policies
installed from protobuf must compile to the same tables as the same policies
installed from JSON (checked by walking both on the host), reject what
npds.pb.validate.go rejects, and give the reference fixtures' verdicts on the
GPU."""
import json

import numpy as np
import pytest

import npds_pb as PB
from cilium_amd import _native as N
from cilium_amd import synth
from cilium_amd.classifier import Classifier
from kat_util import http_requests, load

HTTP = load("http_kat.json")


def _same_tables(pols, rq):
    a, b = Classifier(device=-1), Classifier(device=-1)
    try:
        a.update_http_policy(pols)
        b.update_http_policy_npds(PB.discovery_response(pols))
        va = a.http_eval_host_diag(a.pack_http(**rq))
        vb = b.http_eval_host_diag(b.pack_http(**rq))
        assert np.array_equal(va, vb)
        return va
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("suite", HTTP["suites"], ids=lambda s: s["name"])
def test_pb_http_kat_host(suite):
    names = [p["name"] for p in suite["policy"]]
    rq = http_requests(suite["requests"], lambda n: names.index(n) if n in names else 0xFFFFFFFF)
    got = _same_tables(suite["policy"], rq)
    exp = np.array([r["expect"] for r in suite["requests"]], np.uint8)
    assert np.array_equal(got, exp)


def test_pb_http10k_subset_host():
    pols, info = synth.http10k_rules(n_rules=600)
    rq = synth.http10k_requests(20_000, info)
    v = _same_tables(pols, rq)
    assert 0 < v.mean() < 1


def test_pb_packed_and_unpacked_remotes():
    pols = synth.starwars_policy()
    rq = synth.starwars_requests(2000)
    a, b = Classifier(device=-1), Classifier(device=-1)
    a.update_http_policy_npds(PB.discovery_response(pols, packed=True))
    b.update_http_policy_npds(PB.discovery_response(pols, packed=False))
    assert np.array_equal(a.http_eval_host_diag(a.pack_http(**rq)), b.http_eval_host_diag(b.pack_http(**rq)))
    a.close()
    b.close()


def _rc(cl, blob):
    return N.lib.cg_http_policy_update_npds(cl.h, blob, len(blob))


def test_pb_validation_rejects():
    cl = Classifier(device=-1)
    ok = [{"name": "p", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"remote_policies": [1, 2], "http_rules": {"http_rules": [{"headers": [
            {"name": ":path", "regex_match": "/a.*"}]}]}}]}]}]
    assert _rc(cl, PB.discovery_response(ok)) == N.CG_OK
    bad_port = json.loads(json.dumps(ok))
    bad_port[0]["ingress_per_port_policies"][0]["port"] = 65536
    dup_remote = json.loads(json.dumps(ok))
    dup_remote[0]["ingress_per_port_policies"][0]["rules"][0]["remote_policies"] = [3, 3]
    empty_http = json.loads(json.dumps(ok))
    empty_http[0]["ingress_per_port_policies"][0]["rules"][0]["http_rules"]["http_rules"] = []
    for bad in (PB.discovery_response(bad_port), PB.discovery_response(dup_remote), PB.discovery_response(empty_http),
                PB.discovery_response(ok, type_url="type.googleapis.com/cilium.Other"),
                PB.discovery_response(ok)[:-9],  # truncated inside a field
                b"\x12\xff\xff\xff\xff\x0f"):  # a length past the message
        assert _rc(cl, bad) == N.CG_POLICY_REJECTED, bad
    # the previous snapshot still serves
    assert cl.http_policy_index("p") == 0
    # an empty response installs no policies
    assert _rc(cl, b"") == N.CG_OK
    cl.close()


def test_pb_unknown_fields_skipped():
    pols = synth.starwars_policy()
    blob = PB.discovery_response(pols)
    # unknown fields of every wire type in the DiscoveryResponse
    extra = PB.vi(9, 7) + PB.key(10, 1) + b"\x00" * 8 + PB.ld(11, b"xyz") + PB.key(12, 5) + b"\x00" * 4
    cl = Classifier(device=-1)
    assert _rc(cl, extra + blob + extra) == N.CG_OK
    cl.close()


def test_pb_proxylib_translation_codes():
    from test_proxylib_abi import _lib, open_module
    inst = open_module([(b"node-id", b"cpu-npds-pb")], "-1")

    def upd(pols):
        blob = PB.discovery_response(pols)
        return N.lib.cg_proxylib_policy_update_npds(inst, blob, len(blob))

    def l7(parser, *rs):
        return {"l7_proto": parser, "l7_rules": {"l7_rules": [{"rule": r} for r in rs]}}

    def pol(rules):
        return [{"name": "p", "ingress_per_port_policies": [{"port": 80, "rules": rules}]}]

    assert upd(pol([l7("r2d2", {"cmd": "READ", "file": "^/a"})])) == N.CG_OK
    assert upd(pol([l7("cassandra", {"query_action": "select", "query_table": "t$"})])) == N.CG_OK
    assert upd(pol([l7("cassandra", {"query_action": "explode"})])) == N.CG_POLICY_REJECTED
    assert upd(pol([l7("r2d2", {"cmd": "JUMP"})])) == N.CG_POLICY_REJECTED
    assert upd(pol([{"l7_proto": "r2d2", "l7_rules": {"l7_rules": []}}])) == N.CG_POLICY_REJECTED  # min_items
    _lib.CloseModule(inst)


@pytest.mark.parametrize("seed", range(3))
def test_pb_all_matcher_forms(seed):
    """prefix / suffix / range (negative int64 varints) / invert_match from
    the wire compile to the same tables as their JSON form."""
    import random

    from test_cpu_differential import HDR_NAMES, NUM_VALUES, VALUES, _rand_matcher_ext
    rng = random.Random(seed)
    pols = [{"name": f"p{i}", "policy": i, "ingress_per_port_policies": [{"port": 80, "rules": [
        {"remote_policies": [], "http_rules": {"http_rules": [
            {"headers": [_rand_matcher_ext(rng) for _ in range(rng.randint(1, 3))]} for _ in range(3)]}}]}]}
            for i in range(2)]
    n = 800
    parts, off = [], [0]
    for _ in range(n):
        b = b"".join(nm.encode() + b"\0" + rng.choice(VALUES + NUM_VALUES).encode() + b"\0"
                     for nm in HDR_NAMES if rng.random() < 0.8)
        parts.append(b)
        off.append(off[-1] + len(b))
    rq = dict(policy=np.array([rng.randint(0, 1) for _ in range(n)], np.uint32), ingress=np.ones(n, np.uint8),
              port=np.full(n, 80, np.uint16), remote=np.zeros(n, np.uint32),
              hdr_blob=np.frombuffer(b"".join(parts), np.uint8).copy(), hdr_off=np.array(off, np.uint64))
    v = _same_tables(pols, rq)
    assert 0 < v.sum() < n


def test_pb_singular_messages_merge():
    """Occurrences of a singular embedded message merge (proto3): the
    http_rules oneof member split in two appends its rule lists, a BoolValue
    split in two keeps the set flag, and a later oneof member replaces the
    earlier one."""
    r1 = {"headers": [{"name": ":path", "regex_match": "/a.*"}]}
    r2 = {"headers": [{"name": ":method", "exact_match": "GET"}]}

    def rules_payload(*rs):
        return b"".join(PB.ld(1, b"".join(PB.ld(1, PB.header_matcher(h)) for h in r["headers"])) for r in rs)

    def pol_blob(port_rule_bytes):
        pp = PB.vi(1, 80) + PB.ld(3, port_rule_bytes)
        np_ = PB.s(1, "p") + PB.vi(2, 0) + PB.ld(3, pp)
        return PB.s(1, "1") + PB.ld(2, PB.s(1, PB.TYPE_URL) + PB.ld(2, np_))

    split = pol_blob(PB.ld(100, rules_payload(r1)) + PB.ld(100, rules_payload(r2)))
    whole = [{"name": "p", "policy": 0, "ingress_per_port_policies": [{"port": 80, "rules": [
        {"remote_policies": [], "http_rules": {"http_rules": [r1, r2]}}]}]}]
    # a kafka member first, then http: the last member (http) wins
    replaced = pol_blob(PB.ld(101, PB.ld(1, PB.vi(1, 0))) + PB.ld(100, rules_payload(r1, r2)))
    # deprecated {value, regex} with the BoolValue split: {value: true} then {}
    hm = PB.s(1, ":path") + PB.s(2, "/a.*") + PB.ld(3, PB.vi(1, 1)) + PB.ld(3, b"")
    boolsplit = pol_blob(PB.ld(100, PB.ld(1, PB.ld(1, hm))))
    boolwhole = [{"name": "p", "policy": 0, "ingress_per_port_policies": [{"port": 80, "rules": [
        {"remote_policies": [], "http_rules": {"http_rules": [{"headers": [
            {"name": ":path", "regex_match": "/a.*"}]}]}}]}]}]
    reqs = [[(":path", "/abc"), (":method", "PUT")], [(":path", "/x"), (":method", "GET")],
            [(":path", "/x"), (":method", "PUT")], [(":path", "/a"), (":method", "GET")]]
    parts, off = [], [0]
    for hs in reqs:
        b = b"".join(k.encode() + b"\0" + v.encode() + b"\0" for k, v in hs)
        parts.append(b)
        off.append(off[-1] + len(b))
    n = len(reqs)
    rq = dict(policy=np.zeros(n, np.uint32), ingress=np.ones(n, np.uint8), port=np.full(n, 80, np.uint16),
              remote=np.zeros(n, np.uint32), hdr_blob=np.frombuffer(b"".join(parts), np.uint8).copy(),
              hdr_off=np.array(off, np.uint64))

    def walk_pb(blob):
        cl = Classifier(device=-1)
        cl.update_http_policy_npds(blob)
        v = cl.http_eval_host_diag(cl.pack_http(**rq))
        cl.close()
        return v.tolist()

    def walk_json(pols):
        cl = Classifier(device=-1)
        cl.update_http_policy(pols)
        v = cl.http_eval_host_diag(cl.pack_http(**rq))
        cl.close()
        return v.tolist()

    assert walk_pb(split) == walk_json(whole) == [1, 1, 0, 1]
    assert walk_pb(replaced) == [1, 1, 0, 1]
    assert walk_pb(boolsplit) == walk_json(boolwhole) == [1, 0, 0, 1]


def test_pb_utf8_rule():
    """A proto3 string field that is not UTF-8: Envoy's protobuf runtime
    rejects the response (HTTP update), golang/protobuf of the reference era
    accepts it (proxylib update)."""
    bad = {"name": "p", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"remote_policies": [], "http_rules": {"http_rules": [{"headers": [
            {"name": "x-a", "exact_match": b"\xff\xfe".decode("latin-1")}]}]}}]}]}
    good = json.loads(json.dumps(bad))
    good["ingress_per_port_policies"][0]["rules"][0]["http_rules"]["http_rules"][0]["headers"][0]["exact_match"] = \
        "\u00e9t\u00e9".encode("utf-8").decode("latin-1")
    cl = Classifier(device=-1)
    assert _rc(cl, PB.discovery_response([bad])) == N.CG_POLICY_REJECTED
    assert _rc(cl, PB.discovery_response([good])) == N.CG_OK
    cl.close()
    from test_proxylib_abi import _lib, open_module
    inst = open_module([(b"node-id", b"cpu-npds-utf8")], "-1")
    # a memcache keyExact is []byte(v): the non-UTF-8 string installs
    # (memcached/parser.go:125-130) ...
    pl = [{"name": "p", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "memcache", "l7_rules": {"l7_rules": [{"rule": {"command": "get", "keyExact": "\xff"}}]}}]}]}]
    blob = PB.discovery_response(pl)
    assert N.lib.cg_proxylib_policy_update_npds(inst, blob, len(blob)) == N.CG_OK
    # ... while an r2d2 file regex goes through regexp.MustCompile, which
    # refuses invalid UTF-8: the rule parser panics and the update fails
    # (r2d2parser.go:103, instance.go:169-176)
    pl[0]["ingress_per_port_policies"][0]["rules"][0] = {
        "l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"cmd": "READ", "file": "\xff"}}]}}
    blob = PB.discovery_response(pl)
    assert N.lib.cg_proxylib_policy_update_npds(inst, blob, len(blob)) == N.CG_POLICY_REJECTED
    _lib.CloseModule(inst)


@pytest.mark.gpu
@pytest.mark.parametrize("suite", HTTP["suites"], ids=lambda s: s["name"])
def test_gpu_pb_http_kat(suite):
    cl = Classifier(device=0)
    names = [p["name"] for p in suite["policy"]]
    rq = http_requests(suite["requests"], lambda n: names.index(n) if n in names else 0xFFFFFFFF)
    cl.update_http_policy_npds(PB.discovery_response(suite["policy"]))
    got = cl.http_verdicts(cl.pack_http(**rq))
    exp = np.array([r["expect"] for r in suite["requests"]], np.uint8)
    assert np.array_equal(got, exp)
    cl.close()


@pytest.mark.gpu
def test_gpu_pb_proxylib_reference_policies():
    """The reference's r2d2 test policies (tests/golden/proxylib_kat.json, as
    protobuf text) installed from their binary form; frames through OnData."""
    from cilium_amd import proxylib as P
    from test_proxylib_abi import DROP, F_OK, MORE, PASS, Conn, _lib, open_module
    kat = load("proxylib_kat.json")
    inst = open_module([(b"node-id", b"gpu-npds-pb")], "0")
    pols = [P.parse_policy_text(c["policy"]) for c in kat["r2d2"]]
    blob = PB.discovery_response(pols)
    assert N.lib.cg_proxylib_policy_update_npds(inst, blob, len(blob)) == N.CG_OK
    for case, pol in zip(kat["r2d2"], pols):
        c = Conn(inst, src=kat["remote"], dst_addr=b"2.2.2.2:%d" % kat["port"], policy=pol["name"].encode())
        for line, allow in case["requests"]:
            rc, ops = c.on_data([line.encode() + b"\r\n"])
            assert rc == F_OK and ops == [(PASS if allow else DROP, len(line) + 2), (MORE, 1)], (case["src"], line)
        c.close()
    _lib.CloseModule(inst)
