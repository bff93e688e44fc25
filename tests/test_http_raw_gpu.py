"""Raw HTTP/1 request heads → verdicts on the GPU:
cg_http_verdicts_raw_{host,dev} parse the heads, pack them and evaluate them
on the device (kernels_http_raw.hip + http_kernel).  Checked against the
host path over the same heads (cg_http_parse_heads → cg_http_pack →
http_kernel) and against the oracle (oracle/http1_ref.py for the codec step,
then the Envoy-faithful rule scan).  The codec step is Envoy's http_parser
(external): parity for it is unpinned; the rule verdicts are pinned as in
test_gpu_configs."""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import synth
from cilium_amd.classifier import Classifier
from oracle.http1_ref import MAX_HEAD, parse_head
from test_http_parse import BAD_VALUE_HEAD, CASES, _blob, _line_end_mix, _raw_requests


def _vary(raws, rng, frac=0.3):
    """Heads as clients send them: header-name case, OWS, repeated Host,
    unknown headers, long values (strings past the 128-byte slot), bare-LF /
    CR LF mixes with the codec's other leniencies (test_http_parse
    _line_end_mix), and a few corrupted bytes (heads the codec rejects)."""
    out = []
    for r in raws:
        if rng.random() >= frac:
            out.append(r)
            continue
        head, _, _ = r.partition(b"\r\n\r\n")
        lines = head.split(b"\r\n")
        req, hdrs = lines[0], lines[1:]
        k = int(rng.integers(0, 8))
        if k == 0:
            hdrs = [h.split(b":", 1)[0].upper() + b":" + h.split(b":", 1)[1] for h in hdrs]
        elif k == 1:
            hdrs = [h.replace(b": ", b":\t  ", 1) + b" \t" for h in hdrs]
        elif k == 2:
            hdrs = hdrs + [b"hOsT: other.example.com"]
        elif k == 3:
            hdrs = [b"X-Unrelated-%d: %s" % (int(rng.integers(0, 9)), b"v" * int(rng.integers(0, 40)))] + hdrs
        elif k == 4:
            req = req.replace(b" HTTP/", b"/" + b"p" * int(rng.integers(60, 300)) + b" HTTP/", 1)
        new = b"\r\n".join([req] + hdrs) + b"\r\n\r\n"
        if k == 5:
            b = bytearray(new)
            b[int(rng.integers(0, len(b)))] = int(rng.choice([0x01, 0x0a, 0x20, 0x3a, 0x7f, 0x0d, 0x80, 0x2f]))
            new = bytes(b)
        elif k >= 6:
            new = _line_end_mix(new, rng)
        out.append(new)
    return out


def _oracle(pols, policy, ingress, port, remote, raws):
    """codec step (http1_ref) then the rule scan; rejected heads denied."""
    lists = [parse_head(r) for r in raws]
    blob, off = [], [0]
    for lst in lists:
        one = b"".join(k + b"\0" + v + b"\0" for k, v in (lst or []))
        blob.append(one)
        off.append(off[-1] + len(one))
    hb = np.frombuffer(b"".join(blob) or b"\0", np.uint8).copy()
    v = oracle.HttpOracle(pols).eval(np.asarray(policy, np.uint32), np.asarray(ingress, np.uint8),
                                     np.asarray(port, np.uint16), np.asarray(remote, np.uint32), hb,
                                     np.asarray(off, np.uint64), nthreads=8)
    return np.where([l is not None for l in lists], v, 0).astype(np.uint8)


def _host_path(cl, policy, ingress, port, remote, raws):
    return cl.http_verdicts(cl.pack_http_raw(policy, ingress, port, remote, *_blob(raws)))


def _check(cl, pols, rq, raws, n_oracle):
    args = (rq["policy"], rq["ingress"], rq["port"], rq["remote"])
    got = cl.http_verdicts_raw(*args, *_blob(raws))
    assert np.array_equal(got, _host_path(cl, *args, raws))
    k = min(n_oracle, len(raws))
    exp = _oracle(pols, *(np.asarray(a)[:k] for a in args), raws[:k])
    assert np.array_equal(got[:k], exp)
    return got


@pytest.mark.gpu
def test_gpu_raw_starwars(gpu):
    pols = synth.starwars_policy()
    gpu.update_http_policy(pols)
    rq = synth.starwars_requests(200_000, seed=21)
    raws = _vary(_raw_requests(rq), np.random.default_rng(1))
    got = _check(gpu, pols, rq, raws, 50_000)
    assert 0.1 < got.mean() < 0.9


@pytest.mark.gpu
def test_gpu_raw_10k_rules(gpu):
    pols, info = synth.http10k_rules()
    gpu.update_http_policy(pols)
    rq = synth.http10k_requests(300_000, info, seed=22)
    raws = _vary(_raw_requests(rq), np.random.default_rng(2))
    got = _check(gpu, pols, rq, raws, 30_000)
    assert 0.1 < got.mean() < 0.9


@pytest.mark.gpu
def test_gpu_raw_reference_cases_and_limits(gpu):
    """The codec cases (rejected heads denied), an allow-all port (no HTTP
    rules) where a rejected head is still denied, a port without policy
    (allowed), an unknown policy index (denied), heads past 60 KiB."""
    pols = synth.starwars_policy() + [{"name": "open", "policy": 9, "ingress_per_port_policies": [
        {"port": 80, "rules": [{"remote_policies": [7]}]}]}]
    gpu.update_http_policy(pols)
    sw, op = gpu.http_policy_index(pols[0]["name"]), gpu.http_policy_index("open")
    ok_head = b"GET /v1/ HTTP/1.1\r\nHost: deathstar\r\n\r\n"
    big = b"GET /v1/ HTTP/1.1\r\nHost: deathstar\r\nX-Pad: " + b"a" * MAX_HEAD + b"\r\n\r\n"
    raws = [r for r, _ in CASES] + [ok_head, BAD_VALUE_HEAD, ok_head, ok_head, big]
    n = len(raws)
    pol = [sw] * len(CASES) + [op, op, sw, 0xFFFFFFFF, sw]
    ing = [0] * len(CASES) + [1, 1, 1, 0, 0]
    port = [80] * len(CASES) + [80, 80, 8080, 80, 80]
    rem = [synth.SPACESHIP_ID] * len(CASES) + [7, 7, 1, synth.SPACESHIP_ID, synth.SPACESHIP_ID]
    got = gpu.http_verdicts_raw(pol, ing, port, rem, *_blob(raws))
    exp = _oracle(pols, pol, ing, port, rem, raws)
    assert got.tolist() == exp.tolist()
    assert got.tolist()[len(CASES):] == [1, 0, 1, 0, 0]
    assert np.array_equal(got, _host_path(gpu, pol, ing, port, rem, raws))
    # no requests
    assert len(gpu.http_verdicts_raw([], [], [], [], np.zeros(0, np.uint8), np.zeros(1, np.uint64))) == 0


@pytest.mark.gpu
def test_gpu_raw_dev_tensors():
    """The device entry point on resident tensors (1M requests, 64 copies of
    a 16K-request pool laid out back to back) against the host entry."""
    import torch
    cl = Classifier(device=0)
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    D, reps = 16_384, 64
    rq = synth.http10k_requests(D, info, seed=23)
    raws = _vary(_raw_requests(rq), np.random.default_rng(3))
    blob, off = _blob(raws)
    want = cl.http_verdicts_raw(rq["policy"], rq["ingress"], rq["port"], rq["remote"], blob, off)
    dev = torch.device("cuda:0")
    tot = int(off[-1])
    d_raw = torch.from_numpy(np.tile(blob[:tot], reps)).to(dev)
    base = torch.arange(reps, dtype=torch.int64).unsqueeze(1) * tot
    d_off = torch.cat([(torch.from_numpy(off[:-1].astype(np.int64)).unsqueeze(0) + base).reshape(-1),
                       torch.tensor([tot * reps])]).to(dev)
    rep = lambda a, dt: torch.from_numpy(np.tile(np.asarray(a).astype(dt), reps)).to(dev)
    d_pol, d_ing = rep(rq["policy"], np.int32), rep(rq["ingress"], np.uint8)
    d_port, d_rem = rep(rq["port"], np.int16), rep(rq["remote"], np.int32)
    d_out = torch.zeros(D * reps, dtype=torch.uint8, device=dev)
    cl.http_verdicts_raw_dev(d_raw, d_off, D * reps, d_pol, d_ing, d_port, d_rem, d_out)
    got = d_out.cpu().numpy().reshape(reps, D)
    assert all(np.array_equal(g, want) for g in got)
    cl.close()


@pytest.mark.gpu
def test_gpu_raw_proxylib_snapshot_unsupported():
    from test_proxylib_abi import open_module, _lib
    import json
    inst = open_module([(b"node-id", b"gpu-raw-unsup")], "0")
    t = json.dumps([{"name": "p", "ingress_per_port_policies": [{"port": 80, "rules": [
        {"l7_proto": "r2d2", "l7_rules": {"l7_rules": [{"rule": {"cmd": "READ"}}]}}]}]}]).encode()
    assert N.lib.cg_proxylib_policy_update(inst, t, len(t)) == N.CG_OK
    _lib.CloseModule(inst)
    cl = Classifier(device=0)
    cl.update_http_policy([{"name": "p", "proxylib": True, "ingress_per_port_policies": [{"port": 80, "rules": [
        {"http_rules": {"http_rules": [{"headers": [{"name": "cmd", "exact_match": "READ"}]}]}}]}]}])
    with pytest.raises(N.CiliumGPUError):
        cl.http_verdicts_raw([0], [1], [80], [1], *_blob([b"GET / HTTP/1.1\r\n\r\n"]))
    cl.close()


def test_head_size_limit_host_parser():
    """Heads over Envoy's default 60 KiB header limit are rejected by the
    host codec step and the oracle alike."""
    ok = b"GET / HTTP/1.1\r\nHost: a\r\nX: " + b"a" * (MAX_HEAD - 50) + b"\r\n\r\n"
    big = b"GET / HTTP/1.1\r\nHost: a\r\nX: " + b"a" * MAX_HEAD + b"\r\n\r\n"
    _, _, good = Classifier.parse_http_heads(*_blob([ok, big]))
    assert good.tolist() == [1, 0]
    assert parse_head(ok) is not None and parse_head(big) is None


@pytest.mark.gpu
def test_gpu_raw_config5_full_size():
    """BASELINE config 5's per-GPU batch as raw heads: 1,048,576 distinct
    requests of the 10K-rule set (with client-style variations) laid out
    119 times back to back — 124.8M heads, 8.7 GB resident — through the
    device entry point in one call; every copy's verdicts equal the host
    path's verdicts for the distinct requests (size-independent property:
    verdicts are per request, whatever the batch around it), and those equal
    the oracle's for all 1,048,576 distinct heads."""
    import torch
    cl = Classifier(device=0)
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    D, reps = 1 << 20, 119
    rq = synth.http10k_requests(D, info, seed=synth.SEED ^ 0x4A1)
    raws = _vary(_raw_requests(rq), np.random.default_rng(4), frac=0.02)  # long strings stay within the 256 MiB arena
    blob, off = _blob(raws)
    args = (rq["policy"], rq["ingress"], rq["port"], rq["remote"])
    want = _host_path(cl, *args, raws)
    # every distinct head against the oracle (codec step + Envoy rule scan),
    # so each of the 124.8M device verdicts below is oracle-checked
    assert np.array_equal(want, _oracle(pols, *args, raws))
    dev = torch.device("cuda:0")
    tot = int(off[-1])
    d_raw = torch.from_numpy(blob[:tot]).to(dev).repeat(reps)
    base = torch.arange(reps, dtype=torch.int64, device=dev).unsqueeze(1) * tot
    d_off = torch.cat([(torch.from_numpy(off[:-1].astype(np.int64)).to(dev).unsqueeze(0) + base).reshape(-1),
                       torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    rep = lambda a, dt: torch.from_numpy(np.asarray(a).astype(dt)).to(dev).repeat(reps)
    d_pol, d_ing = rep(args[0], np.int32), rep(args[1], np.uint8)
    d_port, d_rem = rep(args[2], np.int16), rep(args[3], np.int32)
    n = D * reps
    d_out = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    cl.http_verdicts_raw_dev(d_raw, d_off, n, d_pol, d_ing, d_port, d_rem, d_out)
    got = d_out.view(reps, D)
    assert bool((got == torch.from_numpy(want).to(dev).unsqueeze(0)).all())
    assert 0.1 < float(want.mean()) < 0.9
    del d_raw, d_off, d_out
    cl.close()


@pytest.mark.gpu
def test_gpu_raw_arena_split():
    """A batch whose long strings need more than the 256 MiB overflow arena
    (1M heads with 300-400-byte paths, ~350 MB of arena) is evaluated in
    halves: verdicts equal the host path's for every copy."""
    import torch
    cl = Classifier(device=0)
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    D, reps = 16_384, 64
    rq = synth.http10k_requests(D, info, seed=24)
    rng = np.random.default_rng(5)
    raws = [r.replace(b" HTTP/", b"/" + b"q" * int(rng.integers(300, 400)) + b" HTTP/", 1) for r in _raw_requests(rq)]
    blob, off = _blob(raws)
    args = (rq["policy"], rq["ingress"], rq["port"], rq["remote"])
    want = _host_path(cl, *args, raws)
    # every distinct head against the oracle (codec step + Envoy rule scan),
    # so each of the 124.8M device verdicts below is oracle-checked
    assert np.array_equal(want, _oracle(pols, *args, raws))
    dev = torch.device("cuda:0")
    tot = int(off[-1])
    d_raw = torch.from_numpy(blob[:tot]).to(dev).repeat(reps)
    base = torch.arange(reps, dtype=torch.int64, device=dev).unsqueeze(1) * tot
    d_off = torch.cat([(torch.from_numpy(off[:-1].astype(np.int64)).to(dev).unsqueeze(0) + base).reshape(-1),
                       torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    rep = lambda a, dt: torch.from_numpy(np.asarray(a).astype(dt)).to(dev).repeat(reps)
    n = D * reps
    d_out = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    cl.http_verdicts_raw_dev(d_raw, d_off, n, rep(args[0], np.int32), rep(args[1], np.uint8), rep(args[2], np.int16),
                             rep(args[3], np.int32), d_out)
    assert bool((d_out.view(reps, D) == torch.from_numpy(want).to(dev).unsqueeze(0)).all())
    cl.close()


@pytest.mark.gpu
def test_gpu_raw_header_name_keys(gpu):
    """Header names of lengths 1..64 referenced by rules, sent in mixed
    case, among names that share length, first 8 and last 8 bytes with a rule
    name (the structural parser's name key: the middle is verified) — on the
    device against the host path and the oracle."""
    import random
    rng = random.Random(7)
    lengths = list(range(1, 21)) + [23, 26, 29, 32, 35, 38, 40, 47, 64]  # 29 + 3 below: the 32-field limit
    names = ["".join(rng.choice("abcdefghijklmnopqrstuvwxyz-0123456789") for _ in range(L)) for L in lengths]
    names += ["x-aaaaaaaa-1-bbbbbbbb", "x-aaaaaaaa-2-bbbbbbbb", "x-long-header-name-for-key-tests"]
    rules = [{"headers": [{"name": nm, "exact_match": "v%d" % i}]} for i, nm in enumerate(names)]
    pols = [{"name": "p", "policy": 0, "ingress_per_port_policies": [
        {"port": 80, "rules": [{"remote_policies": [], "http_rules": {"http_rules": rules}}]}]}]
    gpu.update_http_policy(pols)
    decoys = ["x-aaaaaaaa-3-bbbbbbbb", "x-aaaaaaaa-1-bbbbbbbc", "y-aaaaaaaa-1-bbbbbbbb"]
    raws = []
    for _ in range(6000):
        hs = []
        for _ in range(rng.randint(0, 4)):
            nm = rng.choice(names + decoys)
            nm = "".join(c.upper() if rng.random() < 0.5 else c for c in nm)
            i = names.index(nm.lower()) if nm.lower() in names else 0
            val = "v%d" % (i if rng.random() < 0.7 else rng.randint(0, len(names)))
            hs.append(b"%s:%s%s" % (nm.encode(), rng.choice([b"", b" ", b"\t "]), val.encode()))
        raws.append(b"GET /x HTTP/1.1\r\nHost: a\r\n" + b"".join(h + b"\r\n" for h in hs) + b"\r\n")
    n = len(raws)
    pol, ing, port, rem = [0] * n, [1] * n, [80] * n, [5] * n
    got = gpu.http_verdicts_raw(pol, ing, port, rem, *_blob(raws))
    assert np.array_equal(got, _host_path(gpu, pol, ing, port, rem, raws))
    assert np.array_equal(got, _oracle(pols, pol, ing, port, rem, raws))
    assert 0.2 < got.mean() < 0.9
