"""Parsed header lists → verdicts on the GPU: cg_http_verdicts_fields_{host,dev}
take cg_http_pack's input ("name\\0value\\0" pairs per request — the header map
AccessFilter::decodeHeaders sees, envoy/cilium_l7policy.cc:127-182) and group,
sort and pack it with the raw path's kernels (kernels_http_raw.hip, list mode)
instead of on the host.  Checked against the host path over the same lists
(cg_http_pack → http_kernel) and against the oracle (oracle.cc or_http_eval:
Envoy's HeaderMap::get and HeaderUtility::matchHeaders semantics)."""
import numpy as np
import pytest

import oracle
from cilium_amd import _native as N
from cilium_amd import synth
from cilium_amd.classifier import Classifier


def _split(blob, off):
    """Per request: the list's bytes."""
    b = bytes(np.asarray(blob, np.uint8)[:int(off[-1])]) if len(off) > 1 else b""
    return [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]


def _join(lists):
    off = np.zeros(len(lists) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in lists])
    return np.frombuffer(b"".join(lists) or b"\0", np.uint8).copy(), off


def _pairs(lst):
    parts = lst.split(b"\0")
    if parts and parts[-1] == b"" and lst.endswith(b"\0"):
        parts = parts[:-1]
    return [(parts[i], parts[i + 1] if i + 1 < len(parts) else b"") for i in range(0, len(parts), 2)]


def _vary(lists, rng, frac=0.3):
    """Lists as a proxy hands them over: name case, repeated names (the
    first value wins), unknown headers, long values (strings past the
    128-byte slot, lists past the kernel's LDS stage), control bytes in a
    value (malformed: denied), empty names and values, a last pair cut
    short (no terminator), empty lists."""
    out = []
    for lst in lists:
        if rng.random() >= frac:
            out.append(lst)
            continue
        ps = _pairs(lst)
        k = int(rng.integers(0, 9))
        if k == 0:
            ps = [(n.upper(), v) for n, v in ps]
        elif k == 1 and ps:
            j = int(rng.integers(0, len(ps)))
            ps = ps[:j + 1] + [(ps[j][0].swapcase(), b"second-" + ps[j][1])] + ps[j + 1:]
        elif k == 2:
            ps = [(b"x-unrelated-%d" % int(rng.integers(0, 9)), b"v" * int(rng.integers(0, 40)))] + ps
        elif k == 3 and ps:
            j = int(rng.integers(0, len(ps)))
            ps[j] = (ps[j][0], ps[j][1] + b"/" + b"p" * int(rng.integers(100, 300)))
        elif k == 4:
            ps = ps + [(b"x-big", b"b" * int(rng.integers(6000, 9000)))]  # past the 6 KiB stage
        elif k == 5 and ps:
            j = int(rng.integers(0, len(ps)))
            v = bytearray(ps[j][1] or b"x")
            v[int(rng.integers(0, len(v)))] = int(rng.choice([0x01, 0x0a, 0x0d, 0x7f, 0x09, 0x80, 0xff]))
            ps[j] = (ps[j][0], bytes(v))
        elif k == 6:
            ps = [(b"", b"empty-name")] + ps + [(b"x-empty", b"")]
        elif k == 7:
            out.append(b"".join(n + b"\0" + v + b"\0" for n, v in ps)[:-1 - int(rng.integers(0, 3))])
            continue
        else:
            out.append(b"")
            continue
        out.append(b"".join(n + b"\0" + v + b"\0" for n, v in ps))
    return out


def _args(rq):
    return rq["policy"], rq["ingress"], rq["port"], rq["remote"]


def _host_path(cl, policy, ingress, port, remote, blob, off):
    return cl.http_verdicts(cl.pack_http(policy, ingress, port, remote, blob, off))


def _oracle(pols, policy, ingress, port, remote, blob, off):
    return oracle.HttpOracle(pols).eval(np.asarray(policy, np.uint32), np.asarray(ingress, np.uint8),
                                        np.asarray(port, np.uint16), np.asarray(remote, np.uint32),
                                        np.asarray(blob, np.uint8), np.asarray(off, np.uint64), nthreads=8)


def _check(cl, pols, args, lists, n_oracle):
    blob, off = _join(lists)
    got = cl.http_verdicts_fields(*args, blob, off)
    assert np.array_equal(got, _host_path(cl, *args, blob, off))
    k = min(n_oracle, len(lists))
    sb, so = _join(lists[:k])
    exp = _oracle(pols, *(np.asarray(a)[:k] for a in args), sb, so)
    bad = np.nonzero(got[:k] != exp)[0]
    assert not len(bad), [(int(i), lists[i][:200], int(got[i]), int(exp[i])) for i in bad[:4]]
    return got


@pytest.mark.gpu
def test_gpu_fields_starwars(gpu):
    pols = synth.starwars_policy()
    gpu.update_http_policy(pols)
    rq = synth.starwars_requests(200_000, seed=31)
    lists = _vary(_split(rq["hdr_blob"], rq["hdr_off"]), np.random.default_rng(11))
    got = _check(gpu, pols, _args(rq), lists, 50_000)
    assert 0.1 < got.mean() < 0.9


@pytest.mark.gpu
def test_gpu_fields_10k_rules(gpu):
    pols, info = synth.http10k_rules()
    gpu.update_http_policy(pols)
    rq = synth.http10k_requests(300_000, info, seed=32)
    lists = _vary(_split(rq["hdr_blob"], rq["hdr_off"]), np.random.default_rng(12))
    got = _check(gpu, pols, _args(rq), lists, 30_000)
    assert 0.1 < got.mean() < 0.9


@pytest.mark.gpu
def test_gpu_fields_host_entry_many_chunks(gpu, monkeypatch):
    """The host entry's chunked staging (capi.cc verdicts_raw_from_host: two
    workers, each its own pinned buffers and stream) at 1 MiB chunks: ~25
    chunks of one call, every chunk boundary inside the batch, verdicts in
    request order equal to the host packer path's."""
    pols, info = synth.http10k_rules()
    gpu.update_http_policy(pols)
    rq = synth.http10k_requests(250_000, info, seed=34)
    lists = _vary(_split(rq["hdr_blob"], rq["hdr_off"]), np.random.default_rng(15), frac=0.1)
    blob, off = _join(lists)
    want = _host_path(gpu, *_args(rq), blob, off)
    monkeypatch.setenv("CILIUM_GPU_HOST_CHUNK_MB", "1")
    assert np.array_equal(gpu.http_verdicts_fields(*_args(rq), blob, off), want)
    monkeypatch.delenv("CILIUM_GPU_HOST_CHUNK_MB")
    assert np.array_equal(gpu.http_verdicts_fields(*_args(rq), blob, off), want)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_gpu_fields_all_matcher_forms(gpu, seed):
    from test_cpu_differential import all_matcher_case
    pols, rq, _ = all_matcher_case(seed, 4000)
    gpu.update_http_policy(pols)
    lists = _vary(_split(rq["hdr_blob"], rq["hdr_off"]), np.random.default_rng(20 + seed), frac=0.2)
    got = _check(gpu, pols, _args(rq), lists, len(lists))
    assert 0.05 < got.mean() < 0.95


@pytest.mark.gpu
def test_gpu_fields_edge_cases(gpu):
    """Hand-made lists: empty, a lone NUL, a pair cut short, names in any
    case, the first of repeated names, DEL / LF in an unrelated value (denied),
    HTAB and bytes >= 0x80 (fine), an empty name, a 20 KiB list (read outside
    the stage), a port without policy, an unknown policy index; a list past
    64 KiB fails the call."""
    pols = synth.starwars_policy()
    gpu.update_http_policy(pols)
    sw = gpu.http_policy_index(pols[0]["name"])
    ok = b":method\0POST\0:path\0/v1/request-landing/\0:authority\0deathstar\0"
    upper = b":METHOD\0POST\0:Path\0/v1/request-landing/\0:AUTHORITY\0deathstar\0"
    lists = [b"", b"\0", ok[:-1], ok, upper, ok + b":method\0GET\0", b":method\0GET\0" + ok,
             ok + b"x-a\0bad\x7fbyte\0", ok + b"x-a\0bad\nbyte\0", ok + b"x-a\0tab\there\0", ok + b"x-a\0\x80\xff\0",
             b"\0v\0" + ok, ok + b"x-big\0" + b"z" * 20_000 + b"\0", ok.replace(b"POST", b"PO\x01ST"), ok, ok]
    n = len(lists)
    pol = [sw] * (n - 2) + [sw, 0xFFFFFFFF]
    ing = [0] * n
    port = [80] * (n - 2) + [8080, 80]
    rem = [synth.SPACESHIP_ID] * n
    blob, off = _join(lists)
    got = gpu.http_verdicts_fields(pol, ing, port, rem, blob, off)
    assert np.array_equal(got, _oracle(pols, pol, ing, port, rem, blob, off))
    assert np.array_equal(got, _host_path(gpu, pol, ing, port, rem, blob, off))
    assert got.tolist() == [0, 0, 1, 1, 1, 1, 0, 0, 0, 1, 1, 1, 1, 0, 1, 0]
    assert len(gpu.http_verdicts_fields([], [], [], [], np.zeros(0, np.uint8), np.zeros(1, np.uint64))) == 0
    big, boff = _join([ok + b"x-huge\0" + b"h" * 70_000 + b"\0"])
    with pytest.raises(N.CiliumGPUError):
        gpu.http_verdicts_fields([sw], [0], [80], [synth.SPACESHIP_ID], big, boff)


@pytest.mark.gpu
def test_gpu_fields_proxylib_snapshot(gpu):
    """A proxylib snapshot: values arrive escaped (bytes 0x00-0x03 as 0x03,
    0x10 + b); a raw byte <= 0x02 or a bad escape pair is malformed.  Against
    the host packer on the same lists."""
    rules = [{"headers": [{"name": "cmd", "exact_match": "READ"}, {"name": "file", "regex_match": "/pub/.*"}]},
             {"headers": [{"name": "cmd", "exact_match": "WR\x01TE"}]}]
    pol = [{"name": "p", "proxylib": True, "policy": 0, "ingress_per_port_policies": [
        {"port": 80, "rules": [{"remote_policies": [1], "http_rules": {"http_rules": rules}}]}]}]
    gpu.update_http_policy(pol)
    rng = np.random.default_rng(13)
    vals = [b"READ", b"WRITE", b"WR\x03\x11TE", b"WR\x01TE", b"RE\x03AD", b"READ\x03", b"\x03\x14x", b"/pub/a",
            b"/pub/\x03\x10", b"/priv/x", b"\x02", b"\x03\x15"]
    lists = []
    for _ in range(20_000):
        ps = [(b"cmd", vals[int(rng.integers(0, len(vals)))])]
        if rng.random() < 0.7:
            ps.append((b"File" if rng.random() < 0.3 else b"file", vals[int(rng.integers(0, len(vals)))]))
        if rng.random() < 0.2:
            ps.reverse()
        lists.append(b"".join(n + b"\0" + v + b"\0" for n, v in ps))
    n = len(lists)
    args = (np.zeros(n, np.uint32), np.ones(n, np.uint8), np.full(n, 80, np.uint16),
            rng.integers(0, 3, n).astype(np.uint32))
    blob, off = _join(lists)
    got = gpu.http_verdicts_fields(*args, blob, off)
    assert np.array_equal(got, _host_path(gpu, *args, blob, off))
    assert 0.02 < got.mean() < 0.9


@pytest.mark.gpu
def test_gpu_fields_dev_tensors():
    """The device entry point on resident tensors (1M lists, 64 copies of a
    16K pool) against the host entry, and a second stream."""
    import torch
    cl = Classifier(device=0)
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    D, reps = 16_384, 64
    rq = synth.http10k_requests(D, info, seed=33)
    lists = _vary(_split(rq["hdr_blob"], rq["hdr_off"]), np.random.default_rng(14))
    blob, off = _join(lists)
    want = cl.http_verdicts_fields(*_args(rq), blob, off)
    dev = torch.device("cuda:0")
    tot = int(off[-1])
    d_blob = torch.from_numpy(blob[:tot]).to(dev).repeat(reps)
    base = torch.arange(reps, dtype=torch.int64, device=dev).unsqueeze(1) * tot
    d_off = torch.cat([(torch.from_numpy(off[:-1].astype(np.int64)).to(dev).unsqueeze(0) + base).reshape(-1),
                       torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    rep = lambda a, dt: torch.from_numpy(np.asarray(a).astype(dt)).to(dev).repeat(reps)
    args = (rep(rq["policy"], np.int32), rep(rq["ingress"], np.uint8), rep(rq["port"], np.int16),
            rep(rq["remote"], np.int32))
    d_out = torch.full((D * reps,), 7, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())  # the inputs were made on the current stream
    # enqueued on s, returns without waiting (the device-layout sequence)
    cl.http_verdicts_fields_dev(d_blob, d_off, D * reps, *args, d_out, stream=C_stream(s))
    s.synchronize()
    assert bool((d_out.view(reps, D) == torch.from_numpy(want).to(dev).unsqueeze(0)).all())
    cl.close()


def C_stream(s):
    import ctypes
    return ctypes.c_void_p(s.cuda_stream)


@pytest.mark.gpu
def test_gpu_fields_config5_full_size_oracle_subsample():
    """BASELINE config 5's per-GPU batch as header lists: 124.5M lists (1M
    distinct, laid out back to back), through the device entry point in one
    call; the first 1M verdicts equal the oracle's on those 1M distinct lists
    and every copy equals them (verdicts are per request)."""
    import torch
    cl = Classifier(device=0)
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    D, total = 1 << 20, 124_500_000
    rq = synth.http10k_requests_fast(D, info, seed=synth.SEED ^ 0xF1E1D)
    blob, off = rq["hdr_blob"], rq["hdr_off"]
    args = _args(rq)
    exp = _oracle(pols, *args, blob, off)
    reps = (total + D - 1) // D
    n = D * reps
    dev = torch.device("cuda:0")
    tot = int(off[-1])
    d_blob = torch.from_numpy(np.asarray(blob[:tot])).to(dev).repeat(reps)
    base = torch.arange(reps, dtype=torch.int64, device=dev).unsqueeze(1) * tot
    d_off = torch.cat([(torch.from_numpy(off[:-1].astype(np.int64)).to(dev).unsqueeze(0) + base).reshape(-1),
                       torch.tensor([tot * reps], dtype=torch.int64, device=dev)])
    rep = lambda a, dt: torch.from_numpy(np.asarray(a).astype(dt)).to(dev).repeat(reps)
    d_out = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    cl.http_verdicts_fields_dev(d_blob, d_off, n, rep(args[0], np.int32), rep(args[1], np.uint8),
                                rep(args[2], np.int16), rep(args[3], np.int32), d_out)
    got = d_out.view(reps, D)
    assert np.array_equal(got[0].cpu().numpy(), exp)
    assert bool((got == got[0].unsqueeze(0)).all())
    assert 0.1 < float(exp.mean()) < 0.9
    del d_blob, d_off, d_out
    cl.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [200, 6000])
def test_gpu_fields_host_many_fields_any_size(gpu, n):
    """A snapshot walking 40 header fields (past the device packer's 32):
    cg_http_verdicts_fields_host decides it at an Envoy-sized call and at a
    call past the small-call limit alike (host packing for both), equal to
    the host path and the oracle; the device entry refuses it."""
    names = ["x-f%02d" % i for i in range(40)]
    rules = [{"headers": [{"name": nm, "exact_match": "v%d" % i}]} for i, nm in enumerate(names)]
    pols = [{"name": "p", "policy": 0, "ingress_per_port_policies": [
        {"port": 80, "rules": [{"remote_policies": [], "http_rules": {"http_rules": rules}}]}]}]
    gpu.update_http_policy(pols)
    rng = np.random.default_rng(n)
    lists = []
    for _ in range(n):
        ps = [(b":method", b"GET"), (b":path", b"/x")]
        for _ in range(int(rng.integers(0, 3))):
            i = int(rng.integers(0, len(names)))
            ps.append((names[i].encode(), b"v%d" % (i if rng.random() < 0.6 else i + 1)))
        lists.append(b"".join(a + b"\0" + b + b"\0" for a, b in ps))
    args = (np.zeros(n, np.uint32), np.ones(n, np.uint8), np.full(n, 80, np.uint16), np.full(n, 5, np.uint32))
    got = _check(gpu, pols, args, lists, n)
    assert 0.2 < got.mean() < 0.9
    import torch
    blob, off = _join(lists)
    d = torch.device("cuda:0")
    with pytest.raises(N.CiliumGPUError):
        gpu.http_verdicts_fields_dev(torch.from_numpy(blob).to(d), torch.from_numpy(off.astype(np.int64)).to(d), n,
                                     torch.from_numpy(args[0].astype(np.int32)).to(d),
                                     torch.from_numpy(args[1]).to(d), torch.from_numpy(args[2].astype(np.int16)).to(d),
                                     torch.from_numpy(args[3].astype(np.int32)).to(d),
                                     torch.zeros(n, dtype=torch.uint8, device=d))
