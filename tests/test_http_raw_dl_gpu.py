"""The raw path's device-layout sequence (the default since round 5;
CILIUM_GPU_RAW_LAYOUT=host selects the round-3 sequence; http_raw.cc
raw_device_layout): the scan takes each request's slot from a
per-bucket counter and writes its class-coded string straight into the
tile-transposed batch, raw_seal_kernel pads the last tiles and writes the
chunk table, http_kernel decides, raw_walk_kernel decides the strings past
the 128-byte slot — all on the caller's stream with no host round trip.

Checked, as the default path is (test_http_raw_gpu.py, test_http_fields_gpu.py),
against the host path over the same requests (cg_http_pack → http_kernel) and
the oracle (oracle/http1_ref.py codec step, then the Envoy-faithful rule
scan), plus its per-program and per-rule counters against the default
path's.  Batches stay small (a few 10K requests): a broken slot protocol
would show as bounded polling (RawLayoutDev.spin), not a hang."""
import os

import numpy as np
import pytest

from cilium_amd import _native as N
from cilium_amd import synth
from cilium_amd.classifier import Classifier
from test_http_fields_gpu import _host_path as _fields_host_path
from test_http_fields_gpu import _join, _split
from test_http_fields_gpu import _oracle as _fields_oracle
from test_http_fields_gpu import _vary as _fields_vary
from test_http_parse import _blob, _raw_requests
from test_http_raw_gpu import _host_path, _oracle, _vary

pytestmark = [pytest.mark.gpu, pytest.mark.run_last]


@pytest.fixture
def dl():
    """The device-layout path for the test's calls (read per call)."""
    old = {k: os.environ.get(k) for k in ("CILIUM_GPU_RAW_LAYOUT", "CILIUM_GPU_RAW_SUBBATCH", "CILIUM_GPU_RAW_SPIN")}
    os.environ["CILIUM_GPU_RAW_LAYOUT"] = "device"
    yield os.environ
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _args(rq):
    return rq["policy"], rq["ingress"], rq["port"], rq["remote"]


def _check_heads(cl, pols, rq, raws, n_oracle):
    args = _args(rq)
    got = cl.http_verdicts_raw(*args, *_blob(raws))
    assert np.array_equal(got, _host_path(cl, *args, raws))
    k = min(n_oracle, len(raws))
    assert np.array_equal(got[:k], _oracle(pols, *(np.asarray(a)[:k] for a in args), raws[:k]))
    return got


def test_gpu_dl_starwars(gpu, dl):
    pols = synth.starwars_policy()
    gpu.update_http_policy(pols)
    rq = synth.starwars_requests(20_000, seed=121)
    got = _check_heads(gpu, pols, rq, _vary(_raw_requests(rq), np.random.default_rng(121)), 20_000)
    assert 0.1 < got.mean() < 0.9


def test_gpu_dl_10k_rules_subbatches(gpu, dl):
    """The 10K-rule set, 30K varied heads in sub-batches of 4096 (each with
    its own chunk directory tag, partly filled last chunks, padding)."""
    dl["CILIUM_GPU_RAW_SUBBATCH"] = "4096"
    pols, info = synth.http10k_rules()
    gpu.update_http_policy(pols)
    rq = synth.http10k_requests(30_000, info, seed=122)
    got = _check_heads(gpu, pols, rq, _vary(_raw_requests(rq), np.random.default_rng(122)), 10_000)
    assert 0.1 < got.mean() < 0.9


def test_gpu_dl_long_strings_and_big_heads(gpu, dl):
    """Walked strings past the slot (raw_walk_kernel) and heads past the
    wave's LDS stage (raw_defer_dl_kernel, then slotted or walked)."""
    pols, info = synth.http10k_rules()
    gpu.update_http_policy(pols)
    rq = synth.http10k_requests(6_000, info, seed=123)
    rng = np.random.default_rng(123)
    raws = []
    for r in _raw_requests(rq):
        k = int(rng.integers(0, 4))
        if k == 1:
            r = r.replace(b" HTTP/", b"/" + b"q" * int(rng.integers(130, 400)) + b" HTTP/", 1)
        elif k == 2:
            r = r.replace(b"\r\n\r\n", b"\r\nX-Big: " + b"b" * int(rng.integers(6000, 9000)) + b"\r\n\r\n", 1)
        raws.append(r)
    _check_heads(gpu, pols, rq, raws, len(raws))


def test_gpu_dl_header_lists(gpu, dl):
    """cg_http_verdicts_fields_* (header lists): name case, repeated names,
    long values, lists past the stage, control bytes, cut pairs, empty lists."""
    pols, info = synth.http10k_rules()
    gpu.update_http_policy(pols)
    rq = synth.http10k_requests(20_000, info, seed=124)
    lists = _fields_vary(_split(rq["hdr_blob"], rq["hdr_off"]), np.random.default_rng(124))
    blob, off = _join(lists)
    got = gpu.http_verdicts_fields(*_args(rq), blob, off)
    assert np.array_equal(got, _fields_host_path(gpu, *_args(rq), blob, off))
    k = 8_000
    sb, so = _join(lists[:k])
    assert np.array_equal(got[:k], _fields_oracle(pols, *(np.asarray(a)[:k] for a in _args(rq)), sb, so))


def test_gpu_dl_counters_match_default_path(gpu, dl):
    """Per-program allowed/denied and per-rule hit counters after a batch
    through the device layout equal the default path's for the same batch
    (slotted requests counted by http_kernel, walked ones by raw_walk_kernel)."""
    pols, info = synth.http10k_rules()
    gpu.update_http_policy(pols)
    rq = synth.http10k_requests(20_000, info, seed=125)
    rng = np.random.default_rng(125)
    raws = [r.replace(b" HTTP/", b"/" + b"z" * 200 + b" HTTP/", 1) if rng.random() < 0.1 else r
            for r in _vary(_raw_requests(rq), rng)]
    blob, off = _blob(raws)

    def run():
        gpu.reset_counters()
        v = gpu.http_verdicts_raw(*_args(rq), blob, off)
        return v, gpu.read_counters(N.CG_CTR_HTTP_PROGRAMS), gpu.read_counters(N.CG_CTR_HTTP_RULES)

    v_dl, p_dl, r_dl = run()
    dl["CILIUM_GPU_RAW_LAYOUT"] = "host"  # the round-3 sequence
    v_def, p_def, r_def = run()
    assert np.array_equal(v_dl, v_def)
    assert np.array_equal(p_dl, p_def)
    assert np.array_equal(r_dl, r_def)


def test_gpu_dl_batches_queued_on_streams(dl):
    """Stream order: three different batches queued on device tensors with
    no host synchronization between them — two back to back on one stream
    (the second reuses the workspace while the first may still run), the
    third on another stream (it waits for the second on the device) — each
    batch's verdicts equal the oracle's."""
    import torch
    cl = Classifier(device=0)
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    dev = torch.device("cuda:0")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(np.asarray(a).astype(dt))).to(dev)
    batches = []
    for k, n in enumerate((24_000, 16_000, 8_000)):
        rq = synth.http10k_requests(n, info, seed=130 + k)
        raws = _vary(_raw_requests(rq), np.random.default_rng(130 + k))
        blob, off = _blob(raws)
        d = (t(blob, np.uint8), t(off, np.int64), n, t(rq["policy"], np.int32), t(rq["ingress"], np.uint8),
             t(rq["port"], np.int16), t(rq["remote"], np.int32))
        batches.append((rq, raws, d))
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    outs = [torch.full((len(r),), 7, dtype=torch.uint8, device=dev) for _, r, _ in batches]
    torch.cuda.synchronize()
    for k, (_, _, d) in enumerate(batches):
        cl.http_verdicts_raw_dev(*d, outs[k], stream=(s1 if k < 2 else s2).cuda_stream)
    torch.cuda.synchronize()
    for k, (rq, raws, _) in enumerate(batches):
        got = outs[k].cpu().numpy()
        assert np.array_equal(got, _oracle(pols, *_args(rq), raws)), k
    cl.close()


def test_gpu_dl_late_slots_padded(gpu, dl):
    """A lane that gives up waiting for its chunk's id (forced here: no
    polling at all, CILIUM_GPU_RAW_SPIN=0) has its request walked and its slot
    padded by raw_seal_kernel from the late list: verdicts equal the host path
    and the oracle, and per-program and per-rule counters equal the default
    sequence's (an unfilled slot read by http_kernel would add a stale
    request's verdict and counts)."""
    pols, info = synth.http10k_rules()
    gpu.update_http_policy(pols)
    rq = synth.http10k_requests(20_000, info, seed=126)
    raws = _vary(_raw_requests(rq), np.random.default_rng(126))
    blob, off = _blob(raws)

    def run():
        gpu.reset_counters()
        v = gpu.http_verdicts_raw(*_args(rq), blob, off)
        return v, gpu.read_counters(N.CG_CTR_HTTP_PROGRAMS), gpu.read_counters(N.CG_CTR_HTTP_RULES)

    # the workspace first holds another batch's slots (stale meta and order)
    dl["CILIUM_GPU_RAW_SPIN"] = "16384"
    gpu.http_verdicts_raw(*_args(rq), *_blob(raws[::-1]))
    dl["CILIUM_GPU_RAW_SPIN"] = "0"
    v_late, p_late, r_late = run()
    dl.pop("CILIUM_GPU_RAW_SPIN")
    dl["CILIUM_GPU_RAW_LAYOUT"] = "host"  # the round-3 sequence
    v_def, p_def, r_def = run()
    assert np.array_equal(v_late, v_def)
    assert np.array_equal(v_late[:8_000], _oracle(pols, *(np.asarray(a)[:8_000] for a in _args(rq)), raws[:8_000]))
    assert np.array_equal(p_late, p_def)
    assert np.array_equal(r_late, r_def)


def test_gpu_dl_policy_swap_after_async_call(dl):
    """cg_http_verdicts_raw_dev returns with its kernels queued; a policy
    update right after it must not free the tables they read (the snapshot's
    fence): the queued batch's verdicts are the old policy's, the next
    batch's the new one's."""
    import torch
    cl = Classifier(device=0)
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    dev = torch.device("cuda:0")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(np.asarray(a).astype(dt))).to(dev)
    rq = synth.http10k_requests(30_000, info, seed=140)
    raws = _vary(_raw_requests(rq), np.random.default_rng(140))
    blob, off = _blob(raws)
    d = (t(blob, np.uint8), t(off, np.int64), len(raws), t(rq["policy"], np.int32), t(rq["ingress"], np.uint8),
         t(rq["port"], np.int16), t(rq["remote"], np.int32))
    exp1 = cl.http_verdicts_raw(*_args(rq), blob, off)  # the same path, synchronous
    s1 = torch.cuda.Stream(device=dev)
    out1 = torch.full((len(raws),), 7, dtype=torch.uint8, device=dev)
    out2 = torch.full((len(raws),), 7, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    cl.http_verdicts_raw_dev(*d, out1, stream=s1.cuda_stream)
    star = synth.starwars_policy()
    cl.update_http_policy(star)  # the old snapshot's last holder lets go here
    cl.http_verdicts_raw_dev(*d, out2, stream=s1.cuda_stream)
    torch.cuda.synchronize()
    got1 = out1.cpu().numpy()
    assert np.array_equal(got1, exp1)
    assert np.array_equal(got1[:8_000], _oracle(pols, *(np.asarray(a)[:8_000] for a in _args(rq)), raws[:8_000]))
    assert np.array_equal(out2.cpu().numpy(), _host_path(cl, *_args(rq), raws))
    cl.close()


def _big_program_policy(n_rules: int, seed: int = 1):
    """One program of n_rules random 12-character path prefixes: 732 rules
    compile to 40,303 table cells, 734 to 40,407 — either side of the
    largest block http_kernel stages in LDS next to the raw-byte path's code
    map (kMaxLdsCells, dev_types.h)."""
    import random
    r = random.Random(seed)
    al = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"
    words = ["".join(r.choice(al) for _ in range(12)) for _ in range(n_rules)]
    rules = [{"headers": [{"name": ":path", "regex_match": "/" + w + ".*"}]} for w in words]
    return [{"name": "big", "policy": 1, "ingress_per_port_policies": [{"port": 80, "rules": [
        {"remote_policies": [7], "http_rules": {"http_rules": rules}}]}]}], words


@pytest.mark.gpu
@pytest.mark.parametrize("n_rules", [732, 734])
def test_gpu_dl_program_at_lds_limit(gpu, n_rules):
    """A program at the LDS limit on the device-layout path (raw bytes coded
    through the LDS code map): its block either fits beside the map or
    walks from global memory; verdicts equal the host path's and the
    oracle's."""
    pols, words = _big_program_policy(n_rules)
    gpu.update_http_policy(pols)
    st = gpu.http_policy_stats()
    assert 40192 < st["max_program_cells"] < 40432, st
    assert st["lds_programs"] == (1 if n_rules == 732 else 0), st
    rng = np.random.default_rng(n_rules)
    raws = []
    for j in range(4000):
        w = words[int(rng.integers(0, len(words)))]
        if rng.random() < 0.5:
            w = w[:-1] + "_"
        raws.append(b"GET /%s/%d HTTP/1.1\r\nHost: big\r\n\r\n" % (w.encode(), j))
    n = len(raws)
    pol, ing, port, rem = [0] * n, [1] * n, [80] * n, [7] * n
    got = gpu.http_verdicts_raw(pol, ing, port, rem, *_blob(raws))
    assert np.array_equal(got, _host_path(gpu, pol, ing, port, rem, raws))
    assert np.array_equal(got, _oracle(pols, pol, ing, port, rem, raws))
    assert 0.3 < got.mean() < 0.7
