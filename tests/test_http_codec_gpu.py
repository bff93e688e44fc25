"""The codec step's known-answer vectors (tests/golden/http1_codec_kat.json:
http_parser's bare-LF line ends, method table, HTTP/1.1 only, Host required,
strict target bytes, Content-Length; led by the reference's Nightly.go head)
through the device parsers of kernels_http_raw.hip, on both sequences:

* every head as it is (parsed from its wave's LDS stage, parse_head_fast),
* the same head behind 7,000 CR / LF bytes — which http_parser's s_start_req
  skips, so the expected result is unchanged — too long for the stage, so it
  is deferred and parsed byte by byte from HBM (parse_head).

Two policies tell accepted from rejected and check the fields: "open" allows
any request that reaches the filter; "fields" allows exactly the (:method,
:path, :authority) triples of the accepted vectors.  Verdicts are compared
with the oracle (oracle/http1_ref.py, then the Envoy rule scan) and with
the vectors' own expectations."""
import os

import numpy as np
import pytest

from test_http_parse import CASES, CASE_NAMES, _blob
from test_http_raw_gpu import _host_path, _oracle

PAD = b"\r\n" * 3500


def _policies():
    triples = []
    for _, exp in CASES:
        if exp is None:
            continue
        d = dict(exp[:3])
        t = (d[b":method"], d[b":path"], d[b":authority"])
        if t[2] and t not in triples:
            triples.append(t)
    rules = [{"headers": [{"name": ":method", "exact_match": m.decode()}, {"name": ":path", "exact_match": p.decode()},
                          {"name": ":authority", "exact_match": a.decode()}]} for m, p, a in triples]
    pols = [{"name": "open", "policy": 9, "ingress_per_port_policies": [{"port": 80, "rules": [
                {"remote_policies": [7]}]}]},
            {"name": "fields", "policy": 10, "ingress_per_port_policies": [{"port": 80, "rules": [
                {"remote_policies": [7], "http_rules": {"http_rules": rules}}]}]}]
    return pols, triples


def _requests(cl):
    raws, pol, names = [], [], []
    for pad in (b"", PAD):
        for name in ("open", "fields"):
            for (raw, _), cname in zip(CASES, CASE_NAMES):
                raws.append(pad + raw)
                pol.append(cl.http_policy_index(name))
                names.append((name, cname, bool(pad)))
    n = len(raws)
    return raws, pol, [1] * n, [80] * n, [7] * n, names


def _expected(names, triples):
    exp = []
    for pname, cname, _ in names:
        e = CASES[CASE_NAMES.index(cname)][1]
        if e is None:
            exp.append(0)
        elif pname == "open":
            exp.append(1)
        else:
            d = dict(e[:3])
            exp.append(int((d[b":method"], d[b":path"], d[b":authority"]) in triples))
    return exp


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["device", "host"])
def test_gpu_codec_kat(gpu, layout, monkeypatch):
    monkeypatch.setenv("CILIUM_GPU_RAW_LAYOUT", layout)
    pols, triples = _policies()
    gpu.update_http_policy(pols)
    raws, pol, ing, port, rem, names = _requests(gpu)
    got = gpu.http_verdicts_raw(pol, ing, port, rem, *_blob(raws))
    exp = _oracle(pols, pol, ing, port, rem, raws)
    bad = [names[i] for i in range(len(raws)) if got[i] != exp[i]]
    assert not bad, bad
    assert got.tolist() == _expected(names, triples)
    # the host codec + packer path agrees
    assert np.array_equal(got, _host_path(gpu, pol, ing, port, rem, raws))
    # the Nightly head is allowed by "open" in both forms
    assert all(got[i] == 1 for i, (p, c, _) in enumerate(names) if p == "open" and c.startswith("nightly echo"))


def test_codec_kat_host_path(host):
    """The same vectors through the host codec and packer (no GPU)."""
    pols, triples = _policies()
    host.update_http_policy(pols)
    raws, pol, ing, port, rem, names = _requests(host)
    got = host.http_eval_host_diag(host.pack_http_raw(pol, ing, port, rem, *_blob(raws)))
    assert got.tolist() == _expected(names, triples)
