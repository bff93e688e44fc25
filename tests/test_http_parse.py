"""HTTP/1.x request heads from raw bytes → the packer.

The codec is Envoy's http_parser (external; parity unpinned): the cases are
written from RFC 7230's request-line / header-field grammar.  The product
parser (csrc/http_parse.cc) is checked against oracle/http1_ref.py, and the
raw path's verdicts against the header-list path's on the same requests."""
import numpy as np
import pytest

import oracle
from cilium_amd import synth
from cilium_amd.classifier import Classifier
from oracle.http1_ref import parse_head

CASES = [
    (b"GET /v1/ HTTP/1.1\r\nHost: deathstar\r\nX-Has-Force: true\r\n\r\n",
     [(b":method", b"GET"), (b":path", b"/v1/"), (b":authority", b"deathstar"), (b"X-Has-Force", b"true")]),
    (b"PUT /a?b=c HTTP/1.0\r\nhost:  h1 \r\nHOST: h2\r\nx:\t v \t\r\n\r\n",
     [(b":method", b"PUT"), (b":path", b"/a?b=c"), (b":authority", b"h1"), (b"x", b"v")]),
    (b"DELETE * HTTP/1.1\r\n\r\n", [(b":method", b"DELETE"), (b":path", b"*")]),
    (b"GET /x HTTP/1.1\r\nEmpty:\r\n\r\nBODY", [(b":method", b"GET"), (b":path", b"/x"), (b"Empty", b"")]),
    (b"GET /x HTTP/1.1\r\nA: 1\r\n", None),            # no final CRLF
    (b"GET /x HTTP/1.1\nA: 1\n\n", None),              # bare LF
    (b"G@T /x HTTP/1.1\r\n\r\n", None),                 # method not a token
    (b"GET  /x HTTP/1.1\r\n\r\n", None),                # empty target
    (b"GET /x HTTP/11\r\n\r\n", None),                  # bad version
    (b"GET /x HTTP/1.1\r\nBad Name: v\r\n\r\n", None),  # space in the name
    (b"GET /x HTTP/1.1\r\nA: v\x01w\r\n\r\n", None),    # control byte in the value
    (b"GET /x HTTP/1.1\r\n: v\r\n\r\n", None),          # empty name
]


def _blob(raws):
    off = np.zeros(len(raws) + 1, np.uint64)
    off[1:] = np.cumsum([len(r) for r in raws])
    return np.frombuffer(b"".join(raws) or b"\0", np.uint8).copy(), off


def _lists(blob, off, ok):
    out = []
    for i in range(len(ok)):
        if not ok[i]:
            out.append(None)
            continue
        parts = bytes(blob[int(off[i]):int(off[i + 1])]).split(b"\0")[:-1]
        out.append(list(zip(parts[0::2], parts[1::2])))
    return out


def test_oracle_cases():
    for raw, exp in CASES:
        assert parse_head(raw) == exp, raw


def test_library_parser_cases():
    blob, off, ok = Classifier.parse_http_heads(*_blob([r for r, _ in CASES]))
    assert _lists(blob, off, ok) == [e for _, e in CASES]


def _raw_requests(rq):
    """synth header lists → raw heads (":authority" sent as Host)."""
    raws = []
    blob, off = rq["hdr_blob"], rq["hdr_off"]
    for i in range(len(off) - 1):
        parts = bytes(blob[int(off[i]):int(off[i + 1])]).split(b"\0")[:-1]
        hs = dict(zip(parts[0::2], parts[1::2]))
        head = hs.pop(b":method") + b" " + hs.pop(b":path") + b" HTTP/1.1\r\n"
        if b":authority" in hs:
            head += b"Host: " + hs.pop(b":authority") + b"\r\n"
        head += b"".join(k + b": " + v + b"\r\n" for k, v in hs.items()) + b"\r\n"
        raws.append(head)
    return raws


def test_random_heads_vs_oracle():
    rq = synth.starwars_requests(3000, seed=5)
    raws = _raw_requests(rq)
    rng = np.random.default_rng(3)
    for i in rng.choice(len(raws), 300, replace=False):  # corrupt a tenth
        r = bytearray(raws[i])
        r[int(rng.integers(0, len(r)))] = int(rng.choice([0x01, 0x0a, 0x20, 0x3a, 0x7f]))
        raws[i] = bytes(r)
    blob, off, ok = Classifier.parse_http_heads(*_blob(raws))
    assert _lists(blob, off, ok) == [parse_head(r) for r in raws]


def _raw_vs_lists(cl, rq, pols):
    raws = _raw_requests(rq)
    b = cl.pack_http_raw(rq["policy"], rq["ingress"], rq["port"], rq["remote"], *_blob(raws))
    exp = oracle.HttpOracle(pols).eval(**rq)
    return b, exp


def test_raw_path_tables(host):
    pols = synth.starwars_policy()
    host.update_http_policy(pols)
    rq = synth.starwars_requests(5000, seed=11)
    b, exp = _raw_vs_lists(host, rq, pols)
    assert np.array_equal(host.http_eval_host_diag(b), exp)


@pytest.mark.gpu
def test_gpu_raw_path(gpu):
    pols = synth.starwars_policy()
    gpu.update_http_policy(pols)
    rq = synth.starwars_requests(50_000, seed=12)
    b, exp = _raw_vs_lists(gpu, rq, pols)
    assert np.array_equal(gpu.http_verdicts(b), exp)
    # rejected heads are denied
    raws = [r for r, e in CASES]
    n = len(raws)
    pidx = gpu.http_policy_index(pols[0]["name"])
    b = gpu.pack_http_raw(np.full(n, pidx, np.uint32), np.zeros(n, np.uint8), np.full(n, 80, np.uint16),
                          np.full(n, synth.SPACESHIP_ID, np.uint32), *_blob(raws))
    got = gpu.http_verdicts(b)
    assert all(got[i] == 0 for i, (_, e) in enumerate(CASES) if e is None)


def test_rejected_heads_denied_without_ok(host):
    """A head the codec rejects is denied even when the caller packs it under
    a real policy whose port allows everything (no HTTP rules): its header
    list carries a DEL value the packer flags malformed."""
    pols = [{"name": "open", "policy": 1, "ingress_per_port_policies": [
        {"port": 80, "rules": [{"remote_policies": [7]}]}]}]
    host.update_http_policy(pols)
    good = b"GET /x HTTP/1.1\r\nHost: a\r\n\r\n"
    bad = [b"GET /x HTTP/1.1\r\nHost: a\x01b\r\n\r\n", b"GET /x HTTP/1.1\r\n", b"G@T /x HTTP/1.1\r\n\r\n"]
    raws = [good] + bad
    blob, off, ok = Classifier.parse_http_heads(*_blob(raws))
    assert ok.tolist() == [1, 0, 0, 0]
    n = len(raws)
    b = host.pack_http(np.zeros(n, np.uint32), np.ones(n, np.uint8), np.full(n, 80, np.uint16),
                       np.full(n, 7, np.uint32), blob, off)
    assert host.http_eval_host_diag(b).tolist() == [1, 0, 0, 0]
