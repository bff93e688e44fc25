"""HTTP/1.x request heads from raw bytes → the packer.

What stands before the filter is Envoy's http_parser plus the connection
manager's checks (external, not vendored).  tests/golden/http1_codec_kat.json
holds 60 hand-written vectors of their rules (bare LF line ends, the method
table, HTTP/1.1 only, Host required, strict target bytes, Content-Length),
led by the reference's own Nightly.go head with `echo -e`'s trailing LF.  The
oracle (oracle/http1_ref.py) and the product parser (csrc/http_parse.cc) are
checked against them and against each other on mutated heads; the raw path's
verdicts against the header-list path's on the same requests."""
import json
import os

import numpy as np
import pytest

import oracle
from cilium_amd import synth
from cilium_amd.classifier import Classifier
from oracle.http1_ref import parse_head

_KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "http1_codec_kat.json")))


def _kat_expect(e):
    return None if e is None else [(k.encode("latin-1"), v.encode("latin-1")) for k, v in e]


CASES = [(c["raw"].encode("latin-1"), _kat_expect(c["expect"])) for c in _KAT["cases"]]
CASE_NAMES = [c["name"] for c in _KAT["cases"]]
BAD_VALUE_HEAD = b"GET /x HTTP/1.1\r\nHost: a\r\nA: v\x01w\r\n\r\n"  # control byte in a value


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
    assert len(CASES) >= 60 and CASE_NAMES[0].startswith("nightly")
    for (raw, exp), name in zip(CASES, CASE_NAMES):
        assert parse_head(raw) == exp, name


def test_library_parser_cases():
    blob, off, ok = Classifier.parse_http_heads(*_blob([r for r, _ in CASES]))
    got = _lists(blob, off, ok)
    for g, (_, e), name in zip(got, CASES, CASE_NAMES):
        assert g == e, name


def _line_end_mix(raw: bytes, rng) -> bytes:
    """Each CR LF of a head as CR LF or a bare LF, sometimes CR / LF bytes
    in front, an extra SP before the target, a Content-Length line."""
    parts = raw.split(b"\r\n")
    out = parts[0]
    for p in parts[1:]:
        out += (b"\n" if rng.random() < 0.5 else b"\r\n") + p
    if rng.random() < 0.1:
        out = rng.choice([b"\r\n", b"\n", b"\r", b"\n\r\n"]) + out
    if rng.random() < 0.1:
        out = out.replace(b" ", b"  ", 1)
    if rng.random() < 0.1:
        cl = rng.choice([b"0", b"12", b"00", b"1x", b"1 ", b"2\t", b"", b"18446744073709551610"])
        i = out.find(b"\n") + 1
        out = out[:i] + b"Content-Length: " + cl + b"\r\n" + out[i:]
    return out


def test_line_end_mixes_vs_oracle():
    """CR LF / bare LF mixes (and the other leniencies) of synth heads: the
    product parser equals the oracle, and the mixes parse as the CR LF heads
    do."""
    rq = synth.starwars_requests(3000, seed=7)
    base = _raw_requests(rq)
    rng = np.random.default_rng(8)
    raws = [_line_end_mix(r, rng) for r in base]
    blob, off, ok = Classifier.parse_http_heads(*_blob(raws))
    got = _lists(blob, off, ok)
    assert got == [parse_head(r) for r in raws]
    plain = [i for i, r in enumerate(raws) if b"Content-Length" not in r]
    assert all(got[i] == parse_head(base[i]) for i in plain)
    assert sum(g is not None for g in got) > 0.9 * len(raws)


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
    for i in rng.choice(len(raws), 900, replace=False):  # corrupt a third
        r = bytearray(raws[i])
        r[int(rng.integers(0, len(r)))] = int(rng.choice([0x01, 0x0a, 0x0d, 0x20, 0x3a, 0x7f, 0x80, 0xc3, 0x2f]))
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
