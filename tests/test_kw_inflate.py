"""The GPU Kafka decoder's gzip / snappy payload decoding
(cilium_amd/csrc/kw_inflate.h) run on the CPU: the header is host+device,
tests/native/kwz_test.cc builds it with hipcc's host compiler.  Every case is
checked against the oracle's restatement of the host decoder
(oracle/kafka_wire_ref.py gunzip / snappy_decode: compress/gzip over zlib,
golang/snappy): a decoded payload must equal the oracle's bytes, an error
must be an oracle error, and "more" (the kernel hands the request to the
host) is allowed only where the device cannot size or finish the payload
alone — a second gzip member, or output beyond the ISIZE / snappy length
the buffer was sized from.  Cases: zlib levels 0-9 (stored, fixed and
dynamic blocks), Z_FIXED and Z_HUFFMAN_ONLY strategies, FNAME / FCOMMENT /
FEXTRA / FHCRC headers, empty payloads, snappy blocks and xerial chunks,
and thousands of randomly damaged members."""
import gzip
import io
import os
import shutil
import struct
import subprocess
import zlib

import numpy as np
import pytest

from cilium_amd import kafka_requests as K
from oracle import kafka_wire_ref as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OK, ERR, MORE = 0, 1, 2


def _gz_raw(data: bytes, level: int, strategy: int = zlib.Z_DEFAULT_STRATEGY, flags: int = 0,
            extra: bytes = b"", name: bytes = b"", comment: bytes = b"", fhcrc: bool = False) -> bytes:
    """A gzip member built by hand around zlib's raw deflate."""
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
    body = c.compress(data) + c.flush()
    flg = (4 if extra else 0) | (8 if name else 0) | (16 if comment else 0) | (2 if fhcrc else 0)
    h = bytes([0x1F, 0x8B, 8, flg]) + b"\0\0\0\0" + bytes([0, 255])
    if extra:
        h += struct.pack("<H", len(extra)) + extra
    if name:
        h += name + b"\0"
    if comment:
        h += comment + b"\0"
    if fhcrc:
        h += struct.pack("<H", zlib.crc32(h) & 0xFFFF)
    return h + body + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data) & 0xFFFFFFFF)


def _payloads(rng):
    words = [b"topic", b"kafka", b"cilium", b"message", b"\x00\x01", b"value-", b"key"]
    for n in (0, 1, 5, 64, 700, 5000, 40000, 70000):
        text = b"".join(words[int(i)] for i in rng.integers(0, len(words), max(1, n // 5)))[:n]
        noise = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        mixed = bytes(a if rng.random() < 0.7 else b for a, b in zip(text, noise)) if n <= 5000 else text[:n // 2] + noise[:n // 2]
        yield text
        yield noise
        yield mixed


def _cases(rng):
    cases = []
    for data in _payloads(rng):
        for lvl in (0, 1, 6, 9):
            cases.append((1, _gz_raw(data, lvl)))
        cases.append((1, _gz_raw(data, 6, zlib.Z_FIXED)))
        cases.append((1, _gz_raw(data, 6, zlib.Z_HUFFMAN_ONLY)))
        cases.append((1, _gz_raw(data, 6, extra=b"xy" * 3, name=b"set.bin", comment=b"c", fhcrc=True)))
        cases.append((1, gzip.compress(data, mtime=0)))
        cases.append((2, K.snappy_block(data)))
        cases.append((2, K.snappy_xerial(data, int(rng.integers(8, 4096)))))
    clean = len(cases)
    # a second member, trailing bytes
    d = b"abc" * 100
    cases.append((1, gzip.compress(d, mtime=0) + gzip.compress(d, mtime=0)))
    cases.append((1, gzip.compress(d, mtime=0) + b"\0\0"))
    # damage: random bytes / bits of valid members
    base = [c for c in cases if len(c[1]) > 12]
    for _ in range(4000):
        codec, b = base[int(rng.integers(0, len(base)))]
        b = bytearray(b)
        for _ in range(int(rng.integers(1, 4))):
            i = int(rng.integers(0, len(b)))
            if rng.random() < 0.5:
                b[i] ^= 1 << int(rng.integers(0, 8))
            else:
                b[i] = int(rng.integers(0, 256))
        if rng.random() < 0.2:
            b = b[:int(rng.integers(1, len(b)))]
        cases.append((codec, bytes(b)))
    return cases, clean


def _oracle(codec, b):
    try:
        return OK, (R.gunzip(b) if codec == 1 else R.snappy_decode(b))
    except Exception:  # noqa: BLE001 — any decode failure is the host's error
        return ERR, None


def test_kw_inflate_against_the_host_restatement(tmp_path):
    hipcc = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)
    if hipcc is None:
        pytest.skip("no hipcc")
    exe = str(tmp_path / "kwz_test")
    subprocess.run([hipcc, "-x", "hip", "--cuda-host-only", "-O2", "-std=c++17",
                    "-I", os.path.join(ROOT, "cilium_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "kwz_test.cc"), "-o", exe],
                   check=True, capture_output=True, timeout=300)
    rng = np.random.default_rng(0x6A1F)
    cases, clean = _cases(rng)
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(fin, "wb") as f:
        for codec, b in cases:
            f.write(bytes([codec]) + struct.pack("<I", len(b)) + b)
    r = subprocess.run([exe, str(fin), str(fout)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "kwz ok" in r.stdout, r.stderr
    res = io.BytesIO(fout.read_bytes())
    counts = {OK: 0, ERR: 0, MORE: 0}
    for k, (codec, b) in enumerate(cases):
        st, cap, ol = res.read(1)[0], *struct.unpack("<II", res.read(8))
        got = res.read(ol)
        counts[st] += 1
        if k < clean:  # every intact single member / snappy payload decodes on the device
            assert st == OK, (k, codec, st)
        ost, exp = _oracle(codec, b)
        if st == OK:
            assert ost == OK and got == exp, (k, codec, b[:40])
        elif st == ERR:
            assert ost == ERR, (k, codec, b[:40], len(exp or b""))
        else:
            assert st == MORE, st
            # only what the device cannot size or finish: several members,
            # or output past the buffer sized from ISIZE / the snappy length
            assert ost == ERR or len(exp) != cap, (k, codec, cap, len(exp))
    print("kw_inflate cases:", counts)
    assert counts[OK] >= 400 and counts[ERR] >= 1000, counts
