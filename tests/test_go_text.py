"""Go string semantics of the proxylib parsers (cilium_amd/csrc/go_text.h):
strings.ToLower (Go 1.10 strings.Map over unicode.ToLower, Unicode 10.0) and
strings.Fields over decoded runes, as cassandraparser.go:372-417 and the
memcache text parser apply them.  The C++ header is compiled with g++ into a
small driver and compared with the oracle's restatement (oracle/memcache_ref.py)
on hand-checked cases and random byte/rune mixtures; CPU only."""
from __future__ import annotations

import os
import shutil
import subprocess

import numpy as np
import pytest

from oracle.memcache_ref import go_fields, go_lower_rune, go_to_lower

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("go_text") / "go_text_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "cilium_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "go_text_check.cc"), "-o", exe], check=True)
    return exe


def _run(exe, strings):
    inp = "".join((s.hex() or "") + "\n" for s in strings)
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    res = []
    for line in out:
        parts = line.split(" ")
        low = b"" if parts[0] == "-" else bytes.fromhex(parts[0])
        res.append((low, [bytes.fromhex(p) for p in parts[1:]]))
    return res


# Known Go 1.10 results (unicode.ToLower is the simple mapping: U+0130 -> "i";
# Unicode 11+ case pairs such as Georgian Mtavruli U+1C90 are unmapped; after
# the first changed rune an invalid byte is re-encoded as U+FFFD)
KNOWN = [
    ("SELECT a FROM Ks.T".encode(), b"select a from ks.t"),
    ("ÜSERS".encode(), "üsers".encode()),
    ("İ".encode(), b"i"),
    ("ΣΑΣ".encode(), "σασ".encode()),
    ("ǅ".encode(), "ǆ".encode()),
    ("Ა".encode(), "Ა".encode()),
    ("Ꞹ".encode(), "Ꞹ".encode()),
    (b"\xffA\xc3\x9c\xff", b"\xff" + b"a" + "ü".encode() + "�".encode()),
    (b"\xff\xfe", b"\xff\xfe"),
    ("Ａ".encode(), "ａ".encode()),
    ("\U00010400".encode(), "\U00010428".encode()),
]


def test_oracle_known_values():
    for s, low in KNOWN:
        assert go_to_lower(s) == low, s
    assert go_lower_rune(0x130) == 0x69 and go_lower_rune(0x212A) == 0x6B  # Kelvin sign
    assert go_fields("a b　c  d\x85e".encode()) == [b"a", b"b", b"c", b"d", b"e"]
    assert go_fields(b"a\xc2b \xffc") == [b"a\xc2b", b"\xffc"]


def test_cpp_matches_oracle_known(driver):
    res = _run(driver, [s for s, _ in KNOWN])
    for (s, low), (clow, _) in zip(KNOWN, res):
        assert clow == low, s


ALPHABET = [b"A", b"z", b" ", b"\t", b";", "Ü".encode(), "ß".encode(), "İ".encode(), "Σ".encode(), " ".encode(),
            "　".encode(), " ".encode(), "Ა".encode(), "Ω".encode(), "Ꭰ".encode(), "\U0001e900".encode(),
            b"\xff", b"\xc3", b"\xe0\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", "�".encode(), b"\x85",
            "\u0085".encode(), "Ⅻ".encode(), "ⓐ".encode(), "Ⓐ".encode()]


def test_cpp_matches_oracle_random(driver):
    rng = np.random.default_rng(5)
    strings = []
    for _ in range(3000):
        k = int(rng.integers(0, 12))
        strings.append(b"".join(ALPHABET[int(i)] for i in rng.integers(0, len(ALPHABET), k)))
    # every BMP + supplementary case pair, one rune per string
    strings += [chr(cp).encode("utf-8", "surrogatepass") for cp in range(0x80, 0x1F000) if not 0xD800 <= cp <= 0xDFFF]
    res = _run(driver, strings)
    for s, (clow, cf) in zip(strings, res):
        assert clow == go_to_lower(s), s
        assert cf == go_fields(s), s
