"""Bounded, seeded fuzz of the host code that parses untrusted bytes, run
against the ASan + UBSan build (tools/sanitize/run.sh sets CILIUM_AMD_LIB):

- npds_pb.cc    mutated serialized DiscoveryResponses (HTTP and proxylib
                updates), including the new matcher forms;
- json.h + http.cc  mutated NPDS JSON policies;
- http_image.cc mutated compiled-policy images;
- http_parse.cc mutated and random HTTP/1 heads (cg_http_parse_heads);
- kafka_wire.cc mutated Kafka requests, plain and compressed
                (cg_kafka_decode on the host decoder);
- proxylib_{memcache,cassandra}.cc and the r2d2 framing: random byte streams
                through OnData on a device=-1 module (no policy installed: the
                framing runs, every frame is denied).

A return code is whatever it is; the run fails only on a sanitizer report
(the process aborts) or a Python exception from the harness itself.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from cilium_amd import _native as N  # noqa: E402
from cilium_amd import kafka_requests as K  # noqa: E402
from cilium_amd import synth  # noqa: E402
from cilium_amd.classifier import Classifier  # noqa: E402


def mutate(b: bytes, rng) -> bytes:
    a = bytearray(b)
    for _ in range(int(rng.integers(1, 6))):
        k = int(rng.integers(0, 5))
        if k == 0 and a:  # flip bits
            i = int(rng.integers(0, len(a)))
            a[i] ^= 1 << int(rng.integers(0, 8))
        elif k == 1 and a:  # truncate
            del a[int(rng.integers(0, len(a))):]
        elif k == 2:  # insert random bytes
            i = int(rng.integers(0, len(a) + 1))
            a[i:i] = rng.integers(0, 256, int(rng.integers(1, 9))).astype(np.uint8).tobytes()
        elif k == 3 and a:  # set a byte to a boundary value
            a[int(rng.integers(0, len(a)))] = int(rng.choice([0, 1, 0x7F, 0x80, 0xFF, 0x0A, 0x0D, 0x3A]))
        elif k == 4 and len(a) > 2:  # duplicate a slice
            i = int(rng.integers(0, len(a) - 1))
            j = int(rng.integers(i + 1, len(a)))
            a[j:j] = a[i:j]
    return bytes(a)


def fuzz_npds(rng, iters):
    import npds_pb as PB
    from test_cpu_differential import all_matcher_case
    cl = Classifier(device=-1)
    seeds = [PB.discovery_response(all_matcher_case(s, 10)[0]) for s in range(3)]
    seeds.append(PB.discovery_response(synth.starwars_policy()))
    for _ in range(iters):
        blob = mutate(seeds[int(rng.integers(0, len(seeds)))], rng)
        N.lib.cg_http_policy_update_npds(cl.h, blob, len(blob))
    cl.close()


def fuzz_json(rng, iters):
    from test_cpu_differential import all_matcher_case
    cl = Classifier(device=-1)
    seeds = [json.dumps(all_matcher_case(s, 10)[0]).encode() for s in range(3)]
    for _ in range(iters):
        blob = mutate(seeds[int(rng.integers(0, len(seeds)))], rng)
        N.lib.cg_http_policy_update(cl.h, blob, len(blob))
    cl.close()


def _fnv64(b: bytes) -> int:
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def fuzz_image(rng, iters):
    """Mutated images with the trailing FNV-64 recomputed (a checksum is no
    MAC), so the structural checks are exercised; every accepted image is
    walked by the host verdict path."""
    cl = Classifier(device=-1)
    cl.update_http_policy(synth.starwars_policy())
    img = cl.export_http_policy()
    rq = synth.starwars_requests(64, seed=9)
    for _ in range(iters):
        body = mutate(img[:-8], rng)
        blob = body + _fnv64(body).to_bytes(8, "little")
        if N.lib.cg_http_policy_import(cl.h, blob, len(blob)) == N.CG_OK:
            try:
                cl.http_eval_host_diag(cl.pack_http(**rq))
            except N.CiliumGPUError:
                pass
    cl.close()


def fuzz_heads(rng, iters):
    from test_http_parse import _raw_requests
    rq = synth.starwars_requests(200, seed=9)
    base = _raw_requests(rq)
    for _ in range(iters // 64):
        raws = [mutate(base[int(rng.integers(0, len(base)))], rng) for _ in range(64)]
        raws.append(rng.integers(0, 256, int(rng.integers(0, 300))).astype(np.uint8).tobytes())
        off = np.zeros(len(raws) + 1, np.uint64)
        off[1:] = np.cumsum([len(r) for r in raws])
        Classifier.parse_http_heads(np.frombuffer(b"".join(raws) or b"\0", np.uint8).copy(), off)


def fuzz_kafka(rng, iters):
    from kafka_corpus import corpus
    pols, info = synth.kafka_policy(n_rules=50, n_topics=20, n_clients=5, seed=3)
    cl = Classifier(device=-1)
    cl.update_kafka_policy(pols)
    topics = [t.encode() for t in info["topics"]]
    clients = [c.encode() for c in info["clients"]]
    base = corpus(3, 300, topics, clients)
    for _ in range(iters // 32):
        reqs = [mutate(base[int(rng.integers(0, len(base)))], rng) for _ in range(32)]
        raw, off = K.concat(reqs)
        n = len(reqs)
        try:
            cl.kafka_decode(raw, off, np.zeros(n, np.uint16), np.zeros(n, np.uint32), diag_cpu=True)
        except N.CiliumGPUError:
            pass
    cl.close()


def fuzz_proxylib(rng, iters):
    from test_proxylib_abi import Conn, _lib, open_module
    inst = open_module([(b"node-id", b"asan-fuzz")], "-1")
    done = 0
    while done < iters:
        proto = [b"r2d2", b"memcache", b"cassandra"][int(rng.integers(0, 3))]
        c = Conn(inst, proto=proto, policy=b"not-installed")
        for _ in range(int(rng.integers(1, 12))):
            chunks = [rng.integers(0, 256, int(rng.integers(0, 200))).astype(np.uint8).tobytes()
                      for _ in range(int(rng.integers(1, 4)))]
            if rng.random() < 0.5 and proto == b"cassandra":
                hdr = bytes([4, 0, 0, int(rng.integers(0, 3)), int(rng.integers(0, 16))])
                body = rng.integers(0, 256, int(rng.integers(0, 64))).astype(np.uint8).tobytes()
                chunks = [hdr + len(body).to_bytes(4, "big") + body]
            c.on_data(chunks, reply=bool(rng.random() < 0.3))
            done += 1
        c.close()
    _lib.CloseModule(inst)


def main():
    budget = float(os.environ.get("FUZZ_SECONDS", "20"))
    rng = np.random.default_rng(int(os.environ.get("FUZZ_SEED", "1")))
    report = {}
    for name, fn, iters in (("npds_pb", fuzz_npds, 3000), ("npds_json", fuzz_json, 1500), ("image", fuzz_image, 1500),
                            ("http_heads", fuzz_heads, 20000), ("kafka_wire", fuzz_kafka, 6000),
                            ("proxylib", fuzz_proxylib, 4000)):
        t0 = time.time()
        n = 0
        while time.time() - t0 < budget / 6 or n == 0:
            fn(rng, iters)
            n += iters
        report[name] = {"inputs": n, "seconds": round(time.time() - t0, 1)}
        print(name, report[name], flush=True)
    print(json.dumps({"fuzz": report, "lib": str(N.LIB_PATH)}))


if __name__ == "__main__":
    main()
