"""Policy updates racing verdict calls on one handle: a thread swaps the
HTTP policy between two versions (the star-wars rules with and without the
PUT rule) while others decide requests through the host entries.  Each call
sees one snapshot whole — its verdicts equal the first version's or the
second's for every request of the call, never a mix — and the tables a call
was launched against stay alive until it is done (cilium_network_policy.h
swaps the policy map under a read-copy-update pointer the same way)."""
import copy
import threading

import numpy as np
import pytest

import oracle
from cilium_amd import synth
from test_http_parse import _blob, _raw_requests

pytestmark = [pytest.mark.gpu]


def _without_put(pols):
    p = copy.deepcopy(pols)
    for pol in p:
        for d in ("ingress_per_port_policies", "egress_per_port_policies"):
            for pp in pol.get(d, []):
                for r in pp["rules"]:
                    hr = r["http_rules"]["http_rules"]
                    r["http_rules"]["http_rules"] = [x for x in hr
                                                     if not any(h.get("regex_match") == "PUT" for h in x["headers"])]
    return p


def test_gpu_policy_swaps_under_calls(gpu):
    p1 = synth.starwars_policy()
    p2 = _without_put(p1)
    rq = synth.starwars_requests(30_000, seed=81)
    args = (rq["policy"], rq["ingress"], rq["port"], rq["remote"])
    want = []
    for p in (p1, p2):
        gpu.update_http_policy(p)
        w = gpu.http_verdicts_fields(*args, rq["hdr_blob"], rq["hdr_off"])
        assert np.array_equal(w, oracle.HttpOracle(p).eval(*args, rq["hdr_blob"], rq["hdr_off"]))
        want.append(w)
    assert not np.array_equal(want[0], want[1])  # the PUT rule matters for these requests
    raw_blob, raw_off = _blob(_raw_requests(rq))
    off = rq["hdr_off"]
    stop = threading.Event()
    errors, seen = [], set()

    def updater():
        k = 0
        while not stop.is_set():
            gpu.update_http_policy(p2 if k % 2 == 0 else p1)
            k += 1

    def caller(t):
        r = np.random.default_rng(900 + t)
        for _ in range(40):
            n = int(r.choice([5, 200, 2000, 9000]))
            a = int(r.integers(0, len(want[0]) - n))
            sub = tuple(np.asarray(x)[a:a + n] for x in args)
            if t % 2:
                got = gpu.http_verdicts_fields(*sub, rq["hdr_blob"], np.ascontiguousarray(off[a:a + n + 1]))
            else:
                got = gpu.http_verdicts_raw(*sub, raw_blob, np.ascontiguousarray(raw_off[a:a + n + 1]))
            which = [v for v in (0, 1) if np.array_equal(got, want[v][a:a + n])]
            if not which:
                errors.append((t, a, n))
            seen.update(which)

    up = threading.Thread(target=updater)
    cs = [threading.Thread(target=caller, args=(t,)) for t in range(4)]
    up.start()
    for x in cs:
        x.start()
    for x in cs:
        x.join(timeout=240)
        assert not x.is_alive(), "a call never returned"
    stop.set()
    up.join(timeout=60)
    assert not errors, errors[:5]
    gpu.update_http_policy(p1)
