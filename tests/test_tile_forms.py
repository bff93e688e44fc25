"""Half last units (cg_http_pack, kTileHalfLast): a tile whose lanes hold at
most 8 bytes in the last string unit stores it as 8 bytes per lane.  Star
wars requests with paths of every length from 4 to 67 bytes, 64 copies of
each, so tiles end at every byte of a unit (tails 1..16): the host walk of
the packed batch equals the oracle (CPU), and http_kernel's verdicts equal
it too (GPU)."""
import numpy as np
import pytest

import oracle
from cilium_amd import synth


def _requests():
    base = synth.starwars_requests(1)
    lists = []
    for k in range(64):
        path = b"/v1/" + bytes(97 + (i % 26) for i in range(k))
        for m, method in enumerate((b"GET", b"POST", b"PUT", b"DELETE")):
            for c in range(16):  # 64 requests of each path length
                h = b":method\0" + method + b"\0:path\0" + path + b"\0:authority\0deathstar.empire.svc\0"
                if c & 1:
                    h += b"X-Has-Force\0" + (b"true" if c & 2 else b"false") + b"\0"
                lists.append(h)
    n = len(lists)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in lists])
    return dict(policy=np.repeat(base["policy"][:1], n), ingress=np.repeat(base["ingress"][:1], n),
                port=np.repeat(base["port"][:1], n),
                remote=np.where(np.arange(n) % 3 == 0, np.uint32(9999), np.repeat(base["remote"][:1], n)).astype(
                    np.uint32),
                hdr_blob=np.frombuffer(b"".join(lists), np.uint8).copy(), hdr_off=off)


def _forms(b):
    ttab_off = int(b.batch[32:40].view(np.uint64)[0])
    ntiles = int(b.batch[12:16].view(np.uint32)[0])
    u = b.batch[ttab_off:ttab_off + 8 * ntiles].view(np.uint32).reshape(-1, 2)[:, 1]
    return (u >> 15) & 1, u >> 16  # half flag, tail bytes


def test_half_last_units_host(host):
    pols = synth.starwars_policy()
    host.update_http_policy(pols)
    rq = _requests()
    b = host.pack_http(**rq)
    half, tail = _forms(b)
    assert half.any() and (~half.astype(bool) & (tail > 8)).any()
    assert np.all(tail[half.astype(bool)] <= 8)
    assert np.array_equal(host.http_eval_host_diag(b), oracle.HttpOracle(pols).eval(**rq))


@pytest.mark.gpu
def test_half_last_units_gpu(gpu):
    pols = synth.starwars_policy()
    gpu.update_http_policy(pols)
    rq = _requests()
    b = gpu.pack_http(**rq)
    assert _forms(b)[0].any()
    assert np.array_equal(gpu.http_verdicts(b), oracle.HttpOracle(pols).eval(**rq))
