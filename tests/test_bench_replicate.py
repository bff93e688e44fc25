"""bench.replicate_batch (the headline's device batch: reps copies of a
packed batch laid out as the packer lays out a batch of reps x D requests)
on the CPU: the host walk of every copy of every tile equals the original
tile's, for both layouts and with half last units and compact meta words in
the batch."""
import numpy as np
import pytest
import torch

import bench
from cilium_amd import synth
from cilium_amd.classifier import Classifier, HttpBatch


@pytest.mark.parametrize("layout", ["tile", "copy"])
def test_replicated_batch_walks_like_the_original(layout):
    cl = Classifier(device=-1)
    pols, info = synth.http10k_rules()
    cl.update_http_policy(pols)
    b = cl.pack_http(**synth.http10k_requests_fast(20_000, info))
    ttab_off = int(b.batch[32:40].view(np.uint64)[0])
    ntiles = int(b.batch[12:16].view(np.uint32)[0])
    form = b.batch[ttab_off:ttab_off + 8 * ntiles].view(np.uint32).reshape(-1, 2)[:, 1]
    assert ((form >> 15) & 1).any() and not ((form >> 15) & 1).all()  # half and whole last units
    v0 = cl.http_eval_host_diag_slots(b)
    reps = 3
    d, nslots, tile_map, _, groups = bench.replicate_batch(b, reps, torch.device("cpu"), torch, layout=layout,
                                                           return_groups=True)
    group_nt = np.zeros(len(tile_map), np.int64)  # "copy": copy r of a group follows r whole groups
    for first, nt, _ in groups:
        group_nt[first:first + nt] = nt
    v1 = cl.http_eval_host_diag_slots(HttpBatch(d.numpy(), b.arena, np.arange(nslots, dtype=np.uint32), nslots,
                                                nslots))
    t = np.asarray(tile_map)
    for k in range(len(t)):
        for r in range(reps):
            at = t[k] + r if layout == "tile" else t[k] + r * group_nt[k]
            assert np.array_equal(v1[at * 64:at * 64 + 64], v0[k * 64:k * 64 + 64]), (k, r)
    cl.close()
