#!/bin/bash
# GPU box, round 6: ring calls through a per-thread cache of the handle, ring
# and snapshot (no lock, no shared reference count per call): the ring and
# fields GPU tests, then the latency driver twice.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zx}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_ring_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
for r in 1 2; do
  CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/ring_$r.jsonl 2> $out/ring_$r.err || exit $?
done
