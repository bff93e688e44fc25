#!/bin/bash
# GPU box, round 6: ring latency with the waiter spinning from the doorbell
# (default) and sleeping 6 / 9 us first (CILIUM_GPU_RING_SLEEP_US), ring only.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zg}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for us in 0 6 9; do
  CILIUM_GPU_RING_SLEEP_US=$us CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/latency_sleep$us.jsonl 2> $out/latency_sleep$us.err || exit $?
done
