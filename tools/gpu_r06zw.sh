#!/bin/bash
# GPU box, round 6: the ring's phase trace of single-request calls from one
# thread alone (the mixed-thread trace averages in the calls of 16 threads,
# whose spills to other workgroups restage programs).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zw}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
CILIUM_LAT_ONLY=1:1 CILIUM_GPU_RING_TRACE=1 CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 timeout -k 10 300 python3 tools/http_latency.py --seconds 2 --entries ring > $out/trace_1x1.jsonl 2> $out/trace_1x1.err || exit $?
CILIUM_LAT_ONLY=1:16 CILIUM_GPU_RING_TRACE=1 CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 timeout -k 10 300 python3 tools/http_latency.py --seconds 2 --entries ring > $out/trace_1x16.jsonl 2> $out/trace_1x16.err || exit $?
