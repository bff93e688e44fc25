#!/bin/bash
# GPU box, round 6: the ring's GPU tests and its latency entries at 1, 4, 8
# and 16 threads (64 workgroups), with the phase trace and without.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06q}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_http_ring_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 CILIUM_GPU_RING_TRACE=1 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/latency64.jsonl 2> $out/latency64.err || exit $?
CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/latency64_notrace.jsonl 2> $out/latency64_notrace.err || exit $?
