#!/bin/bash
# GPU box, round 6: the ring with the mask-based list parse and the LDS
# string walk — its GPU tests, then the latency entries with the phase
# trace at 16 and 64 workgroups.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06k}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_http_ring_gpu.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
CILIUM_GPU_RING_TRACE=1 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/latency.jsonl 2> $out/latency.err || exit $?
CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 CILIUM_GPU_RING_TRACE=1 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/latency64.jsonl 2> $out/latency64.err || exit $?
