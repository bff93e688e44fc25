#!/bin/bash
# GPU box, round 6: the ring after its staged program record left scratch
# (no flat load per call) and its whole-quad walk steps lost their guards:
# the ring and raw-path GPU tests, then the latency driver and a phase trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zr}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_ring_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
lat() {  # name, env...
  local name=$1; shift
  env "$@" CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/$name.jsonl 2> $out/$name.err
  local rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
}
lat ring_1 CILIUM_GPU_DEBUG=1
lat ring_trace CILIUM_GPU_RING_TRACE=1
lat ring_2 A=1
exit 0
