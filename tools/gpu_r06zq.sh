#!/bin/bash
# GPU box, round 6: the ring with its request slots in fine-grained device
# memory written by the host (the new default) against pinned host slots
# (CILIUM_GPU_RING_SLOTS=host): the ring GPU tests (both placements), then
# the latency driver per placement, the transport floor (echo 1) of each,
# and a phase trace of the new default.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zq}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_http_ring_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
lat() {  # name, env...
  local name=$1; shift
  env "$@" CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/$name.jsonl 2> $out/$name.err
  local rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
}
lat dev_1 CILIUM_GPU_DEBUG=1
lat host_1 CILIUM_GPU_RING_SLOTS=host
lat dev_echo1 CILIUM_GPU_RING_ECHO=1
lat host_echo1 CILIUM_GPU_RING_SLOTS=host CILIUM_GPU_RING_ECHO=1
lat dev_2 A=1
lat host_2 CILIUM_GPU_RING_SLOTS=host
lat dev_trace CILIUM_GPU_RING_TRACE=1
exit 0
