#!/bin/bash
# GPU box, round 6: the ring with its phase trace (CILIUM_GPU_RING_TRACE=1:
# mean device time per phase of a batch, printed at close), then
# gpu_r06g.sh on the re-encoded ipcache chunks (16-byte round-1 pairs,
# 56-key map words).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06i}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 180 python3 -u -m pytest tests/test_http_ring_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
CILIUM_GPU_RING_TRACE=1 CILIUM_GPU_DEBUG=1 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/latency.jsonl 2> $out/latency.err || exit $?
bash tools/gpu_r06g.sh ${2:-r06i_ipc} || exit $?
