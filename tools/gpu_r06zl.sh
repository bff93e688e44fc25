#!/bin/bash
# GPU box, round 6: ring tests, then the transport floor (echo modes) and the
# ring with relaxed polls (one acquire per served slot, one release).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zl}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_http_ring_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
bash tools/gpu_r06zj.sh $tag
