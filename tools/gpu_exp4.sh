#!/bin/bash
# GPU box: raw HTTP/1 path tests, then L4 variants.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/exp4
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_http_raw_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/exp4/pytest_raw.log 2>&1 || exit $?
bash tools/exp_paths.sh l4 l4_ > gpurun_out/exp4/l4.txt 2>&1 || exit $?
