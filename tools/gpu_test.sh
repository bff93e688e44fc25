#!/bin/bash
# GPU box: the -m gpu suite (optionally a -k filter), one process.
#   bash tools/gpu_test.sh <outdir> [pytest -k expression]
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-test}
mkdir -p $out
export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$2" > $out/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
fi
