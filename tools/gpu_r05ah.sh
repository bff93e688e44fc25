#!/bin/bash
# GPU box: the mixed-entry concurrency test (tests/test_gpu_mixed_concurrency.py)
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05ah}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mixed_concurrency.py -m gpu -v --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
echo "pytest rc=$?" > $out/rc.txt
