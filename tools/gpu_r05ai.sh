#!/bin/bash
# GPU box: the policy swaps racing verdict calls
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05ai}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_policy_swap_concurrency.py -m gpu -v --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
echo "pytest rc=$?" > $out/rc.txt
