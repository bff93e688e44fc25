#!/bin/bash
# GPU box: L4 parity tests on the in-tree library, then L4 variants.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/exp3
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "l4 or L4 or ipcache or smoke" > gpurun_out/exp3/pytest.log 2>&1 || exit $?
bash tools/exp_paths.sh l4 l4_ > gpurun_out/exp3/l4.txt 2>&1 || exit $?
