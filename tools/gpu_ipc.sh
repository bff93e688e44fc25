#!/bin/bash
# GPU box: ipcache tests (incl. the fused L4 path) and the ipcache / l4ipc bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-ipc}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_ipcache.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_paths.py --paths ipcache,l4ipc > $out/paths.jsonl 2> $out/paths.err || exit $?
