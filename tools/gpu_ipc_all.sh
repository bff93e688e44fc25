#!/bin/bash
# GPU box: ipcache GPU tests, per-family split for the main library and the
# ipc_ variants, bench lines, PMC passes of the bench ipcache line.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-ipcall}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_ipcache.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
bash tools/gpu_ipc_split.sh $tag/split ipc_ || exit $?
timeout -k 10 600 python3 tools/bench_paths.py --paths ipcache,l4ipc --cpu-seconds 0 > $out/paths.jsonl 2> $out/paths.err || exit $?
bash tools/gpu_pmc_paths.sh $tag/pmc ipcache || exit $?
