#!/bin/bash
# GPU box: ipcache parity tests, kernel throughput line, kernel trace, then
# the PMC passes (each counter group in its own rocprofv3 run).
#   bash tools/gpu_ipcache.sh <outdir> [pmc=0|1]
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-ipc}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_ipcache.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_paths.py --paths ipcache > $out/paths.jsonl 2> $out/paths.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_paths.py --paths ipcache --steps 3 --cpu-seconds 0 > $out/prof.log 2>&1 || exit $?
[ "${2:-0}" = "1" ] || exit 0
bash tools/gpu_pmc_paths.sh ${1:-ipc}_pmc ipcache
