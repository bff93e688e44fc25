#!/bin/bash
# GPU box: the whole -m gpu suite, smoke, the bench line and its kernel trace.
#   bash tools/gpu_full.sh <outdir>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-full}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > $out/bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > $out/prof.log 2>&1 || exit $?
