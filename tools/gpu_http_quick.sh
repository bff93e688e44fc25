#!/bin/bash
# GPU box: HTTP GPU tests (-k http or rule) then bench.py with kernel trace.
#   bash tools/gpu_http_quick.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-hq}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "http or rule or config" > $out/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --cpu-seconds 3 > $out/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > $out/prof.log 2>&1 || exit $?
