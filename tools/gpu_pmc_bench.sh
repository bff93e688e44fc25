#!/bin/bash
# GPU box: PMC passes over the HTTP kernel (tools/gpu_pmc.sh), then a bench
# line and its kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-pmcb}
bash tools/gpu_pmc.sh $tag || exit $?
out=gpurun_out/$tag
timeout -k 10 400 python3 bench.py > $out/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > $out/prof.log 2>&1 || exit $?
