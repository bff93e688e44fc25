#!/bin/bash
# GPU box: bench_paths.py lines for the given paths (one process).
#   bash tools/gpu_paths2.sh <tag> <paths>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-paths}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/bench_paths.py --paths $2 > $out/paths.jsonl 2> $out/paths.err || exit $?
