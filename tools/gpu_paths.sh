#!/bin/bash
# GPU box: L4 / prefilter / Kafka kernel throughput + kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-paths}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/bench_paths.py > $out/paths.jsonl 2> $out/paths.err || exit $?
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_paths.py --steps 3 --cpu-seconds 0.5 > $out/prof.log 2>&1 || exit $?
