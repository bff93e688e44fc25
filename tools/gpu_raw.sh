#!/bin/bash
# GPU box: bench lines for the raw HTTP/1 path, L4 and L4+ipcache, then a
# kernel trace of the raw path.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-raw}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/bench_paths.py --paths httpraw,l4,l4ipc > $out/paths.jsonl 2> $out/paths.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/prof.log 2>&1 || exit $?
