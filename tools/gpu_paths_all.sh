#!/bin/bash
# GPU box: every bench_paths line (one JSON line each) and a kernel trace of them.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-pathsall}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/bench_paths.py --paths l4,lpm,kafka,ipcache,proxylib,l4ipc,kafkawire,httpraw,httpfields > $out/paths.jsonl 2> $out/paths.err || exit $?
