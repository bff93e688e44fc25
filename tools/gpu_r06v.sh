#!/bin/bash
# GPU box, round 6: ipcache with the exact /32 and /128 tables — the family
# split (tools/ipcache_split.py), then gpu_r06g.sh (ipcache / L4 GPU tests,
# the ipcache and L4 + ipcache path lines, the ipcache PMC passes).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06v}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/ipcache_split.py > $out/split.jsonl 2> $out/split.err || exit $?
bash tools/gpu_r06g.sh ${tag}_ipc || exit $?
