#!/bin/bash
# GPU box, round 6: ipcache_kernel split by family, encoded vs all-dense v4
# chunks (tools/ipcache_split.py), then the Kafka wire lines with the
# inflate kernel at two workgroups per CU.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06j}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/ipcache_split.py > $out/split.jsonl 2> $out/split.err || exit $?
timeout -k 10 300 python3 tools/ipcache_split.py --dense >> $out/split.jsonl 2>> $out/split.err || exit $?
timeout -k 10 500 python3 tools/bench_paths.py --paths kafkawire,kafkawirez --steps 5 --cpu-seconds 2 > $out/paths.jsonl 2> $out/paths.err || exit $?
