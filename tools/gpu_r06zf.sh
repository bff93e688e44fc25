#!/bin/bash
# GPU box, round 6: Kafka wire decode with the pool in its drawn order and
# grouped by (apiKey, version) — the lane-divergence A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zf}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_paths.py --paths kafkawire --steps 5 --cpu-seconds 0.2 > $out/paths_drawn.jsonl 2> $out/paths_drawn.err || exit $?
CILIUM_BENCH_KAFKA_SORTED=1 timeout -k 10 300 python3 tools/bench_paths.py --paths kafkawire --steps 5 --cpu-seconds 0.2 > $out/paths_sorted.jsonl 2> $out/paths_sorted.err || exit $?
