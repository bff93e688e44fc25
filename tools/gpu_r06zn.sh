#!/bin/bash
# GPU box, round 6: the headline with and without the time-based prewarm
# (bench.py --prewarm-seconds), interleaved on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zn}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
  for pw in 0 0.5; do
    timeout -k 10 300 python3 bench.py --no-e2e --no-cpu-baseline --no-check --small-distinct 0 --sustain-seconds 1 --prewarm-seconds $pw > $out/bench_pw${pw}_$r.json 2> $out/bench_pw${pw}_$r.err || exit $?
  done
done
