#!/bin/bash
# GPU box: bench.py with the tile-major and copy-major replicated layouts.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-layout}
mkdir -p $out
for l in tile copy tile; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --layout $l > $out/bench_$l.log 2>&1 || exit $?
  echo "$l: $(tail -1 $out/bench_$l.log | cut -c1-200)" >> $out/summary.txt
done
