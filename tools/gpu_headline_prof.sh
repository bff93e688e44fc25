#!/bin/bash
# The bench headline's kernel alone: a rocprofv3 kernel trace of exactly the
# headline launches (no oracle check, no 262K / end-to-end / CPU legs), then
# FETCH_SIZE and WRITE_SIZE PMC passes of the same command, summarized per
# request of the headline layout (profiles/<tag>_http_pmc.json is what
# bench.py's roofline.traffic reads).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r04_headline}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
B=${B:-125829120}   # requests per launch: 15 copies of 8,388,608 distinct
cmd="python3 bench.py --no-e2e --small-distinct 0 --no-cpu-baseline --no-check"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- $cmd --steps 20 --warmup 3 > $out/kt.log 2>&1 || exit $?
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- $cmd --steps 3 --warmup 0 > $out/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $out --items $B --workload "$cmd (8,388,608 distinct x 15 = $B requests per launch)" --out $out/http_pmc.json > $out/summary.log 2>&1
