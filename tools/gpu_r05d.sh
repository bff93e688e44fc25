#!/bin/bash
# GPU box: fresh PMC passes of the table-bound kernels (L4, Kafka split
# layout, ipcache, LPM) through bench_paths, each counter group in its own
# rocprofv3 run, summarized per kernel (tools/pmc_summary.py); then the
# bench_paths lines of the same kernels under a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05d}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
for path in l4 kafka ipcache lpm; do
  cmd="python3 tools/bench_paths.py --paths $path --steps 2 --cpu-seconds 0"
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    mkdir -p $out/$path
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $out/$path/p$i -o run -- $cmd > $out/$path/p$i.log 2>&1
    rc=$?; echo "$path p$i rc=$rc" >> $out/rc.txt; fatal $rc
  done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python3 tools/bench_paths.py --paths l4,kafka,ipcache,lpm,l4ipc --steps 5 --cpu-seconds 2 > $out/paths.jsonl 2> $out/paths.err
rc=$?; echo "paths rc=$rc" >> $out/rc.txt; fatal $rc
