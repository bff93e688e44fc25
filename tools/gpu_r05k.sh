#!/bin/bash
# GPU box: PMC passes (FETCH_SIZE, WRITE_SIZE, an SQ group) over the raw-heads
# line on the device layout (the default), each group in its own rocprofv3
# run, summarized per kernel by tools/pmc_summary.py afterwards.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05k}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
: > $out/rc.txt
cmd="python3 tools/bench_paths.py --paths httpraw --steps 2 --cpu-seconds 0"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- $cmd > $out/p$i.log 2>&1
  rc=$?; echo "p$i rc=$rc" >> $out/rc.txt
  case $rc in 124|134|137|139) exit $rc;; esac
done
