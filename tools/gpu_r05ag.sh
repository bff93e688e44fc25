#!/bin/bash
# GPU box: issue-side PMC of the headline kernel (bench.py's headline
# workload only, as tools/gpu_headline_prof.sh runs it): VALU / LDS / SALU
# instruction counts, wave cycles and waits, LDS bank conflicts, one counter
# group per rocprofv3 pass (no trace domains).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05ag}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
cmd="python3 bench.py --no-e2e --small-distinct 0 --no-cpu-baseline --no-check --steps 3 --warmup 0"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- $cmd > $out/p$i.log 2>&1
  rc=$?; echo "p$i rc=$rc" >> $out/rc.txt; fatal $rc
done
