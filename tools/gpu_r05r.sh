#!/bin/bash
# GPU box: issue-side PMC of the device-layout raw sequence (config 5 heads):
# VALU / SALU / LDS / VMEM instruction counts and active cycles per kernel,
# each counter group in its own pass; counter names checked against
# rocprofv3 -L first (a group with an unknown name is skipped).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05r}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 120 rocprofv3 -L > $out/counters.txt 2>&1
rc=$?; echo "list rc=$rc" >> $out/rc.txt; fatal $rc
cmd="python3 tools/bench_paths.py --paths httpraw --steps 2 --cpu-seconds 0"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  ok=1
  for c in $grp; do grep -q "\b$c\b" $out/counters.txt || { echo "pass $i: no $c" >> $out/rc.txt; ok=0; }; done
  [ $ok = 1 ] || grp=$(for c in $grp; do grep -q "\b$c\b" $out/counters.txt && echo -n "$c "; done)
  [ -n "$grp" ] || continue
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- $cmd > $out/p$i.log 2>&1
  rc=$?; echo "p$i rc=$rc ($grp)" >> $out/rc.txt; fatal $rc
done
