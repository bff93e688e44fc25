#!/bin/bash
# GPU box: what the raw path's verdict scatter (out[order[slot]], one byte
# per request at its request index) costs: a measuring build writing the
# verdict over its own order entry instead (h_noscatter; verdicts not
# delivered) against the main library, raw heads line (no check), kernel
# trace, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05ad}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
cmd="python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0"
for r in 1 2; do
  CG_EXP_NOCHECK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/main_$r -o run --output-format csv -- $cmd > $out/main_$r.log 2>&1
  rc=$?; echo "main_$r rc=$rc" >> $out/rc.txt; fatal $rc
  CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/tools/_exp/lib_h_noscatter.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/nosc_$r -o run --output-format csv -- $cmd > $out/nosc_$r.log 2>&1
  rc=$?; echo "nosc_$r rc=$rc" >> $out/rc.txt; fatal $rc
done
