#!/bin/bash
# GPU box: where the headline kernel's non-walk time goes — measuring
# builds without per-rule hit counting (h_nohits), without the remote row
# lookup (h_norow) and without the DFA walk (h_nowalk) against the main
# library, prof_http's workload (half last units), kernel trace, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05ab}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 tools/prof_http.py --requests 124780544 --iters 10 > $out/$name.log 2>&1
}
for r in 1 2; do
  run main$r; rc=$?; echo "main$r rc=$rc" >> $out/rc.txt; fatal $rc
  for n in h_nohits h_norow h_nowalk; do
    run ${n}_$r CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/tools/_exp/lib_$n.so; rc=$?; echo "${n}_$r rc=$rc" >> $out/rc.txt; fatal $rc
  done
done
