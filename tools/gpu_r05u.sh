#!/bin/bash
# GPU box: compact 4-byte meta words (main library, "CGH5" batches) against
# half last units alone (tools/_exp/lib_h_half.so, "CGH4"), interleaved on
# the same box: the headline kernel on prof_http's workload and the raw
# heads path (bench_paths httpraw, checked against the host path).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05u}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
run() {  # name, cmd-kind, env...
  local name=$1 kind=$2; shift 2
  if [ $kind = h ]; then cmd="python3 tools/prof_http.py --requests 124780544 --iters 10"
  else cmd="python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0"; fi
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- $cmd > $out/$name.log 2>&1
}
for r in 1 2; do
  for k in h r; do
    run new_$k$r $k; rc=$?; echo "new_$k$r rc=$rc" >> $out/rc.txt; fatal $rc
    run half_$k$r $k CILIUM_AMD_LIB=$PWD/tools/_exp/lib_h_half.so; rc=$?; echo "half_$k$r rc=$rc" >> $out/rc.txt; fatal $rc
  done
done
