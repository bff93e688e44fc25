#!/bin/bash
# GPU box: http_kernel at 4 waves/SIMD (tools/_exp/lib_h_pair_w4*.so,
# lib_h_w4_pre4.so: real kernel variants, checked by prof_http against the
# oracle sample) against the main library, interleaved, on the bench's
# 124.8M-request workload under a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05n}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 tools/prof_http.py --requests 124780544 --iters 10 --digest $out/digest.txt > $out/$name.log 2>&1
}
for r in 1 2; do
  run main$r CG_EXP_NOCHECK=0; rc=$?; echo "main$r rc=$rc" >> $out/rc.txt; fatal $rc
  for n in h_pair_w4 h_pair_w4_pre2 h_w4_pre4; do
    run ${n}_$r CG_EXP_NOCHECK=0 CILIUM_AMD_LIB=$PWD/tools/_exp/lib_$n.so; rc=$?; echo "${n}_$r rc=$rc" >> $out/rc.txt; fatal $rc
  done
done
