#!/bin/bash
# GPU box: verdict bytes stored nontemporal (tools/_exp/lib_h_ntout.so)
# against the main library ("new"), the headline kernel on prof_http's
# workload, kernel trace, interleaved (verdict digests checked).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05af}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
run() {  # name, digest file, env...
  local name=$1 dg=$2; shift 2
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 tools/prof_http.py --requests 124780544 --iters 10 --digest $out/$dg > $out/$name.log 2>&1
}
for r in 1 2; do
  run new$r digest_new.txt; rc=$?; echo "new$r rc=$rc" >> $out/rc.txt; fatal $rc
  run ntout$r digest_nt.txt CILIUM_AMD_LIB=$PWD/tools/_exp/lib_h_ntout.so; rc=$?; echo "ntout$r rc=$rc" >> $out/rc.txt; fatal $rc
done
