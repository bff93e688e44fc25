#!/bin/bash
# GPU box: the scan's window search over two 64-bit halves (main library)
# against the four-word select version (tools/_exp/lib_wn_old.so): the raw
# heads and header-list paths, checked against the host path, kernel trace,
# interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05x}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
cmd="python3 tools/bench_paths.py --paths httpraw,httpfields --steps 3 --cpu-seconds 0"
for r in 1 2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/new_$r -o run --output-format csv -- $cmd > $out/new_$r.log 2>&1
  rc=$?; echo "new_$r rc=$rc" >> $out/rc.txt; fatal $rc
  CILIUM_AMD_LIB=$PWD/tools/_exp/lib_wn_old.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/old_$r -o run --output-format csv -- $cmd > $out/old_$r.log 2>&1
  rc=$?; echo "old_$r rc=$rc" >> $out/rc.txt; fatal $rc
done
