#!/bin/bash
# GPU box: the Kafka verdict kernel at 2 / 4 (main) / 8 requests per lane
# (tools/_exp/lib_kv_r2.so, lib_kv_r8.so), bench_paths kafka (checked
# against the oracle), interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05ae}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
cmd="python3 tools/bench_paths.py --paths kafka --steps 5 --cpu-seconds 0"
for r in 1 2; do
  timeout -k 10 300 $cmd > $out/main_$r.log 2>&1; rc=$?; echo "main_$r rc=$rc" >> $out/rc.txt; fatal $rc
  for v in kv_r2 kv_r8; do
    CILIUM_AMD_LIB=$PWD/tools/_exp/lib_$v.so timeout -k 10 300 $cmd > $out/${v}_$r.log 2>&1; rc=$?; echo "${v}_$r rc=$rc" >> $out/rc.txt; fatal $rc
  done
done
