#!/bin/bash
# GPU box: the device-layout raw path at 4 / 8 / 16 slot-counter stripes:
# the httpraw line under a kernel trace, then a WRITE_SIZE pass of each.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05m}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
cmd="python3 tools/bench_paths.py --paths httpraw --steps 2 --cpu-seconds 0"
for S in 4 8 16; do
  CILIUM_GPU_RAW_STRIPES=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt_s$S -o run --output-format csv -- $cmd > $out/kt_s$S.log 2>&1
  rc=$?; echo "kt_s$S rc=$rc" >> $out/rc.txt; fatal $rc
  CILIUM_GPU_RAW_STRIPES=$S timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/w_s$S -o run -- $cmd > $out/w_s$S.log 2>&1
  rc=$?; echo "w_s$S rc=$rc" >> $out/rc.txt; fatal $rc
done
