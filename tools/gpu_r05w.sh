#!/bin/bash
# GPU box: the device-layout raw path at sub-batches of 2^25 (default),
# 2^26 and 2^27 requests (CILIUM_GPU_RAW_SUBBATCH), interleaved, each
# checked against the host path, under a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05w}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
cmd="python3 tools/bench_paths.py --paths httpraw,httpfields --steps 3 --cpu-seconds 0"
for r in 1 2; do
  for sb in 8388608 16777216 33554432; do
    CILIUM_GPU_RAW_SUBBATCH=$sb timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/s${sb}_$r -o run --output-format csv -- $cmd > $out/s${sb}_$r.log 2>&1
    rc=$?; echo "s${sb}_$r rc=$rc" >> $out/rc.txt; fatal $rc
  done
done
