#!/bin/bash
# GPU box: the device-layout scan at 3 (default), 2 and 1 workgroups per CU
# (CILIUM_GPU_RAW_SCAN_WG), raw heads line checked against the host path,
# kernel trace, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05z}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
cmd="python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0"
for r in 1 2; do
  for wg in 3 2 1; do
    CILIUM_GPU_RAW_SCAN_WG=$wg timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/wg${wg}_$r -o run --output-format csv -- $cmd > $out/wg${wg}_$r.log 2>&1
    rc=$?; echo "wg${wg}_$r rc=$rc" >> $out/rc.txt; fatal $rc
  done
done
