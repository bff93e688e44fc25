#!/bin/bash
# GPU box: the device-layout raw path with striped slot counters — its GPU
# tests, then the httpraw line under a kernel trace at 1 / 16 / 64 stripes
# (CILIUM_GPU_RAW_STRIPES) and the default sequence for reference.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05e}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 300 python3 -u -m pytest tests/test_http_raw_dl_gpu.py -x -v --timeout 120 --timeout-method thread > $out/pytest_dl.log 2>&1
rc=$?; echo "pytest_dl rc=$rc" >> $out/rc.txt; fatal $rc
[ $rc -eq 0 ] || exit 1
for S in 16 64 1; do
  CILIUM_GPU_RAW_LAYOUT=device CILIUM_GPU_RAW_STRIPES=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/dl_s$S -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/dl_s$S.log 2>&1
  rc=$?; echo "dl_s$S rc=$rc" >> $out/rc.txt; fatal $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/host -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/host.log 2>&1
rc=$?; echo "host rc=$rc" >> $out/rc.txt; fatal $rc
