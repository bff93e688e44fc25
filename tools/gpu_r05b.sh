#!/bin/bash
# GPU box: the run_last tests (device-layout raw sequence incl. the late-slot
# and policy-swap cases, the OnData batching window), then the end-to-end raw
# path with the device layout (bench.py e2e object) and a kernel trace of the
# httpraw line on the device layout.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05b}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
timeout -k 10 300 python3 -u -m pytest tests -m "gpu and run_last" -v -s --timeout 120 --timeout-method thread > $out/pytest_last.log 2>&1
rc=$?; echo "pytest_last rc=$rc" > $out/rc.txt; fatal $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline --e2e-layout device > $out/bench_dev.log 2>&1
rc=$?; echo "bench_dev rc=$rc" >> $out/rc.txt; fatal $rc
export CILIUM_GPU_RAW_LAYOUT=device
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/raw_dev -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/raw_dev.log 2>&1
rc=$?; echo "raw_dev rc=$rc" >> $out/rc.txt; fatal $rc
