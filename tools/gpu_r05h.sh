#!/bin/bash
# GPU box: the device-layout raw path (raw-byte tiles coded in http_kernel)
# tests, then the raw path on both layouts under a kernel trace, then the
# Envoy-batch latency driver and the small-call tests.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05h}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 400 python3 -u -m pytest tests/test_http_raw_dl_gpu.py tests/test_http_small_batches_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/rc.txt; fatal $rc
[ $rc -eq 0 ] || exit 1
CILIUM_GPU_RAW_LAYOUT=device timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/dl -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw,httpfields --steps 3 --cpu-seconds 0 > $out/dl.log 2>&1
rc=$?; echo "dl rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 400 python3 tools/http_latency.py --seconds 0.5 > $out/latency.jsonl 2> $out/latency.err
rc=$?; echo "latency rc=$rc" >> $out/rc.txt; fatal $rc
