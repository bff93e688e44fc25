#!/bin/bash
# GPU box: the whole -m gpu suite (run_last included), then the raw path on
# both layouts under a kernel trace, the headline kernel's trace on the
# prof_http workload, and the Envoy-batch latency driver.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05g}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/rc.txt; fatal $rc
CILIUM_GPU_RAW_LAYOUT=device timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/dl -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw,httpfields --steps 3 --cpu-seconds 0 > $out/dl.log 2>&1
rc=$?; echo "dl rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/head -o run --output-format csv -- python3 tools/prof_http.py --requests 124780544 --iters 10 > $out/head.log 2>&1
rc=$?; echo "head rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 400 python3 tools/http_latency.py --seconds 0.5 > $out/latency.jsonl 2> $out/latency.err
rc=$?; echo "latency rc=$rc" >> $out/rc.txt; fatal $rc
