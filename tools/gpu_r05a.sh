#!/bin/bash
# GPU box, round 5 first call: the verified -m gpu suite (run_last excluded),
# then the device-layout raw sequence's tests on their own (first GPU run),
# then the OnData C-thread bench.  A timeout, abort or crash ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05a}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests -m "gpu and not run_last" -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $out/rc.txt; fatal $rc
timeout -k 10 300 python3 -u -m pytest tests/test_http_raw_dl_gpu.py -x -v -s --timeout 120 --timeout-method thread > $out/pytest_dl.log 2>&1
rc=$?; echo "pytest_dl rc=$rc" >> $out/rc.txt; fatal $rc
CILIUM_GPU_DEVICE=0 timeout -k 10 300 tools/ondata_bench ${2:-2000} 16 > $out/ondata.jsonl 2> $out/ondata.err
rc=$?; echo "ondata rc=$rc" >> $out/rc.txt; fatal $rc
