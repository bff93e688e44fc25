#!/bin/bash
# GPU box: Envoy-shaped HTTP latency (tools/http_latency), then the
# http_kernel measuring variants (tools/_exp/lib_h_*.so) against the main
# library on the bench's 124.8M-request workload under a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05c}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
timeout -k 10 400 python3 tools/http_latency.py --seconds 0.5 > $out/latency.jsonl 2> $out/latency.err
rc=$?; echo "latency rc=$rc" > $out/rc.txt; fatal $rc
CILIUM_GPU_RAW_LAYOUT=device timeout -k 10 400 python3 tools/http_latency.py --seconds 0.5 > $out/latency_dev.jsonl 2> $out/latency_dev.err
rc=$?; echo "latency_dev rc=$rc" >> $out/rc.txt; fatal $rc
# the pair walker (a real kernel variant, not a measuring device): the HTTP
# parity tests through it before it is timed
CILIUM_AMD_LIB=$PWD/tools/_exp/lib_h_pair.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_rule_counters.py tests/test_http_raw_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_pair.log 2>&1
rc=$?; echo "pytest_pair rc=$rc" >> $out/rc.txt; fatal $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 tools/prof_http.py --requests 124780544 --iters 10 > $out/$name.log 2>&1
}
run main CG_EXP_NOCHECK=0; rc=$?; echo "main rc=$rc" >> $out/rc.txt; fatal $rc
for lib in tools/_exp/lib_h_*.so; do
  [ -f "$lib" ] || continue
  n=$(basename $lib .so)
  run $n CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/$lib; rc=$?; echo "$n rc=$rc" >> $out/rc.txt; fatal $rc
done
run main2 CG_EXP_NOCHECK=0; rc=$?; echo "main2 rc=$rc" >> $out/rc.txt; fatal $rc
