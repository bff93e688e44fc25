#!/bin/bash
# GPU box: the fixed header-list device test, then the headline kernel
# against its s_setprio variant (tools/_exp/lib_h_prio.so) on the prof_http
# workload, twice each, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05l}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 300 python3 -u -m pytest tests/test_http_fields_gpu.py -m gpu -v -k dev_tensors --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/rc.txt; fatal $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 tools/prof_http.py --requests 124780544 --iters 10 > $out/$name.log 2>&1
}
for k in 1 2; do
  run main$k; rc=$?; echo "main$k rc=$rc" >> $out/rc.txt; fatal $rc
  run prio$k CILIUM_AMD_LIB=$PWD/tools/_exp/lib_h_prio.so; rc=$?; echo "prio$k rc=$rc" >> $out/rc.txt; fatal $rc
done
