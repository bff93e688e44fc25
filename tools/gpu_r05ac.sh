#!/bin/bash
# GPU box: meta words carrying the remote-identity row in cg_http_pack's
# tiles of one-part LDS programs (kTileRowMeta, main library) against half
# last units alone (tools/_exp/lib_h_half.so): the HTTP GPU tests first,
# then the headline kernel on prof_http's workload, kernel trace,
# interleaved (each library's verdict digest checked across its runs).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05ac}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_rule_counters.py tests/test_tile_forms.py tests/test_http_raw_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/rc.txt; fatal $rc
[ $rc = 0 ] || exit 1
run() {  # name, digest file, env...
  local name=$1 dg=$2; shift 2
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 tools/prof_http.py --requests 124780544 --iters 10 --digest $out/$dg > $out/$name.log 2>&1
}
for r in 1 2; do
  run new$r digest_new.txt; rc=$?; echo "new$r rc=$rc" >> $out/rc.txt; fatal $rc
  run half$r digest_half.txt CILIUM_AMD_LIB=$PWD/tools/_exp/lib_h_half.so; rc=$?; echo "half$r rc=$rc" >> $out/rc.txt; fatal $rc
done
