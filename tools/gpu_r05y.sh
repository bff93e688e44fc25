#!/bin/bash
# GPU box: the device-layout scan's strings through per-lane LDS unit
# buffers (LdsUnitOut, main library) against TileOut<false>
# (tools/_exp/lib_emit_old.so): the raw-path GPU tests first, then the raw
# heads / header-list lines (checked against the host path) under a kernel
# trace, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05y}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_dl_gpu.py tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py tests/test_http_small_batches_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/rc.txt; fatal $rc
[ $rc = 0 ] || exit 1
cmd="python3 tools/bench_paths.py --paths httpraw,httpfields --steps 3 --cpu-seconds 0"
for r in 1 2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/new_$r -o run --output-format csv -- $cmd > $out/new_$r.log 2>&1
  rc=$?; echo "new_$r rc=$rc" >> $out/rc.txt; fatal $rc
  CILIUM_AMD_LIB=$PWD/tools/_exp/lib_emit_old.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/old_$r -o run --output-format csv -- $cmd > $out/old_$r.log 2>&1
  rc=$?; echo "old_$r rc=$rc" >> $out/rc.txt; fatal $rc
done
