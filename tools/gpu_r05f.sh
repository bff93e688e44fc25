#!/bin/bash
# GPU box: the Kafka decoder with compressed payloads decoded on the device
# (GPU tests), then the device-layout raw path against its measuring
# variants (tools/_exp/lib_rawdl_*.so) under a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05f}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kafka_wire.py -m gpu -v -s --timeout 120 --timeout-method thread > $out/pytest_kafka.log 2>&1
rc=$?; echo "pytest_kafka rc=$rc" >> $out/rc.txt; fatal $rc
run() {  # name, env...
  local name=$1; shift
  env CILIUM_GPU_RAW_LAYOUT=device "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/$name.log 2>&1
}
run main; rc=$?; echo "main rc=$rc" >> $out/rc.txt; fatal $rc
for lib in tools/_exp/lib_rawdl_*.so; do
  n=$(basename $lib .so)
  run $n CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/$lib; rc=$?; echo "$n rc=$rc" >> $out/rc.txt; fatal $rc
done
