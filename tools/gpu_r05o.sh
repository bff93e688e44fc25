#!/bin/bash
# GPU box: the device-layout scan's occupancy experiments — the main library
# against 512-thread scan workgroups with 5 KiB stages (rawdl_t512_s5k) and
# 5 KiB stages alone (rawdl_s5k), each checked against the host path, under
# a kernel trace (interleaved), plus the phase-clock build (raw_clocks).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05o}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
cmd="python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0"
run() {  # name, env...
  local name=$1; shift
  env CILIUM_GPU_DEBUG=1 "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- $cmd > $out/$name.log 2>&1
}
for r in 1 2; do
  run main$r; rc=$?; echo "main$r rc=$rc" >> $out/rc.txt; fatal $rc
  for n in rawdl_t512_s5k rawdl_s5k; do
    run ${n}_$r CILIUM_AMD_LIB=$PWD/tools/_exp/lib_$n.so; rc=$?; echo "${n}_$r rc=$rc" >> $out/rc.txt; fatal $rc
  done
done
CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/tools/_exp/lib_raw_clocks.so timeout -k 10 300 $cmd > $out/clocks.log 2>&1
rc=$?; echo "clocks rc=$rc" >> $out/rc.txt; fatal $rc
