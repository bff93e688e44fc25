#!/bin/bash
# GPU box: the host entry (header lists in host memory → verdicts, PCIe
# included; bench_paths httpfields' host_entry) at staging chunks of 160
# (default), 64, 32 and 16 MiB (CILIUM_GPU_HOST_CHUNK_MB), interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05aa}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
for r in 1 2; do
  for mb in 160 64 32 16; do
    CILIUM_GPU_HOST_CHUNK_MB=$mb timeout -k 10 400 python3 tools/bench_paths.py --paths httpfields --steps 3 --cpu-seconds 0 > $out/c${mb}_$r.log 2>&1
    rc=$?; echo "c${mb}_$r rc=$rc" >> $out/rc.txt; fatal $rc
  done
done
