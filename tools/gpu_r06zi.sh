#!/bin/bash
# GPU box, round 6: the device-layout scan's phase clocks (raw_clocks
# experiment build, one wave's shader-clock totals per launch) on the
# raw-heads path.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zi}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/tools/_exp/lib_raw_clocks.so timeout -k 10 300 python3 tools/bench_paths.py --paths httpraw --steps 1 --cpu-seconds 0 > $out/clocks.log 2>&1 || exit $?
