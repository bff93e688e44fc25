#!/bin/bash
# GPU box: the raw scan's phase clocks (tools/_exp/lib_raw_clocks.so) on the
# bench's end-to-end data and on bench_paths' httpraw data.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-e2eclk}
mkdir -p $out
export TMPDIR=/tmp
CILIUM_AMD_LIB=$PWD/tools/_exp/lib_raw_clocks.so timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-check --steps 3 --warmup 1 > $out/bench.log 2>&1 || exit $?
CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/tools/_exp/lib_raw_clocks.so timeout -k 10 300 python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/paths.log 2>&1 || exit $?
