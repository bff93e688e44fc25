#!/bin/bash
# GPU box: A/B of bench_paths lines between the main library and
# tools/_exp/lib_<variant>.so, alternated twice on the same box.
#   bash tools/gpu_ab_paths.sh <tag> <variant> <paths>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-ab}
mkdir -p $out
export TMPDIR=/tmp
lib=$PWD/tools/_exp/lib_$2.so
[ -f "$lib" ] || exit 3
cmd="python3 tools/bench_paths.py --paths $3 --steps 5 --cpu-seconds 0"
for r in 1 2; do
  timeout -k 10 300 $cmd > $out/main_$r.jsonl 2> $out/main_$r.err || exit $?
  CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$lib timeout -k 10 300 $cmd > $out/$2_$r.jsonl 2> $out/$2_$r.err || exit $?
done
