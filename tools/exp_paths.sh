#!/bin/bash
# GPU box: bench_paths.py for one path once per library variant in tools/_exp
# whose name starts with the given prefix (through CILIUM_AMD_LIB).
#   bash tools/exp_paths.sh <path> <prefix>
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/expp
for lib in tools/_exp/lib_$2*.so; do
  name=$(basename $lib .so)
  CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 tools/bench_paths.py --paths $1 --steps 10 --cpu-seconds 0 \
    > gpurun_out/expp/$name.log 2>&1 || exit $?
  echo "$name: $(tail -1 gpurun_out/expp/$name.log | cut -c1-160)"
done
