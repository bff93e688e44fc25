#!/bin/bash
# GPU box: time every variant built by tools/exp_http.py (one process each).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/exp
for lib in tools/_exp/lib_*.so; do
  name=$(basename $lib .so)
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 tools/prof_http.py --requests ${1:-64000000} --iters 5 \
    > gpurun_out/exp/$name.log 2>&1 || exit $?
  echo "$name: $(tail -1 gpurun_out/exp/$name.log)"
done
