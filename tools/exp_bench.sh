#!/bin/bash
# GPU box: bench.py (BASELINE config 5 layout) once per kernel variant built by
# tools/exp_http.py, through CILIUM_AMD_LIB.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/expb
for lib in tools/_exp/lib_*.so; do
  name=$(basename $lib .so)
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check --steps 20 \
    > gpurun_out/expb/$name.log 2>&1 || exit $?
  echo "$name: $(tail -1 gpurun_out/expb/$name.log | cut -c1-140)"
done
