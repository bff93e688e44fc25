#!/bin/bash
# GPU box: HTTP kernel variants (tools/_exp/lib_h_*.so) through bench.py.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/exph
export TMPDIR=/tmp
for lib in tools/_exp/lib_h_*.so; do
  name=$(basename $lib .so)
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check --steps 50 \
    > gpurun_out/exph/$name.log 2>&1 || exit $?
  echo "$name: $(tail -1 gpurun_out/exph/$name.log | cut -c1-140)"
done
