#!/bin/bash
# GPU box: LPM per family (tools/lpm_split.py) for the main library and each
# tools/_exp/lib_lpm_*.so, main run first and last.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-lpmvar}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/lpm_split.py > $out/main.log 2>&1 || exit $?
for lib in tools/_exp/lib_lpm_*.so; do
  [ -f "$lib" ] || continue
  name=$(basename $lib .so)
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 tools/lpm_split.py > $out/$name.log 2>&1 || exit $?
done
timeout -k 10 300 python3 tools/lpm_split.py > $out/main2.log 2>&1 || exit $?
