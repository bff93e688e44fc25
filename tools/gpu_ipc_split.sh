#!/bin/bash
# GPU box: ipcache per family (tools/ipc_split.py) for the main library and
# each tools/_exp/lib_<prefix>*.so, then FETCH / hit-miss passes (main).
#   bash tools/gpu_ipc_split.sh <tag> <prefix>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-ipcsplit}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/ipc_split.py > $out/main.log 2>&1 || exit $?
for lib in tools/_exp/lib_${2:-ipc_}*.so; do
  [ -f "$lib" ] || continue
  name=$(basename $lib .so)
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 tools/ipc_split.py > $out/$name.log 2>&1 || exit $?
done
timeout -k 10 300 python3 tools/ipc_split.py > $out/main2.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pf -o run -- python3 tools/ipc_split.py > $out/pf.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/ph -o run -- python3 tools/ipc_split.py > $out/ph.log 2>&1 || exit $?
