#!/bin/bash
# GPU box: time each HTTP kernel variant library (tools/exp_http.py) with
# prof_http.py under a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-exph}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for lib in tools/_exp/lib_*.so; do
  [ -e "$lib" ] || continue
  name=$(basename $lib .so)
  case $name in lib_kw_*) continue;; esac
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$name -o run -- python3 tools/prof_http.py --requests 64000000 --iters 4 > $out/$name.log 2>&1 || exit $?
done
