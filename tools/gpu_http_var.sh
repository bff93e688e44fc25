#!/bin/bash
# GPU box: the bench's HTTP workload (tools/prof_http.py, 124.8M requests)
# and the httpraw line under a kernel trace, for the main library and each
# tools/_exp/lib_<prefix>*.so.
#   bash tools/gpu_http_var.sh <tag> <prefix>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-httpvar}
mkdir -p $out
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name/h -o run --output-format csv -- python3 tools/prof_http.py --requests 124780544 --iters 10 > $out/$name.h.log 2>&1 || return $?
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name/r -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/$name.r.log 2>&1 || return $?
}
run main CG_EXP_NOCHECK=0 || exit $?
for lib in tools/_exp/lib_${2:-h_}*.so; do
  [ -f "$lib" ] || continue
  run $(basename $lib .so) CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/$lib || exit $?
done
