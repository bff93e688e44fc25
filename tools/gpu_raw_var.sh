#!/bin/bash
# GPU box: raw-path tests on the main library, then a kernel trace of the
# httpraw line for the main library and each tools/_exp/lib_<prefix>*.so;
# per-kernel mean durations in <out>/<name>_stats.csv.
#   bash tools/gpu_raw_var.sh <tag> <prefix>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-rawvar}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
cmd="python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/main -o run --output-format csv -- $cmd > $out/main.log 2>&1 || exit $?
for lib in tools/_exp/lib_${2:-rb_}*.so; do
  [ -f "$lib" ] || continue
  name=$(basename $lib .so)
  CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- $cmd > $out/$name.log 2>&1 || exit $?
done
# memory traffic of the main library's raw kernels (one counter group per pass)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pf -o run -- $cmd > $out/pf.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pw -o run -- $cmd > $out/pw.log 2>&1 || exit $?
