#!/bin/bash
# GPU box: raw-path tests, the httpraw line on the main library and on each
# experiment library tools/_exp/lib_<prefix>*.so, a kernel trace of the main one.
#   bash tools/gpu_raw_exp.sh <tag> <prefix>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-rawexp}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_paths.py --paths httpraw --steps 5 --cpu-seconds 0 > $out/main.jsonl 2> $out/main.err || exit $?
for lib in tools/_exp/lib_${2:-raw_}*.so; do
  name=$(basename $lib .so)
  CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 \
    > $out/$name.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/prof.log 2>&1 || exit $?
