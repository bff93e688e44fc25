#!/bin/bash
# GPU box: raw-path tests, bench.py without the CPU legs (headline +
# end-to-end objects), a kernel trace of the httpraw line.
#   bash tools/gpu_e2e.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-e2e}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $out/bench.log 2> $out/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/main -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/main.log 2>&1 || exit $?
