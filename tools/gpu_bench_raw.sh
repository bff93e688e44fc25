#!/bin/bash
# GPU box: raw-path tests, bench.py (default args: 8M distinct, 262K line,
# end-to-end raw line, CPU baseline), raw kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-braw}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_http_raw_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py > $out/bench.log 2> $out/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/prof.log 2>&1 || exit $?
