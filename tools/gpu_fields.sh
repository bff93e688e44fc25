#!/bin/bash
# GPU box: raw-path and header-list tests, then bench.py (default args) and
# a raw + lists kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-fields}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py > $out/bench.log 2> $out/bench.err || exit $?
timeout -k 10 400 python3 tools/bench_paths.py --paths httpfields,httpraw > $out/paths.jsonl 2> $out/paths.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/prof.log 2>&1 || exit $?
