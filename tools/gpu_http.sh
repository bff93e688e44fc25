#!/bin/bash
# GPU box: HTTP + raw-path GPU tests, bench.py (default args), a kernel
# trace of a short bench run, the httpraw/httpfields lines.
#   bash tools/gpu_http.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-http}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py tests/test_rule_counters.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $out/bench.log 2> $out/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check > $out/prof.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_paths.py --paths httpraw,httpfields --steps 5 --cpu-seconds 0 > $out/paths.jsonl 2> $out/paths.err || exit $?
