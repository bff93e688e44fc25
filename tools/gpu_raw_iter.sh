#!/bin/bash
# GPU box, one raw-path iteration: raw + header-list tests, the httpraw and
# httpfields bench lines, a kernel trace of the httpraw line.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-rawit}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/bench_paths.py --paths httpraw,httpfields --steps 3 --cpu-seconds 0 > $out/paths.jsonl 2> $out/paths.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/prof.log 2>&1 || exit $?
