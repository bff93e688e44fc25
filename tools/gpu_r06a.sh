#!/bin/bash
# GPU box, round 6: the codec-step change (bare LF, method table, HTTP/1.1,
# Host, Content-Length, strict target) — codec KATs and every raw-path GPU
# test, then the raw / list path lines under a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06a}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_codec_gpu.py tests/test_http_raw_gpu.py tests/test_http_raw_dl_gpu.py tests/test_http_parse.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/paths -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw,httpfields --steps 3 --cpu-seconds 1 > $out/paths.jsonl 2> $out/paths.err || exit $?
