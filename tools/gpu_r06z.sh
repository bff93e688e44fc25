#!/bin/bash
# GPU box, round 6: the list scans parse over register mask windows — the
# fields / raw / codec GPU tests, then the header-list and raw-head path
# lines.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06z}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_fields_gpu.py tests/test_http_raw_dl_gpu.py tests/test_http_raw_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_paths.py --paths httpfields,httpraw,httpfields --steps 5 --cpu-seconds 1 > $out/paths.jsonl 2> $out/paths.err || exit $?
