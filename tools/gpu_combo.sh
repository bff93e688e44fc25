#!/bin/bash
# GPU box: raw-path tests and bench line, then PMC passes (HTTP, L4, Kafka)
# and the prefilter ILP variants.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-combo}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_http_raw_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest_raw.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_paths.py --paths httpraw > $out/raw.jsonl 2> $out/raw.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/rawprof -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/rawprof.log 2>&1 || exit $?
bash tools/gpu_pmc_all.sh $tag || exit $?
