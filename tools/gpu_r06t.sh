#!/bin/bash
# GPU box, round 6: the Kafka wire GPU tests and path lines with fixed-code
# DEFLATE blocks decoded arithmetically (kw_inflate.h codes_fixed).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06t}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kafka_wire.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python3 tools/bench_paths.py --paths kafkawire,kafkawirez --steps 5 --cpu-seconds 2 > $out/paths.jsonl 2> $out/paths.err || exit $?
