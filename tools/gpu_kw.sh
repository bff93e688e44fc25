#!/bin/bash
# GPU box: Kafka wire tests, bench line + kernel trace.
#   bash tools/gpu_kw.sh <outdir> [noprof]
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-kw}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kafka_wire.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_paths.py --paths kafkawire > $out/paths.jsonl 2> $out/paths.err || exit $?
[ "$2" = "noprof" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_paths.py --paths kafkawire --steps 3 --cpu-seconds 0.5 > $out/prof.log 2>&1 || exit $?
