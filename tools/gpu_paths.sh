#!/bin/bash
# GPU box: L4 / prefilter / Kafka parity tests, kernel throughput + kernel trace.
#   bash tools/gpu_paths.sh <outdir> [paths=l4,lpm,kafka] [pytest -k expr]
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-paths}
paths=${2:-l4,lpm,kafka}
mkdir -p $out
export TMPDIR=/tmp
if [ -n "$3" ]; then
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -k "$3" > $out/pytest.log 2>&1 || exit $?
fi
timeout -k 10 900 python3 tools/bench_paths.py --paths $paths > $out/paths.jsonl 2> $out/paths.err || exit $?
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_paths.py --paths $paths --steps 3 --cpu-seconds 0.5 > $out/prof.log 2>&1 || exit $?
