#!/bin/bash
# GPU session: HTTP parity tests + bench (+ optional rocprofv3 kernel trace).
# usage: tools/gpu_bench.sh <tag> [requests_per_gpu] [prof]
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-run}; req=${2:-125000000}; prof=${3:-0}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --requests-per-gpu $req --cpu-seconds 10 > gpurun_out/bench_$tag.log 2>&1 || exit $?
if [ "$prof" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --requests-per-gpu $req --no-cpu-baseline --no-check > gpurun_out/prof_$tag.log 2>&1 || exit $?
fi
exit $rc
