#!/bin/bash
# First GPU session: parity tests, smoke, short bench + rocprofv3 kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
(command -v go && go version) > gpurun_out/go_probe.txt 2>&1 || echo "go: not found" >> gpurun_out/go_probe.txt
nproc > gpurun_out/host.txt; grep -m1 "model name" /proc/cpuinfo >> gpurun_out/host.txt
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --requests-per-gpu 16000000 --cpu-seconds 5 > gpurun_out/bench_16m.log 2>&1 || exit $?
exit $rc
