#!/bin/bash
# GPU box: prefilter parity tests, then LPM traffic per family
# (tools/lpm_split.py) — FETCH / hit-miss passes and a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-lpmsplit}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k prefilter --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/lpm_split.py > $out/plain.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pf -o run -- python3 tools/lpm_split.py > $out/pf.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/ph -o run -- python3 tools/lpm_split.py > $out/ph.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 tools/lpm_split.py > $out/kt.log 2>&1 || exit $?
