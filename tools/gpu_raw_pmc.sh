#!/bin/bash
# GPU box: raw-path tests, the httpraw line, one SQ PMC pass over the raw
# kernels (instruction mix, wave cycles, waits, LDS conflicts).
#   bash tools/gpu_raw_pmc.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-rawpmc}
mkdir -p $out
export TMPDIR=/tmp
cmd="python3 tools/bench_paths.py --paths httpraw --steps 2 --cpu-seconds 0"
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_paths.py --paths httpraw,httpfields --steps 5 --cpu-seconds 0 > $out/main.jsonl 2> $out/main.err || exit $?
for lib in tools/_exp/lib_${2:-raw_clocks}*.so; do
  [ -f "$lib" ] || continue
  CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 \
    > $out/$(basename $lib .so).log 2>&1 || exit $?
done
sq="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
timeout -s KILL 120 rocprofv3 --pmc $sq --output-format csv -d $out/p1 -o run -- $cmd > $out/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- $cmd > $out/prof.log 2>&1 || exit $?
