#!/bin/bash
# GPU box: raw-path A/B (structural-bitmap vs dword-step parsing in the scan)
# and one SQ PMC pass per variant over the raw kernels.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-rawab}
mkdir -p $out
export TMPDIR=/tmp
cmd="python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0"
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 300 $cmd > $out/masks.jsonl 2> $out/masks.err || exit $?
CG_RAW_PARSE=bytes timeout -k 10 300 $cmd > $out/bytes.jsonl 2> $out/bytes.err || exit $?
sq="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -k 10 300 rocprofv3 --pmc $sq --output-format csv -d $out/pm/p1 -o run -- $cmd > $out/pm.log 2>&1 || exit $?
CG_RAW_PARSE=bytes timeout -k 10 300 rocprofv3 --pmc $sq --output-format csv -d $out/pb/p1 -o run -- $cmd > $out/pb.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pm/p2 -o run -- $cmd > $out/pm2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pm/p3 -o run -- $cmd > $out/pm3.log 2>&1 || exit $?
