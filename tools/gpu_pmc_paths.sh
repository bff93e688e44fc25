#!/bin/bash
# PMC passes over bench_paths kernels (each counter group in its own
# rocprofv3 run; no tracing domains combined with --pmc).
#   bash tools/gpu_pmc_paths.sh <tag> <path> [<path> ...]
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-pmcp}; shift
export TMPDIR=/tmp
for path in "$@"; do
  out=gpurun_out/$tag/$path
  mkdir -p $out
  cmd="python3 tools/bench_paths.py --paths $path --steps 2 --cpu-seconds 0"
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- $cmd > $out/p$i.log 2>&1 || exit $?
  done
done
