#!/bin/bash
# PMC passes over one of the L4 / prefilter / Kafka kernels (each counter
# group in its own rocprofv3 run; no tracing domains combined with --pmc).
#   bash tools/gpu_pmc_paths.sh <tag> <path: l4|lpm|kafka>
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-pmcp}; path=${2:-kafka}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
cmd="python3 tools/bench_paths.py --paths $path --steps 2 --cpu-seconds 0"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$tag/p$i -o run -- $cmd > gpurun_out/$tag/p$i.log 2>&1 || exit $?
done
