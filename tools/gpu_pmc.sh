#!/bin/bash
# PMC passes over the HTTP verdict kernel (each counter group in its own
# rocprofv3 run; no tracing domains are combined with --pmc).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-pmc}; req=${2:-32000000}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/prof_http.py --requests $req --iters 3 > gpurun_out/$tag/plain.log 2>&1 || exit $?
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$tag/p$i -o run -- python3 tools/prof_http.py --requests $req --iters 3 > gpurun_out/$tag/p$i.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/kt -o run -- python3 tools/prof_http.py --requests $req --iters 3 > gpurun_out/$tag/kt.log 2>&1 || exit $?
