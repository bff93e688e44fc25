#!/bin/bash
# GPU box: PMC passes over the HTTP verdict kernel at the bench size, then the
# L4 and Kafka kernels (bench_paths), each counter group in its own run.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-pmcall}
bash tools/gpu_pmc.sh $tag/http 124780544 || exit $?
bash tools/gpu_pmc_paths.sh $tag l4 kafka || exit $?
bash tools/exp_paths.sh lpm lpm_ > gpurun_out/$tag/lpm_exp.txt 2>&1 || exit $?
