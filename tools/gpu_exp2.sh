#!/bin/bash
# GPU box: HTTP parity tests on the in-tree library, then L4 variants through
# bench_paths and HTTP variants through bench.py (tools/_exp libraries).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/exp2
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "http or Http or starwars or rule_counters or configs" > gpurun_out/exp2/pytest.log 2>&1 || exit $?
bash tools/exp_paths.sh l4 l4_ > gpurun_out/exp2/l4.txt 2>&1 || exit $?
for lib in tools/_exp/lib_h_*.so; do
  name=$(basename $lib .so)
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check --steps 20 \
    > gpurun_out/exp2/$name.log 2>&1 || exit $?
  echo "$name: $(tail -1 gpurun_out/exp2/$name.log | cut -c1-140)" >> gpurun_out/exp2/http.txt
done
