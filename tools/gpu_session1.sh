#!/bin/bash
# GPU session: parity tests, smoke, bench, kernel trace of the bench, then the
# kernel variants built by tools/exp_http.py.  Every GPU step has its own time
# limit and the steps are chained so that a failure ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-s1}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
nproc > $out/host.txt; grep -m1 "model name" /proc/cpuinfo >> $out/host.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $out/bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > $out/prof.log 2>&1 || exit $?
for lib in tools/_exp/lib_*.so; do
  [ -e "$lib" ] || continue
  name=$(basename $lib .so)
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 tools/prof_http.py --requests 64000000 --iters 5 > $out/exp_$name.log 2>&1 || exit $?
done
