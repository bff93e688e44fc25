#!/bin/bash
# GPU box: Kafka wire tests on the in-tree library, then each kw_ variant
# library built by tools/exp_http.py timed by tools/prof_kw.py.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-expkw}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kafka_wire.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
for lib in tools/_exp/lib_kw_*.so; do
  [ -e "$lib" ] || continue
  name=$(basename $lib .so)
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$name -o run -- python3 tools/prof_kw.py --iters 3 > $out/$name.log 2>&1 || exit $?
done
