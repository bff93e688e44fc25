#!/bin/bash
# GPU box: HTTP parity tests, one bench line, then every kernel variant built
# by tools/exp_http.py (one process each, own time limit).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-exp}; req=${2:-64000000}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k http --timeout 200 --timeout-method thread > $out/pytest_http.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.log 2>&1 || exit $?
for lib in tools/_exp/lib_*.so; do
  [ -e "$lib" ] || continue
  name=$(basename $lib .so)
  CILIUM_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 tools/prof_http.py --requests $req --iters 5 > $out/$name.log 2>&1 || exit $?
  echo "$name: $(tail -1 $out/$name.log)"
done
