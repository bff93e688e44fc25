#!/bin/bash
# GPU box: the whole -m gpu suite (verbose), smoke(), bench.py (default args)
# and a kernel trace of the same bench run.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-full}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $out/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check > $out/prof.log 2>&1 || exit $?
