#!/bin/bash
# GPU box, round 6: the whole -m gpu suite, smoke() and the default bench
# line.  A failing test does not stop smoke / bench; a timeout, abort or
# crash ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06full}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 500 python3 bench.py > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $out/rc.txt; fatal $rc
