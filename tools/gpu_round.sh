#!/bin/bash
# One GPU call: the -m gpu suite, smoke(), the default bench line, then the
# headline-only kernel trace + PMC passes (tools/gpu_headline_prof.sh).  A
# failing test does not stop the measurements; a timeout, abort or crash
# (124, 134, 137, 139) ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r04}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $out/rc.txt; fatal $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 400 python3 bench.py > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $out/rc.txt; fatal $rc
bash tools/gpu_headline_prof.sh ${tag}_headline
echo "prof rc=$?" >> $out/rc.txt
