#!/bin/bash
# GPU box, the round's final tree: the whole -m gpu suite, smoke(), the
# default bench line, the headline kernel trace + PMC (gpu_headline_prof.sh),
# the raw / list / Kafka / table paths under a kernel trace, and the
# Envoy-batch latency driver.  A failing test does not stop the
# measurements; a timeout, abort or crash ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05final}; out=gpurun_out/$tag
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
bash tools/gpu_headline_prof.sh ${tag}_headline
rc=$?; echo "headline rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/paths -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw,httpfields,kafka,l4,ipcache,lpm,l4ipc --steps 3 --cpu-seconds 2 > $out/paths.jsonl 2> $out/paths.err
rc=$?; echo "paths rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 400 python3 tools/http_latency.py --seconds 0.5 > $out/latency.jsonl 2> $out/latency.err
rc=$?; echo "latency rc=$rc" >> $out/rc.txt; fatal $rc
