#!/bin/bash
# GPU box, round 6 final tree: the whole -m gpu suite, smoke(), the default
# bench line, the headline's rocprof kernel trace, every path line under a
# kernel trace, and the Envoy-shaped latency entries (ring and fields).
# A failing test does not stop the rest; a timeout, abort or crash ends the
# call.
cd "$GRAFT_REPO_ROOT" || exit 1
# part a: tests, smoke, bench, bench trace; part b: paths and latency
tag=${1:-r06final}; part=${2:-a}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
if [ "$part" = a ]; then
: > $out/rc.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 500 python3 bench.py > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/benchkt -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --sustain-seconds 0 --no-cpu-baseline > $out/bench_kt.log 2>&1
rc=$?; echo "bench kt rc=$rc" >> $out/rc.txt; fatal $rc
else
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/paths -o run --output-format csv -- python3 tools/bench_paths.py --paths l4,lpm,kafka,ipcache,l4ipc,proxylib,memcache,cassandra,kafkawire,kafkawirez,httpraw,httpfields --steps 5 --cpu-seconds 2 > $out/paths.jsonl 2> $out/paths.err
rc=$?; echo "paths rc=$rc" >> $out/rc.txt; fatal $rc
CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 timeout -k 10 500 python3 tools/http_latency.py --seconds 0.5 --entries ring,fields > $out/latency.jsonl 2> $out/latency.err
rc=$?; echo "latency rc=$rc" >> $out/rc.txt; fatal $rc
fi
