#!/bin/bash
# proxylib OnData through the C ABI (tools/ondata_bench, built on the CPU):
# r2d2 / memcache / cassandra, 1 and 16 threads, latency and calls/s.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-ondata}; out=gpurun_out/$tag
mkdir -p $out
CILIUM_GPU_DEVICE=0 timeout -k 10 300 tools/ondata_bench ${2:-2000} ${3:-16} > $out/ondata.jsonl 2> $out/ondata.err
