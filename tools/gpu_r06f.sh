#!/bin/bash
# GPU box, round 6: the ring's GPU tests and latency entries, then the path
# lines round 5 left stale (Kafka wire decode with and without compressed
# sets, proxylib r2d2 / memcache / cassandra on http_kernel) under a kernel
# trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06f}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 180 python3 -u -m pytest tests/test_http_ring_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
CILIUM_GPU_DEBUG=1 timeout -k 10 400 python3 tools/http_latency.py --seconds 0.5 --entries ring,fields > $out/latency.jsonl 2> $out/latency.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/paths -o run --output-format csv -- python3 tools/bench_paths.py --paths kafkawire,kafkawirez,proxylib,memcache,cassandra --steps 5 --cpu-seconds 2 > $out/paths.jsonl 2> $out/paths.err || exit $?
timeout -k 10 120 ./tools/stream_ab 8 3 > $out/stream_ab_u3.jsonl 2>&1 || exit $?
timeout -k 10 120 ./tools/stream_ab 8 4 > $out/stream_ab_u4.jsonl 2>&1 || exit $?
