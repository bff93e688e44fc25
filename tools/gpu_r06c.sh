#!/bin/bash
# GPU box, round 6: the persistent verdict ring — its GPU tests first (short
# limit: a resident kernel), then the latency driver's ring / fields entries.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06c}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 180 python3 -u -m pytest tests/test_http_ring_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/http_latency.py --seconds 0.5 --entries ring,fields > $out/latency.jsonl 2> $out/latency.err || exit $?
