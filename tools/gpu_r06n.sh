#!/bin/bash
# GPU box, round 6: every raw-path / fields / codec GPU test (field_of_words
# now reads a name-key slot in two 16-byte loads) and the ring's, then the
# ring latency entries with the phase trace at 64 workgroups.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06n}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py tests/test_http_raw_dl_gpu.py tests/test_http_codec_gpu.py tests/test_http_ring_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 CILIUM_GPU_RING_TRACE=1 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring,fields > $out/latency64.jsonl 2> $out/latency64.err || exit $?
