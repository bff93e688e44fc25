#!/bin/bash
# GPU box, round 6: the Kafka wire GPU tests, then the decode path line at
# 4, 8 and 16 KiB per-wave stages (CILIUM_GPU_KAFKA_STAGE_KB) on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06ze}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kafka_wire.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
for kb in 4 8 16 8; do
  CILIUM_GPU_KAFKA_STAGE_KB=$kb timeout -k 10 300 python3 tools/bench_paths.py --paths kafkawire,kafkawirez --steps 5 --cpu-seconds 0.2 > $out/paths_$kb.jsonl 2> $out/paths_$kb.err || exit $?
done
