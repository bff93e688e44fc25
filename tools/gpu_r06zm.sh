#!/bin/bash
# GPU box, round 6: Kafka wire decode with the per-wave stage filled in
# rounds (every request parses from LDS) against the single-stage build
# (abtmp/libold.so), same box, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zm}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kafka_wire.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_paths.py --paths kafkawire,kafkawirez --steps 5 --cpu-seconds 0.2 > $out/paths_new$r.jsonl 2> $out/paths_new$r.err || exit $?
  CILIUM_AMD_LIB=abtmp/libold.so timeout -k 10 300 python3 tools/bench_paths.py --paths kafkawire,kafkawirez --steps 5 --cpu-seconds 0.2 > $out/paths_old$r.jsonl 2> $out/paths_old$r.err || exit $?
done
