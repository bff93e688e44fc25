#!/bin/bash
# GPU box, round 6: gpu_r06z.sh (list scans over register mask windows),
# then the Kafka wire GPU tests and path lines with small payloads inflated
# into LDS.
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r06z.sh r06z || exit $?
bash tools/gpu_r06t.sh r06za || exit $?
