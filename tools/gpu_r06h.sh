#!/bin/bash
# GPU box, round 6: gpu_r06f.sh (ring tests + latency, stale path lines,
# LDS-DMA stream A/B) then gpu_r06g.sh (encoded ipcache chunks: tests,
# path lines, PMC) in one call.
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r06f.sh ${1:-r06h} || exit $?
bash tools/gpu_r06g.sh ${2:-r06h_ipc} || exit $?
