#!/bin/bash
# GPU box, round 6: the ring's transport floor — the same latency driver with
# the kernel storing `done` at once (CILIUM_GPU_RING_ECHO=1) and after the
# data's copy-in (=2); verdicts are not decided in these modes, so the
# driver's bad-call counts are expected.  Then the normal ring for reference.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zj}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for e in 1 2 0; do
  CILIUM_GPU_RING_ECHO=$e CILIUM_RING_WORKGROUPS=64 CILIUM_RING_SLOTS=128 timeout -k 10 300 python3 tools/http_latency.py --seconds 0.5 --entries ring > $out/latency_echo$e.jsonl 2> $out/latency_echo$e.err
  rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
