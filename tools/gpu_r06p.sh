#!/bin/bash
# GPU box, round 6: ipcache GPU tests, then the family / encoding / K split
# (tools/ipcache_split.py) with the second round-1 pair for run lines and
# sparse maps.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06p}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_ipcache.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ipcache_split.py > $out/split.jsonl 2> $out/split.err || exit $?
timeout -k 10 300 python3 tools/ipcache_split.py --dense >> $out/split.jsonl 2>> $out/split.err || exit $?
