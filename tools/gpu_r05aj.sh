#!/bin/bash
# GPU box: the whole -m gpu suite on the final tree (with the concurrency
# tests added after r05final).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05aj}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
echo "pytest rc=$?" > $out/rc.txt
