#!/bin/bash
# GPU box: the raw / header-list test files (NULL-stream device-layout calls).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05j}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_http_raw_gpu.py tests/test_http_fields_gpu.py tests/test_http_raw_dl_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $out/rc.txt
case $rc in 124|134|137|139) exit $rc;; esac
exit 0
