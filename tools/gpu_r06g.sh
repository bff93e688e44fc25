#!/bin/bash
# GPU box, round 6: the encoded ipcache v4 chunks — every ipcache / L4 GPU
# test, the ipcache and fused L4 + ipcache path lines under a kernel trace,
# then the ipcache PMC passes (one counter group per rocprofv3 run,
# summarized by tools/pmc_summary.py).
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06g}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 400 python3 -u -m pytest tests/test_ipcache.py tests/test_gpu_configs.py tests/test_entities_e2e.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/rc.txt; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python3 tools/bench_paths.py --paths ipcache,l4ipc --steps 5 --cpu-seconds 2 > $out/paths.jsonl 2> $out/paths.err
rc=$?; echo "paths rc=$rc" >> $out/rc.txt; fatal $rc
cmd="python3 tools/bench_paths.py --paths ipcache --steps 2 --cpu-seconds 0"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  mkdir -p $out/ipcache
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $out/ipcache/p$i -o run -- $cmd > $out/ipcache/p$i.log 2>&1
  rc=$?; echo "ipcache p$i rc=$rc" >> $out/rc.txt; fatal $rc
done
