#!/bin/bash
# GPU box: Kafka slow-path queue carrying the head words (main library)
# against the round-5 kernel that re-reads heads (tools/_exp/lib_kf_old.so):
# bench_paths kafka (checked against the oracle) under a kernel trace, and
# FETCH_SIZE / WRITE_SIZE passes of each, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05p}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
cmd="python3 tools/bench_paths.py --paths kafka --steps 5 --cpu-seconds 0"
for r in 1 2; do
  for v in main kf_old; do
    if [ $v = main ]; then lib=""; else lib="CILIUM_AMD_LIB=$PWD/tools/_exp/lib_$v.so"; fi
    env $lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${v}_kt$r -o run --output-format csv -- $cmd > $out/${v}_kt$r.log 2>&1
    rc=$?; echo "${v}_kt$r rc=$rc" >> $out/rc.txt; fatal $rc
    if [ $r = 1 ]; then
      for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
        n=$(echo $grp | cut -d' ' -f1)
        env $lib timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $out/${v}_$n -o run -- $cmd > $out/${v}_$n.log 2>&1
        rc=$?; echo "${v}_$n rc=$rc" >> $out/rc.txt; fatal $rc
      done
    fi
  done
done
