#!/bin/bash
# GPU box: compact 4-byte meta words (+ half last units) vs half last units alone:
# the last unit store it as 8 B per lane): the whole -m gpu suite, then the
# headline kernel A/B against the library before the change
# (tools/_exp/lib_h_half.so) on prof_http's workload (interleaved, verdict
# digests of each library's own batch layout compared within a library),
# the headline kernel trace + PMC passes (tools/gpu_headline_prof.sh), and
# the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05t}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/rc.txt; fatal $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 tools/prof_http.py --requests 124780544 --iters 10 > $out/$name.log 2>&1
}
for r in 1 2; do
  run new$r; rc=$?; echo "new$r rc=$rc" >> $out/rc.txt; fatal $rc
  run old$r CILIUM_AMD_LIB=$PWD/tools/_exp/lib_h_half.so; rc=$?; echo "old$r rc=$rc" >> $out/rc.txt; fatal $rc
done
bash tools/gpu_headline_prof.sh ${tag}_headline
rc=$?; echo "headline rc=$rc" >> $out/rc.txt; fatal $rc
timeout -k 10 500 python3 bench.py > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $out/rc.txt; fatal $rc
