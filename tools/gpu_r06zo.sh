#!/bin/bash
# GPU box, round 6: the device-layout scan's string-unit stores — plain
# (main library), nontemporal (tools/_exp/lib_rawdl_ntunits.so, verdicts
# checked against the host path) and none (lib_rawdl_nounitst.so, measuring
# device) — under a kernel trace, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r06zo}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal $1" >> $out/rc.txt; exit $1;; esac; }
: > $out/rc.txt
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 tools/bench_paths.py --paths httpraw --steps 3 --cpu-seconds 0 > $out/$name.jsonl 2> $out/$name.err
}
for r in 1 2; do
  run main_$r A=1; rc=$?; echo "main_$r rc=$rc" >> $out/rc.txt; fatal $rc
  run nt_$r CILIUM_AMD_LIB=$PWD/tools/_exp/lib_rawdl_ntunits.so; rc=$?; echo "nt_$r rc=$rc" >> $out/rc.txt; fatal $rc
  run nost_$r CG_EXP_NOCHECK=1 CILIUM_AMD_LIB=$PWD/tools/_exp/lib_rawdl_nounitst.so; rc=$?; echo "nost_$r rc=$rc" >> $out/rc.txt; fatal $rc
done
