#!/bin/bash
# ASan + UBSan run of the host code paths (CPU only, no GPU): build the
# sanitized library, then the CPU test suite and the bounded parser fuzz
# against it.  Output: profiles/<tag>_asan.log (committed summary).
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
tag=${1:-r03}
python3 tools/sanitize/build_asan.py || exit 1
export CILIUM_AMD_LIB=$PWD/tools/sanitize/_build/libciliumgpu_asan.so
export LD_PRELOAD=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
log=profiles/${tag}_asan.log
{
  echo "# ASan+UBSan host build: $CILIUM_AMD_LIB"
  echo "# runtime: $LD_PRELOAD"
  date -u
  python3 -m pytest tests -m "not gpu" -q -p no:cacheprovider --deselect tests/test_multirank_gloo.py 2>&1 | tail -5
  FUZZ_SECONDS=${FUZZ_SECONDS:-60} python3 tools/sanitize/fuzz.py 2>&1 | tail -12
} > $log 2>&1
rc=$?
grep -E "ERROR: AddressSanitizer|runtime error:|passed|failed|fuzz" $log | head -20
exit $rc
