#!/bin/bash
# GPU round check: parity debug, GPU test suite, variant sweep.
#   tools/gpu_check.sh <tag> [sweep-spec]
# Stops at the first crash/timeout (rc not in {0,1}); test failures (rc 1) go on.
TAG=${1:-chk}; SPEC=$2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 150 python -u tools/dbg_parity.py 64 0 > "$OUT/dbg.log" 2>&1; rc=$?
grep -v amdgpu.ids "$OUT/dbg.log"; ok $rc || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
tail -4 "$OUT/gpu_tests.log"; ok $rc || exit $rc
if [ -n "$SPEC" ]; then
  timeout -k 10 400 python -u tools/sweep.py "$SPEC" > "$OUT/sweep.log" 2>&1; rc=$?
  grep -v amdgpu.ids "$OUT/sweep.log"; ok $rc || exit $rc
fi
exit 0
