#!/bin/bash
# Round 6: library variants -- a parity subset of the GPU suite per variant,
# then the interleaved A/B (tools/ab.sh) and the driver-command trace of each.
#   tools/r06_variants.sh <tag> variant.so ...
TAG=${1:-r06v}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for v in "$@"; do
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_abort.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_${v%.so}.log" 2>&1 || { tail -20 "$OUT/pytest_${v%.so}.log"; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_${v%.so}.log)"
done
bash tools/ab.sh "$TAG" base "$@" || exit 1
bash tools/r06_trace.sh "$TAG" base "$@" 2>&1 | grep -v "^kernel\|^cdc::\|^enc::\|^__amd" || exit 1
echo done
