#!/bin/bash
# Round 6: GPU suite on the current tree, then an interleaved A/B of library
# variants (tools/ab.sh), then SQ instruction-count PMC passes of the C1 / C3
# scans for each variant.
#   tools/r06_check.sh <tag> [variant.so ...]
TAG=${1:-r06c}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[1] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "[2] A/B"
bash tools/ab.sh "$TAG" base "$@" || exit 1
echo "[3] PMC"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib="$PWD/plakar_amd/_lib/$v"
  for wl in c1 c3; do
    PLAKAR_CDC_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d "$OUT/pmc_${v%.so}_$wl" -o run -- \
        python3 bench.py --workload $wl --roofline-only --steps 5 --warmup 0 > "$OUT/pmc_${v%.so}_$wl.json" 2> "$OUT/pmc_${v%.so}_$wl.err" || echo "pmc $v $wl failed"
    for k in k_scan k_scan_f; do python tools/pmc_summary.py "$OUT" $k --glob "pmc_${v%.so}_$wl" 2>/dev/null | grep -v "^$" ; done
  done
done
echo done
