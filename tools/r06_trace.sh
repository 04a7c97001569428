#!/bin/bash
# Round 6: the driver's exact command under a rocprofv3 kernel trace, per
# library variant, with tools/timeline.py's per-pass timeline.
#   tools/r06_trace.sh <tag> [variant.so ...]   ("base" = the in-tree library)
TAG=${1:-r06t}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for v in "$@"; do
  lib=""; [ "$v" != base ] && lib="$PWD/plakar_amd/_lib/$v"
  n=${v%.so}
  PLAKAR_CDC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$n" -o run -- \
      python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/kt_$n.json" 2> "$OUT/kt_$n.err" || exit 1
  f=$(ls $OUT/kt_$n/*/run_kernel_trace.csv $OUT/kt_$n/run_kernel_trace.csv 2>/dev/null | head -1)
  python tools/kstats.py "$f" > "$OUT/kt_${n}_summary.txt"
  python tools/timeline.py "$f" --warmup 5 --steps 20 > "$OUT/kt_${n}_timeline.txt" 2>&1 || true
  echo "== $n"; cut -c1-150 "$OUT/kt_$n.json"; head -12 "$OUT/kt_${n}_summary.txt"; tail -8 "$OUT/kt_${n}_timeline.txt"
done
echo done
