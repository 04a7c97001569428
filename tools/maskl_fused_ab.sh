#!/bin/bash
# Fused MaskS+MaskL pass (k_scan_f): GPU parity in the default mode and with
# every group fused (CDC_MASKL_INDEX=2), C3 kernel trace, then warm A/B of
# the previous build (variants/old.so) against the current one on C3 and C1.
set -e
OUT=gpurun_out/mlfused; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
echo "default: $(tail -1 $OUT/gpu_tests.log)"
CDC_MASKL_INDEX=2 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_m2.log 2>&1
echo "mode 2: $(tail -1 $OUT/gpu_tests_m2.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt3" -o run -- \
    python3 bench.py --workload c3 --steps 100 --warmup 200 --streams 1 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 > "$OUT/kt3_bench.json" 2> "$OUT/kt3.err"
python tools/kstats.py "$OUT/kt3/run_kernel_trace.csv" | head -8
V=$PWD/plakar_amd/_lib/variants
for wl in c3 c1; do
  for r in 1 2; do
    for lib in $V/old.so $PWD/plakar_amd/_lib/libplakar_cdc.so; do
      PLAKAR_CDC_LIB=$lib timeout -k 10 120 python bench.py --workload $wl --no-cpu-baseline --e2e-reps 0 --digest-reps 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print('$wl $(basename $lib)', d['value'], r['frac'], r.get('pipeline_avg_ms'), d.get('parity_vs_oracle'))"
    done
  done
done
