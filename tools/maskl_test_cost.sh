#!/bin/bash
# Cost of k_scan_l's selection test on C1 (nothing selected): the default
# build against variants t1 (test returns at once) and t2 (record loads and
# ballots only), k_scan_l launched every group.
set -e
OUT=gpurun_out/mltest; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=$PWD/plakar_amd/_lib/variants
for lib in $PWD/plakar_amd/_lib/libplakar_cdc.so $V/t1.so $V/t2.so; do
  n=$(basename $lib .so)
  CDC_MASKL_INDEX=2 PLAKAR_CDC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n" -o run -- \
    python3 bench.py --steps 50 --warmup 100 --streams 1 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 > "$OUT/$n.json" 2> "$OUT/$n.err"
  echo "== $n"; python tools/kstats.py "$OUT/$n/run_kernel_trace.csv" | grep -E "k_scan"
done
