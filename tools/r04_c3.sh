#!/bin/bash
# C3 (1 GiB zeros + 1 % random): MaskL index modes (CDC_MASKL_INDEX 1 adaptive -> fused k_scan_f, 3 k_scan + selective k_scan_l, 0 raw scans).
O=gpurun_out/${1:-r04c3}; mkdir -p $O
export PYTHONUNBUFFERED=1
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 --no-parity --workload c3"
for r in 1 2; do for m in 1 3 0; do
  CDC_MASKL_INDEX=$m timeout -k 10 120 python bench.py $FAST > $O/c3_m${m}_$r.json 2>>$O/err.txt || exit 1
  python -c "import json; d=json.load(open('$O/c3_m${m}_$r.json')); r=d['roofline']; print('c3 mode $m run $r', d['value'], d['ms_per_step'], 'scan', r['kernel_avg_ms'], r['frac'], 'pass', r['pipeline_avg_ms'])"
done; done
