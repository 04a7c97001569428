#!/bin/bash
# Scan grid x resolution segment size under the driver's command: fewer scan
# workgroups leave CUs on which the previous pass's resolution runs beside the
# next pass's scan.
O=gpurun_out/${1:-r03pk}; mkdir -p $O
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
show() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['pipeline_avg_ms'])"; }
for rep in 1 2; do
  for cfg in "249 16" "240 16" "240 32" "232 32" "224 32" "240 24" "249 32"; do
    set -- $cfg
    CDC_SCAN_WGS=$1 CDC_SEG_MULT=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/w$1_m$2.$rep.json 2>>$O/err.txt || exit 1
    show $O/w$1_m$2.$rep.json
  done
done
