#!/bin/bash
# Resolution segment length under the driver's command (and warm), plus the skip walk for the record.
O=gpurun_out/${1:-r03sg}; mkdir -p $O
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
show() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['pipeline_avg_ms'], d['parity_vs_oracle'])"; }
for rep in 1 2 3; do
  for m in 16 32 48; do
    CDC_SEG_MULT=$m timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/m$m.$rep.json 2>>$O/err.txt || exit 1
    show $O/m$m.$rep.json
  done
done
for m in 16 32 48; do
  CDC_SEG_MULT=$m timeout -k 10 120 python bench.py $FAST > $O/warm_m$m.json 2>>$O/err.txt || exit 1
  show $O/warm_m$m.json
done
for wl in c2 c3; do for m in 16 32; do
  CDC_SEG_MULT=$m timeout -k 10 120 python bench.py --workload $wl $FAST > $O/${wl}_m$m.json 2>>$O/err.txt || exit 1
  show $O/${wl}_m$m.json
done; done
CDC_WALK_MODE=2 timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/skip_cold.json 2>>$O/err.txt && show $O/skip_cold.json
CDC_WALK_MODE=2 timeout -k 10 120 python bench.py $FAST > $O/skip_warm.json 2>>$O/err.txt && show $O/skip_warm.json
