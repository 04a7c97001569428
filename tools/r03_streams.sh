#!/bin/bash
O=gpurun_out/r03st; mkdir -p $O
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
show() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['pipeline_avg_ms'])"; }
for rep in 1 2; do
  for s in 2 3 4; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --streams $s $FAST > $O/s$s.$rep.json 2>>$O/err.txt || exit 1
    show $O/s$s.$rep.json
  done
done
