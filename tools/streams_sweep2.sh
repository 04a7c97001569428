#!/bin/bash
# Pipelined rate against the number of alternating streams (C1 and C3).
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/s31
for wl in c1 c3; do
  for n in 2 3 4 2 3 4; do
    timeout -k 10 120 python bench.py --workload $wl --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --streams $n > gpurun_out/s31/$wl-b$n.json 2>gpurun_out/s31/$wl-b$n.err
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/s31/$wl-b$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl streams=$n', d['value'], d['ms_per_step'], r['frac'])"
  done
done
