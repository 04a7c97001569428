#!/bin/bash
# The driver's command (--steps 20 --warmup 5) with 2 / 3 / 4 pass streams, interleaved, three rounds.
O=gpurun_out/${1:-r04streams}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for n in 2 3 4; do
    timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams $n --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0 > $O/s${n}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$O/s${n}_$r.json').read().strip().splitlines()[-1]); print('streams $n run $r', d['value'], d['ms_per_step'])"
  done
done
