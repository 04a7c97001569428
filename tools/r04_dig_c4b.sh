#!/bin/bash
# The pipelined digest leg on C1 / C3 (digest windows on alternating streams), then c4b with its pipeline trace.
O=gpurun_out/${1:-r04dc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for wl in c1 c3; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 20 --warmup 20 --no-cpu-baseline --e2e-reps 0 --encode-reps 0 > $O/$wl.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$wl.json').read().strip().splitlines()[-1]); c=d['chunk_digests']; print('$wl digests', c['value'], c.get('ms_per_pass'), 'pipelined', c['pipelined_with_chunking'])"
done
bash tools/r04_c4b_trace.sh ${1:-r04dc}/c4b
