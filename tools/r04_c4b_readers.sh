#!/bin/bash
# c4b with 12 / 14 / 16 reader threads (the box's CPU share is 16), interleaved, two rounds.
O=gpurun_out/${1:-r04readers}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for n in 16 12 14; do
    timeout -k 10 300 python3 bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline --backup-readers $n > $O/r${n}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$O/r${n}_$r.json').read().strip().splitlines()[-1]); b=d['backup_stages']; print('readers $n run $r', d['value'], d['ms_per_step'], b['wall_s'], b['objhash_s'], b['read_s'])"
  done
done
