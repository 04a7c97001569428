#!/bin/bash
# c4b with 256 / 384 / 512 / 768-MiB device batches on the final pipeline, interleaved, two rounds.
O=gpurun_out/${1:-r04batch2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for n in 512 256 384 768; do
    timeout -k 10 300 python3 bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline --backup-batch-mib $n > $O/b${n}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$O/b${n}_$r.json').read().strip().splitlines()[-1]); b=d['backup_stages']; print('batch $n run $r', d['value'], d['ms_per_step'], b['wall_s'], b['batches'])"
  done
done
