#!/bin/bash
# c4b with GPU_MAX_HW_QUEUES 8 vs 16 (BENCH_HW_QUEUES), interleaved, N rounds (arg 2, default 2).
O=gpurun_out/${1:-r04hwq}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in $(seq 1 ${2:-2}); do
  for q in 8 16; do
    BENCH_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline > $O/q${q}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$O/q${q}_$r.json').read().strip().splitlines()[-1]); b=d['backup_stages']; print('hwq $q run $r', d['value'], d['ms_per_step'], b['wall_s'], b['hw_queues'])"
  done
done
