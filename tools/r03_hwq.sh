#!/bin/bash
O=gpurun_out/r03hwq; mkdir -p $O
for rep in 1 2; do
  for q in 4 8; do
    sed "s/os.environ\[\"GPU_MAX_HW_QUEUES\"\] = \"8\"/os.environ[\"GPU_MAX_HW_QUEUES\"] = \"$q\"/" bench.py > $O/bench_q$q.py
    cp $O/bench_q$q.py bench_q$q.py
    timeout -k 10 300 python bench_q$q.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline > $O/q$q.$rep.json 2>>$O/err.txt || { rm -f bench_q*.py; exit 1; }
    python3 -c "import json; d=json.load(open('$O/q$q.$rep.json')); b=d['backup_stages']; print('q$q', d['value'], d['ms_per_step'], b['wall_s'], b['GPU_MAX_HW_QUEUES'])"
  done
done
rm -f bench_q*.py
