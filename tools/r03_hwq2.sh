#!/bin/bash
# Chunking + digest legs with 4 (the box) vs 8 hardware queues per process.
O=gpurun_out/r03hwq2; mkdir -p $O
python3 - <<'PY'
s=open('bench.py').read()
s=s.replace('    if WORKLOADS[args.workload].get("backup"):\n        # the backup','    if True:\n        # the backup',1)
open('bench_hwq.py','w').write(s)
PY
for rep in 1 2; do
  for q in 4 8; do
    for wl in c1 c2; do
      if [ $q = 8 ]; then B=bench_hwq.py; else B=bench.py; fi
      timeout -k 10 300 python $B --workload $wl --no-cpu-baseline --encode-reps 0 --e2e-reps 0 --digest-reps 3 > $O/q$q.$wl.$rep.json 2>>$O/err.txt || { rm -f bench_hwq.py; exit 1; }
      python3 -c "import json; d=json.load(open('$O/q$q.$wl.$rep.json')); g=d['chunk_digests']; print('q$q $wl', d['value'], g['value'], g['pipelined_with_chunking']['value'])"
    done
  done
done
rm -f bench_hwq.py
