set -e
for t in 4 8 12 16; do
  CDC_COPY_THREADS=$t timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('threads=$t', d['value'], d['ms_per_step'])"
done
