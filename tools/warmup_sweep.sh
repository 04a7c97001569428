set -e
for wu in 3 50 200; do for st in 20 200; do
timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --steps $st --warmup $wu 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print('warmup=$wu steps=$st', d['value'], d['ms_per_step'], r['achieved'])"
done; done
