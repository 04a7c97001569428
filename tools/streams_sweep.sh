set -e
for r in 1 2; do for n in 2 3 4; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --streams $n 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print('streams=$n', d['value'], d['ms_per_step'], r['achieved'])"
done; done
