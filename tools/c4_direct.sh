set -e
for r in 1 2; do for dd in 0 1; do
  CDC_HOST_DIRECT=$dd timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('direct=$dd', d['value'], d['ms_per_step'])"
done; done
for dd in 0 1; do
  CDC_HOST_DIRECT=$dd timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-reps 3 --digest-reps 0 --steps 20 --warmup 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C1 e2e direct=$dd', d['e2e_host_path'])"
done
