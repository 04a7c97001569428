set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/s30
for n in 2 3 4 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --streams $n > gpurun_out/s30/b$n.json 2>gpurun_out/s30/b$n.err
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/s30/b$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('streams=$n', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
done
