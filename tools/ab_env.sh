# A/B of an environment knob on the C1 bench: tools/ab_env.sh VAR "v1 v2 ..." [bench args]
set -e
VAR=$1; VALS=$2; shift 2
for r in 1 2; do
for v in $VALS; do
  env $VAR=$v timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0 --steps 30 "$@" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print('$VAR=$v', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('pipeline_avg_ms'))"
done
done
