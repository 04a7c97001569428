# Warm A/B of built variants (default bench warm-up): tools/ab_warm.sh "v1 v2" [bench args]
set -e
VS=$1; shift
for r in 1 2; do for v in $VS; do
  PLAKAR_CDC_LIB=plakar_amd/_lib/variants/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0 "$@" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('pipeline_avg_ms'))"
done; done
