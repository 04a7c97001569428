# Sustained (scan-only, back-to-back) vs isolated scan rates of built variants: tools/sustained.sh "v1 v2"
set -e
for v in $1; do for so in 1 0; do for n in 1 2; do
  CDC_DIAG_SCAN_ONLY=$so PLAKAR_CDC_LIB=plakar_amd/_lib/variants/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --steps 40 --streams $n 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print('$v scan_only=$so streams=$n', d['value'], d['ms_per_step'], r['achieved'])"
done; done; done
