# Warm steady state: full pipeline vs scan-only launches, 1 and 2 streams.
set -e
for so in 0 1; do for n in 1 2; do
  CDC_DIAG_SCAN_ONLY=$so timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --streams $n 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print('scan_only=$so streams=$n', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
done; done
