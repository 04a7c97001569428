# scan fence A/B on the pipelined bench (cold 20/5 and warm 200/200), 1 vs 2 streams
for f in 0 1; do
  for st in 2 3; do
  for sw in "20 5" "200 200"; do
    set -- $sw
    CDC_SCAN_FENCE=$f timeout -k 10 120 python3 bench.py --steps $1 --warmup $2 --streams $st --no-cpu-baseline --e2e-reps 0 --digest-reps 0 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fence', $f, 'streams', $st, '$sw', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" || exit 1
  done
  done
done
