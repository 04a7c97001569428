# seg-size sweep of the pipelined bench (cold 20/5 and warm 200/200)
for m in 16 32 64; do
  for sw in "20 5" "200 200"; do
    set -- $sw
    CDC_SEG_MULT=$m timeout -k 10 120 python3 bench.py --steps $1 --warmup $2 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('seg', $m, '$sw', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['pipeline_avg_ms'])" || exit 1
  done
done
