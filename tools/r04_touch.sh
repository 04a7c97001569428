#!/bin/bash
# driver command A/B: streams bound to their hardware queues at setup (BENCH_TOUCH_STREAMS=1) or on first use (0).
O=gpurun_out/${1:-r04touch}; mkdir -p $O
export PYTHONUNBUFFERED=1
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 --no-parity"
for r in 1 2 3; do for t in 1 0; do
  BENCH_TOUCH_STREAMS=$t timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/drv_t${t}_$r.json 2>>$O/err.txt || exit 1
  python -c "import json; d=json.load(open('$O/drv_t${t}_$r.json')); print('touch $t run $r', d['value'], d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 $FAST > $O/drv_trace.json 2>>$O/err.txt || exit 1
f=$(ls $O/trace/*kernel_trace.csv $O/trace/*/*kernel_trace.csv 2>/dev/null | head -1); python tools/timeline.py $f --warmup 5 --steps 20 > $O/timeline.txt 2>&1; head -12 $O/timeline.txt; tail -8 $O/timeline.txt
