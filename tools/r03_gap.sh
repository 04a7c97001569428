#!/bin/bash
O=gpurun_out/${1:-r03f}; mkdir -p $O
export PYTHONUNBUFFERED=1
# (suite run separately)
: timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
echo "pytest rc=$?"; tail -1 $O/pytest.txt
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
show() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['pipeline_avg_ms'])"; }
for rep in 1 2; do
  for m in 0 2; do
    CDC_WALK_MODE=$m timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/drv_m$m.$rep.json 2>>$O/err.txt || exit 1
    show $O/drv_m$m.$rep.json
  done
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --streams 1 $FAST > $O/drv_s1.$rep.json 2>>$O/err.txt || exit 1
  show $O/drv_s1.$rep.json
done
timeout -k 10 120 python bench.py $FAST > $O/def.json 2>>$O/err.txt && show $O/def.json
CDC_DEBUG_PHASE=16 timeout -k 10 120 python tools/tsdump.py --warm 30 > $O/ts.txt 2>&1; grep -E "wave0 end|k_resolve segs|inclusive" $O/ts.txt
