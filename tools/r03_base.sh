#!/bin/bash
# Session re-entry baseline: GPU suite, the driver's command x2, warm default, loop ceiling ubench.
O=gpurun_out/${1:-r03s}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 60 tools/_bin/ubl > $O/ubl.txt 2>&1; echo "ubl rc=$?"; cat $O/ubl.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
show() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['pipeline_avg_ms'])"; }
for rep in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/drv.$rep.json 2>>$O/err.txt || exit 1
  show $O/drv.$rep.json
done
timeout -k 10 120 python bench.py $FAST > $O/def.json 2>>$O/err.txt && show $O/def.json
CDC_DEBUG_PHASE=16 timeout -k 10 120 python tools/tsdump.py --warm 5 > $O/ts_warm5.txt 2>&1
CDC_DEBUG_PHASE=16 timeout -k 10 120 python tools/tsdump.py --warm 300 > $O/ts_warm300.txt 2>&1
echo done
