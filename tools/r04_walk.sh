#!/bin/bash
# skip walk (CDC_WALK_MODE=2): parity suite, then the driver's command and the warm default, walk vs full scan.
O=gpurun_out/${1:-r04walk}; mkdir -p $O
export PYTHONUNBUFFERED=1
CDC_WALK_MODE=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -m gpu --timeout 200 --timeout-method thread --deselect tests/test_gpu_parity.py::test_maskl_adaptive_follows_the_data > $O/pytest_walk.txt 2>&1; rc=$?
tail -3 $O/pytest_walk.txt
[ $rc -eq 0 ] || exit $rc
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
for m in 2 0 2 0; do
  CDC_WALK_MODE=$m timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/c1_drv_m$m.json 2>>$O/err.txt || exit 1
  python -c "import json,sys; d=json.load(open('$O/c1_drv_m$m.json')); print('mode $m driver', d['value'], d['ms_per_step'], d['roofline']['pipeline_avg_ms'])"
done
for m in 2 0; do
  CDC_WALK_MODE=$m timeout -k 10 120 python bench.py $FAST > $O/c1_def_m$m.json 2>>$O/err.txt || exit 1
  python -c "import json,sys; d=json.load(open('$O/c1_def_m$m.json')); print('mode $m default', d['value'], d['ms_per_step'], d['roofline']['pipeline_avg_ms'])"
done
CDC_WALK_MODE=2 CDC_DEBUG_PHASE=16 timeout -k 10 120 python tools/tsdump.py --warm 5 > $O/tsdump_walk.txt 2>&1 || exit 1
grep -v "amdgpu.ids\|UserWarning\|ensure_init" $O/tsdump_walk.txt | head -40
