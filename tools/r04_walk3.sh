#!/bin/bash
# k_walk: parity under the walk, then round 3's skip_scan vs the pipelined one (tsdump, cold), then the driver command.
O=gpurun_out/${1:-r04walk3}; mkdir -p $O
export PYTHONUNBUFFERED=1
CDC_WALK_MODE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread --deselect tests/test_gpu_parity.py::test_maskl_adaptive_follows_the_data > $O/pytest_walk.txt 2>&1; rc=$?
tail -2 $O/pytest_walk.txt
[ $rc -eq 0 ] || exit $rc
run() { # name lib debug
  CDC_WALK_MODE=2 PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 CDC_DEBUG_PHASE=$3 timeout -k 10 120 python tools/tsdump.py --warm 5 > $O/$1.txt 2>&1 || { echo "$1 failed"; tail -5 $O/$1.txt; exit 1; }
  echo "== $1"; grep -v "amdgpu.ids\|UserWarning\|ensure_init" $O/$1.txt | grep -A8 "k_walk segs"
}
run v3 var_skipv3.so 16 && run v4 libplakar_cdc.so 16 || exit 1
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
for m in 2 0; do
  CDC_WALK_MODE=$m timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/c1_drv_m$m.json 2>>$O/err.txt || exit 1
  python -c "import json,sys; d=json.load(open('$O/c1_drv_m$m.json')); print('mode $m driver', d['value'], d['ms_per_step'], d['roofline']['pipeline_avg_ms'])"
done
