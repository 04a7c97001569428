#!/bin/bash
# Persistent scan: parity + tasks-per-wave sweep on the driver command and the warm default.
set -o pipefail
O=gpurun_out/${1:-r03d}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
echo "pytest rc=$?" | tee -a $O/status.txt; tail -2 $O/pytest.txt
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
show() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['pipeline_avg_ms'], d['config']['chunks_per_step'])"; }
for rep in 1 2; do
for t in 0 2 3 4 6; do
  CDC_SCAN_TASKS_PER_WAVE=$t timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/drv_t$t.$rep.json 2>>$O/err.txt || exit 1
  show $O/drv_t$t.$rep.json
done
done
for t in 0 3 6; do
  CDC_SCAN_TASKS_PER_WAVE=$t timeout -k 10 120 python bench.py $FAST > $O/def_t$t.json 2>>$O/err.txt || exit 1
  show $O/def_t$t.json
done
