#!/bin/bash
# C3 fused scan: compact MaskL records vs base vs no records (timing only).
O=gpurun_out/r03c3; mkdir -p $O
export PYTHONUNBUFFERED=1
PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/var_lc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_lc.txt 2>&1
echo "pytest var_lc rc=$?"; tail -1 $O/pytest_lc.txt
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
show() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['frac'], r['pipeline_avg_ms'])"; }
for rep in 1 2; do
  for v in base var_lc var_nol; do
    lib=""; [ $v != base ] && lib=$PWD/plakar_amd/_lib/$v.so
    PLAKAR_CDC_LIB=$lib timeout -k 10 120 python bench.py --workload c3 $FAST > $O/$v.$rep.json 2>>$O/err.txt || exit 1
    show $O/$v.$rep.json
  done
done
