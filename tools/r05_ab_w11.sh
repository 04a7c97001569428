#!/bin/bash
# round 5: scan waves per CU 12 vs 11 (one SIMD keeps room for a 1-wave k_resolve beside the next pass's scan)
O=gpurun_out/$1; mkdir -p $O
export PYTHONUNBUFFERED=1
PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/v_w11.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or sizes or sweep or pipelined or c1_full or c2_shape" > $O/pytest_w11.txt 2>&1 || { echo "w11 parity failed"; tail -20 $O/pytest_w11.txt; exit 1; }
tail -1 $O/pytest_w11.txt
drv() {  # name lib extra
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 timeout -k 10 200 python bench.py --gpus 1 $3 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/$1.json 2>>$O/err.txt || { echo "$1 failed"; tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);print('$1', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('pipeline_avg_ms'), d['parity_vs_oracle'])"
}
for r in 1 2; do
  drv drv_base_$r libplakar_cdc.so "--steps 20 --warmup 5"
  drv drv_w11_$r v_w11.so "--steps 20 --warmup 5"
  drv drv_r1_$r v_r1.so "--steps 20 --warmup 5"
done
drv warm_base libplakar_cdc.so ""
drv warm_w11 v_w11.so ""
