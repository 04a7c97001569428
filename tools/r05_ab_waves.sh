#!/bin/bash
# Round 5: scan waves per CU 8 / 10 vs 12 (fewer waves: less power in the cold clock dip?)
#   tools/r05_ab_waves.sh <tag>
O=gpurun_out/${1:-r05abw}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for v in v_w8 v_w10; do
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or sizes or c1_full or c3" > $O/pytest_$v.txt 2>&1 || { echo "$v parity failed"; tail -20 $O/pytest_$v.txt; exit 1; }
  tail -1 $O/pytest_$v.txt
done
drv() {  # name lib extra
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 timeout -k 10 200 python bench.py --gpus 1 $3 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/$1.json 2>>$O/err.txt || { echo "$1 failed"; tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);print('$1', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('pipeline_avg_ms'), d['parity_vs_oracle'])"
}
for r in 1 2; do
  drv drv_base_$r libplakar_cdc.so "--steps 20 --warmup 5"
  drv drv_w8_$r v_w8.so "--steps 20 --warmup 5"
  drv drv_w10_$r v_w10.so "--steps 20 --warmup 5"
done
drv warm_base libplakar_cdc.so ""
drv warm_w8 v_w8.so ""
drv warm_w10 v_w10.so ""
echo done
