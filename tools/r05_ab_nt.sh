#!/bin/bash
# Round 5: nontemporal staging loads in the scan (-DCDC_SCAN_DMA_NT) vs default; the pattern microbenchmark first.
O=gpurun_out/${1:-r05abnt}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 120 tools/_bin/ubench_pattern > $O/pattern.txt 2>&1 || { cat $O/pattern.txt; exit 1; }
cat $O/pattern.txt
PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/v_nt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or sizes or c1_full or c3 or c2_shape" > $O/pytest_nt.txt 2>&1 || { echo "nt parity failed"; tail -20 $O/pytest_nt.txt; exit 1; }
tail -1 $O/pytest_nt.txt
drv() {  # name lib extra
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 timeout -k 10 200 python bench.py --gpus 1 $3 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/$1.json 2>>$O/err.txt || { echo "$1 failed"; tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);print('$1', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('pipeline_avg_ms'), d['parity_vs_oracle'])"
}
for r in 1 2 3; do
  drv drv_base_$r libplakar_cdc.so "--steps 20 --warmup 5"
  drv drv_nt_$r v_nt.so "--steps 20 --warmup 5"
done
drv warm_base libplakar_cdc.so ""
drv warm_nt v_nt.so ""
drv c2_base libplakar_cdc.so "--workload c2"
drv c2_nt v_nt.so "--workload c2"
drv c3_base libplakar_cdc.so "--workload c3"
drv c3_nt v_nt.so "--workload c3"
echo done
