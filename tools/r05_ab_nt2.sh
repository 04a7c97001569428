#!/bin/bash
# Round 5: confirmation of nontemporal scan staging (now the default) against the default-policy build (v_dflt).
O=gpurun_out/${1:-r05abnt2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
drv() {  # name lib extra
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 timeout -k 10 200 python bench.py --gpus 1 $3 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/$1.json 2>>$O/err.txt || { echo "$1 failed"; tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);print('$1', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('pipeline_avg_ms'), d['parity_vs_oracle'])"
}
for r in 1 2 3 4; do
  drv drv_nt_$r libplakar_cdc.so "--steps 20 --warmup 5"
  drv drv_dflt_$r v_dflt.so "--steps 20 --warmup 5"
done
drv warm_nt libplakar_cdc.so ""
drv warm_dflt v_dflt.so ""
drv c2_nt libplakar_cdc.so "--workload c2"
drv c2_dflt v_dflt.so "--workload c2"
echo done
