#!/bin/bash
# Round 5: deferred recheck (CDC_SCAN_DEFER) vs the default immediate recheck: parity, driver command x3
# interleaved, warm, the cold roofline loop under a trace, and the scan's instruction counts (PMC).
#   tools/r05_ab_defer.sh <tag>
O=gpurun_out/${1:-r05abd}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/v_defer.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > $O/pytest_defer.txt 2>&1 || { echo "defer parity failed"; tail -20 $O/pytest_defer.txt; exit 1; }
tail -1 $O/pytest_defer.txt
drv() {  # name lib extra
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 timeout -k 10 200 python bench.py --gpus 1 $3 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/$1.json 2>>$O/err.txt || { echo "$1 failed"; tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);print('$1', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('pipeline_avg_ms'), d['parity_vs_oracle'])"
}
for r in 1 2 3; do
  drv drv_base_$r libplakar_cdc.so "--steps 20 --warmup 5"
  drv drv_defer_$r v_defer.so "--steps 20 --warmup 5"
done
drv warm_base libplakar_cdc.so ""
drv warm_defer v_defer.so ""
drv c3_base libplakar_cdc.so "--workload c3"
drv c3_defer v_defer.so "--workload c3"
for v in libplakar_cdc v_defer; do
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/roof_$v -o run -- \
      python3 bench.py --roofline-only --steps 20 --warmup 0 > $O/roof_$v.json 2>> $O/err.txt || { echo "roofline $v failed"; exit 1; }
  f=$(ls $O/roof_$v/*/run_kernel_trace.csv $O/roof_$v/run_kernel_trace.csv 2>/dev/null | head -1)
  python tools/kstats.py "$f" > $O/roof_${v}_summary.txt
  echo "$v"; grep "k_scan " $O/roof_${v}_summary.txt
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$v.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_$v -o run -- \
      python3 bench.py --roofline-only --steps 5 --warmup 0 > $O/pmc_$v.json 2>> $O/err.txt || echo "pmc $v failed"
  python tools/pmc_summary.py $O k_scan --glob "pmc_$v" > $O/pmc_${v}.txt 2>&1; cat $O/pmc_${v}.txt
done
echo done
