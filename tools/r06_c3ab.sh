#!/bin/bash
# Round 6: k_scan_f with one filter key (the bits MaskS and MaskL share)
# against variants (var_*.so): the parity subset on each library, C3
# lines interleaved twice, and the k_scan_f instruction counts
# (CDC_MASKL_INDEX=2: the fused pass every launch group).
#   tools/r06_c3ab.sh <tag> variant.so ...
TAG=${1:-r06c3}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib="$PWD/plakar_amd/_lib/$v"
  n=${v%.so}
  PLAKAR_CDC_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_abort.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$n.log" 2>&1 || { tail -20 "$OUT/pytest_$n.log"; exit 1; }
  echo "$n: $(tail -1 $OUT/pytest_$n.log)"
done
QUIET="--no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0"
for rep in 1 2; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib="$PWD/plakar_amd/_lib/$v"
    n=${v%.so}
    PLAKAR_CDC_LIB=$lib timeout -k 10 300 python3 bench.py --workload c3 $QUIET > "$OUT/c3_${n}_$rep.json" 2> "$OUT/c3_${n}_$rep.err" || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c3', sys.argv[2], d['value'], 'scan', r['kernel'][:12], r['kernel_avg_ms'], 'frac', r['frac'], 'pass', r['pipeline_avg_ms'])" "$OUT/c3_${n}_$rep.json" "$n.$rep"
  done
done
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib="$PWD/plakar_amd/_lib/$v"
  n=${v%.so}
  CDC_MASKL_INDEX=2 PLAKAR_CDC_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d "$OUT/pmcf_$n" -o run -- \
      python3 bench.py --workload c3 --roofline-only --steps 5 --warmup 0 > "$OUT/pmcf_$n.json" 2> "$OUT/pmcf_$n.err" || { echo "pmc $n failed"; exit 1; }
  python tools/pmc_summary.py "$OUT" k_scan_f --glob "pmcf_$n"
done
echo done
