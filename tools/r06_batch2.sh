#!/bin/bash
# Round 6: (1) cross-stream scan order A/B (CDC_SCAN_ORDER) on the driver's
# command; (2) C3 lines and k_scan_f instruction counts (CDC_MASKL_INDEX=2:
# the fused pass every launch group) for the round-6 scan and round 5's.
TAG=${1:-r06b2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
bash tools/ab_env_driver.sh "$TAG" CDC_SCAN_ORDER "0 1" 3 || exit 1
QUIET="--no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0"
for v in base var_r05scan.so; do
  lib=""; [ "$v" != base ] && lib="$PWD/plakar_amd/_lib/$v"
  n=${v%.so}
  PLAKAR_CDC_LIB=$lib timeout -k 10 300 python3 bench.py --workload c3 $QUIET > "$OUT/c3_$n.json" 2> "$OUT/c3_$n.err" || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c3', sys.argv[2], d['value'], 'scan', r['kernel'][:12], r['kernel_avg_ms'], 'frac', r['frac'], 'pass', r['pipeline_avg_ms'])" "$OUT/c3_$n.json" $n
  SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  CDC_MASKL_INDEX=2 PLAKAR_CDC_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d "$OUT/pmcf_$n" -o run -- \
      python3 bench.py --workload c3 --roofline-only --steps 5 --warmup 0 > "$OUT/pmcf_$n.json" 2> "$OUT/pmcf_$n.err" || echo "pmc $n failed"
  python tools/pmc_summary.py "$OUT" k_scan_f --glob "pmcf_$n"
done
echo done
