#!/bin/bash
# Round 6: HBM bytes per scan launch (FETCH_SIZE, one counter pass per run) for
# C1 (k_scan), C2 (k_scan) and C3 (k_scan_f, CDC_MASKL_INDEX=2), the roofline
# loop alone (--roofline-only, 5 launches); feeds profiles/traffic.json.
#   tools/r06_traffic.sh <tag>
TAG=${1:-r06tr}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for wl in c1 c2 c3; do
  k=k_scan; [ $wl = c3 ] && k=k_scan_f
  CDC_MASKL_INDEX=$([ $wl = c3 ] && echo 2 || echo 1) timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE \
      --output-format csv -d "$OUT/fetch_$wl" -o run -- \
      python3 bench.py --workload $wl --roofline-only --steps 5 --warmup 0 > "$OUT/fetch_$wl.json" 2> "$OUT/fetch_$wl.err" || { echo "pmc $wl failed"; exit 1; }
  echo "== $wl $k"
  python tools/pmc_summary.py "$OUT" $k --glob "fetch_$wl"
done
echo done
