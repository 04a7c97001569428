#!/bin/bash
# Round 5: c4b pipeline traces (default 6 slots, then 7 and 8 slot variants), interleaved twice.
#   tools/r05_c4b_trace.sh <tag>
O=gpurun_out/${1:-r05c4bt}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
run() {  # name lib
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 CDC_BACKUP_TRACE=$O/$1_trace.csv timeout -k 10 300 python bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/$1.json 2>>$O/err.txt || { echo "$1 failed"; tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);s=d['backup_stages'];print('$1', d['value'], s['wall_s'], s['device_s'], s['read_wait_s'], d['parity_vs_oracle'])"
  python tools/backup_trace.py $O/$1_trace.csv > $O/$1_trace.txt 2>&1 || true
}
for r in 1 2; do
  run s6_$r libplakar_cdc.so
  run s7_$r v_s7.so
  run s8_$r v_s8.so
done
head -14 $O/s6_1_trace.txt
echo done
