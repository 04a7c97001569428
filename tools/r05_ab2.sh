#!/bin/bash
# Round 5 A/Bs: k_resolve with 8-wave workgroups (two waves per SIMD, half the CUs held) vs 4; the backup's
# CU-masked digest streams vs unmasked; C2 Encode per call under a kernel + copy trace; c4bl with its
# pipeline trace.   tools/r05_ab2.sh <tag>
O=gpurun_out/${1:-r05ab2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/v_ww8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or sizes or sweep or pipelined or c1_full or c2_shape or c3" > $O/pytest_ww8.txt 2>&1 || { echo "ww8 parity failed"; tail -20 $O/pytest_ww8.txt; exit 1; }
tail -1 $O/pytest_ww8.txt
drv() {  # name lib extra
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 timeout -k 10 200 python bench.py --gpus 1 $3 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/$1.json 2>>$O/err.txt || { echo "$1 failed"; tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);print('$1', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('pipeline_avg_ms'), d['parity_vs_oracle'])"
}
for r in 1 2 3; do
  drv drv_base_$r libplakar_cdc.so "--steps 20 --warmup 5"
  drv drv_ww8_$r v_ww8.so "--steps 20 --warmup 5"
done
drv warm_base libplakar_cdc.so ""
drv warm_ww8 v_ww8.so ""
c4b() {  # name env
  env $2 timeout -k 10 300 python bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/$1.json 2>>$O/err.txt || { echo "$1 failed"; tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);s=d['backup_stages'];print('$1', d['value'], s['wall_s'], s['device_s'], s['read_wait_s'])"
}
for r in 1 2 3; do
  c4b c4b_mask_$r CDC_BACKUP_DIGEST_CUS=half
  c4b c4b_all_$r CDC_BACKUP_DIGEST_CUS=all
done
echo "[encode C2 per call, kernel + copy trace]"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/enc_trace -o run -- \
    python3 tools/encode_reps.py --workload c2 --reps 12 > $O/enc_reps.txt 2> $O/enc_reps.err || { echo "encode trace failed"; tail $O/enc_reps.err; exit 1; }
cat $O/enc_reps.txt
echo "[c4bl with its pipeline trace]"
CDC_BACKUP_TRACE=$O/c4bl_trace.csv timeout -k 10 600 python bench.py --workload c4bl --steps 2 --warmup 1 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/c4bl.json 2>>$O/err.txt || { echo "c4bl failed"; tail $O/err.txt; exit 1; }
python tools/backup_trace.py $O/c4bl_trace.csv > $O/c4bl_trace.txt 2>&1 || true
head -30 $O/c4bl_trace.txt
echo done
