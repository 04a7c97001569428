#!/bin/bash
# k_gcm with two GHASH chains in H^128 and the plaintext loads ahead of the AES: parity, then A/B.
O=gpurun_out/r03gcmp; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
V=$PWD/plakar_amd/_lib/var_gcmp.so
PLAKAR_CDC_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_encode.py tests/test_backup.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest var_gcmp rc=$rc"; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit 1
show() { python3 -c "import json; d=json.load(open('$1')); e=d['encode']; print('$1', json.dumps(e)[:400])"; }
for rep in 1 2; do
  for v in base var_gcmp; do
    lib=""; [ $v != base ] && lib=$V
    for wl in c1 c2; do
      PLAKAR_CDC_LIB=$lib timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --digest-reps 0 --e2e-reps 0 --encode-reps 5 > $O/${v}_$wl.$rep.json 2>>$O/err.txt || exit 1
      show $O/${v}_$wl.$rep.json
    done
  done
done
for v in base var_gcmp; do
  lib=""; [ $v != base ] && lib=$V
  PLAKAR_CDC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 tools/encode_bench.py --size-mib 512 --reps 5 > $O/encbench_$v.txt 2>&1 || exit 1
  tail -4 $O/encbench_$v.txt
  s=$(ls $O/prof_$v/*/run_kernel_stats.csv $O/prof_$v/run_kernel_stats.csv 2>/dev/null | head -1); grep -E "k_gcm|k_lz4_seq|k_xxh" "$s" | cut -c1-120
done
