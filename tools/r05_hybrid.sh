#!/bin/bash
# Round 5: the hybrid digest split with a calibrated host rate and overlapped copies -- tests and the C1/C2/C3 digest legs.
O=gpurun_out/${1:-r05hy}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_digest.py -x -q --timeout 200 --timeout-method thread -k hybrid > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for w in c1 c2 c3; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --encode-reps 0 --e2e-reps 0 > $O/$w.json 2>>$O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/$w.json').read().strip().splitlines()[-1]);c=d['chunk_digests'];h=c['hybrid'];print('$w', 'device', c['value'], c['ms_per_pass'], 'hybrid', h['value'], h['ms_per_pass'], h['host_chunks'], h['host_bytes'], h['equal_to_device_only'], c['parity_vs_hashlib'])"
done
echo done
