#!/bin/bash
# Round 5: the measured stream-read peak -- its GPU test and the C1 lines (driver command, default) that report it.
O=gpurun_out/${1:-r05str}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread -k "stream_read" > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for a in "--steps 20 --warmup 5" ""; do
  timeout -k 10 300 python bench.py --gpus 1 $a --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/c1.json 2>>$O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/c1.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$a', d['value'], r['frac'], r.get('measured_stream_read'), r.get('frac_of_measured_peak'))"
done
echo done
