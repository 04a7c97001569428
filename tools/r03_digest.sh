#!/bin/bash
# Digest launch groups past 32 buffers: tests, then the C1 / C2 digest legs.
O=gpurun_out/${1:-r03d}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_digest.py tests/test_entropy.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for w in c1 c2; do
  timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 20 --no-cpu-baseline --e2e-reps 0 --encode-reps 0 > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], json.dumps(d.get('chunk_digests')))"
done
