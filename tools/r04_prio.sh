#!/bin/bash
# k_resolve on a high-priority stream (CDC_RESOLVE_PRIO=1): parity tests with it on, then the driver's command A/B, interleaved.
O=gpurun_out/${1:-r04prio}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CDC_RESOLVE_PRIO=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in 0 1; do
    CDC_RESOLVE_PRIO=$v timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0 > $O/p${v}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$O/p${v}_$r.json').read().strip().splitlines()[-1]); print('prio $v run $r', d['value'], d['ms_per_step'], d['parity_vs_oracle'])"
  done
done
