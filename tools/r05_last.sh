#!/bin/bash
# Round 5, last check on the final tree: GPU suite, smoke, the driver's command.
O=gpurun_out/${1:-r05last}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_bench.json 2> $O/driver_bench.err || { tail $O/driver_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/driver_bench.json').read().strip().splitlines()[-1]);r=d['roofline'];print('driver', d['value'], d['ms_per_step'], r['frac'], r.get('frac_of_measured_peak'), d['parity_vs_oracle'])"
echo done
