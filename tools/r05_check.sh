#!/bin/bash
# round 5: full GPU suite, then the driver's command, C3 and c4b lines
O=gpurun_out/$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv.json 2>$O/drv_err.txt || { echo "driver bench failed"; tail $O/drv_err.txt; exit 1; }
python -c "import json;d=json.loads(open('$O/drv.json').read().strip().splitlines()[-1]);print('driver', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity_vs_oracle']); print('digest', json.dumps(d.get('chunk_digests'))[:900])"
timeout -k 10 300 python bench.py --workload c4b > $O/c4b.json 2>$O/c4b_err.txt || { echo "c4b failed"; tail $O/c4b_err.txt; exit 1; }
python -c "import json;d=json.loads(open('$O/c4b.json').read().strip().splitlines()[-1]);print('c4b', d['value'], json.dumps(d['roofline'])[:700])"
