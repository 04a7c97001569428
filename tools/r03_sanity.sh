#!/bin/bash
O=gpurun_out/r03sanity; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_bench.json 2> $O/driver_bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/driver_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['encode']['value'], d['chunk_digests']['value'])"
