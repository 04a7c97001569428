#!/bin/bash
O=gpurun_out/${1:-r03chk}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c4b.json 2> $O/bench_c4b.err || exit 1
cut -c1-120 $O/bench_c4b.json
