#!/bin/bash
# Rehearse bench.py's N-rank path on a one-GPU box (all ranks on device 0, gloo).
set -e
OUT=gpurun_out/rehearse; mkdir -p $OUT
for n in 2 4; do
  BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 50 --warmup 50 \
    > $OUT/n$n.json 2> $OUT/n$n.err
  tail -1 $OUT/n$n.json | cut -c1-400
done
