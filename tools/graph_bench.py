"""Pipelined C1 passes launched eagerly vs replayed from captured HIP graphs
(one graph per stream/workspace): python tools/graph_bench.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch

from bench import WORKLOADS, make_buffers
from plakar_amd import _lib, chunkers, device

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
_lib.ensure_init()
dev = torch.device("cuda", 0)
bufs = make_buffers(torch, WORKLOADS["c1"], 0, dev, 1 << 30)
opts = chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20)
nb = 2
batches = [device.DeviceBatch(bufs, opts) for _ in range(nb)]
streams = [torch.cuda.Stream(dev) for _ in range(nb)]


def run_eager():
    for i in range(steps):
        batches[i % nb].launch(streams[i % nb])


graphs = []
for i in range(nb):
    g = torch.cuda.CUDAGraph()
    batches[i].launch(streams[i])  # warm
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=streams[i]):
        batches[i].launch(streams[i])
    graphs.append(g)


def run_graph():
    for i in range(steps):
        with torch.cuda.stream(streams[i % nb]):
            graphs[i % nb].replay()


ref = None
for name, fn in (("eager", run_eager), ("graph", run_graph), ("eager", run_eager), ("graph", run_graph)):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    cuts, _ = batches[0].results()
    n = int(cuts[0].shape[0])
    ref = n if ref is None else ref
    print(f"{name}: {dt * 1e3:.4f} ms per pass, {(1 << 30) / dt / 2**30:.1f} GiB/s, cuts {n} (same={n == ref})", flush=True)
