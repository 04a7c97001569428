"""Per-chunk SHA-256 (+ histogram) throughput on the device path's cut list.
    python tools/digest_bench.py [size_mib]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch

from bench import WORKLOADS, make_buffers
from plakar_amd import _lib, chunkers, device, hashing

size = (int(sys.argv[1]) if len(sys.argv) > 1 else 1024) << 20
_lib.ensure_init()
bufs = make_buffers(torch, WORKLOADS["c1"], 0, torch.device("cuda", 0), size)
b = device.DeviceBatch(bufs, chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20))
b.launch()
(cuts,), res = b.results()
n = cuts.shape[0]
lens = cuts[:, 1].float()
print(f"{n} chunks, mean {lens.mean().item()/1024:.1f} KiB, max {lens.max().item()/1024:.1f} KiB")
for hist in (False, True):
    for _ in range(2):
        hashing.chunk_digests(bufs[0], cuts, hist=hist)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        hashing.chunk_digests(bufs[0], cuts, hist=hist)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"hist={hist}: {ms:.3f} ms per pass, {size / ms / 1e6 / 1.073741824:.1f} GiB/s")
