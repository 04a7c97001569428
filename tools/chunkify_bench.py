"""Batched chunkify (snapshot.chunkify_batch) on a C4-like corpus: files in
host memory -> objects.Object records (cuts, chunk SHA-256, counts, entropy,
object SHA-256).  Reports the end-to-end GiB/s and its parts.
    python tools/chunkify_bench.py [nfiles] [batch_mib]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

from datagen import zipf_sizes
from plakar_amd import _lib, snapshot

nfiles = int(sys.argv[1]) if len(sys.argv) > 1 else 512
batch = (int(sys.argv[2]) if len(sys.argv) > 2 else 1024) << 20
_lib.ensure_init()
sizes = zipf_sizes(nfiles, 300)
rng = np.random.default_rng(300)
files = [rng.integers(0, 256, int(s), dtype=np.uint8) for s in sizes]
total = sum(int(s) for s in sizes)
print(f"{nfiles} files, {total / 2**30:.2f} GiB, largest {max(sizes) / 2**20:.1f} MiB", flush=True)
# batches of about `batch` bytes, files in order
groups, cur, acc = [], [], 0
for f in files:
    cur.append(f)
    acc += f.size
    if acc >= batch:
        groups.append(cur)
        cur, acc = [], 0
if cur:
    groups.append(cur)
snapshot.chunkify_batch(groups[0][:4])  # warm-up
torch.cuda.synchronize()
t0 = time.perf_counter()
nchunks = 0
for g in groups:
    objs = snapshot.chunkify_batch(g)
    nchunks += sum(len(o.Chunks) for o in objs)
dt = time.perf_counter() - t0
print(f"chunkify_batch: {total / dt / 2**30:.2f} GiB/s end to end ({dt:.2f} s, {len(groups)} batches, "
      f"{nchunks} chunks)", flush=True)
