"""cdc_chunk (host buffers in, cut lists out) from pageable vs pinned host
memory, per call, at 64 MiB and 1 GiB; plus the bare torch H2D copy of the
same bytes.  Run under rocprofv3 --memory-copy-trace to see the copies."""
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from plakar_amd import _lib, chunkers  # noqa: E402

_lib.ensure_init()
opts = chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20)
d = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
for size in (64 << 20, 1 << 30):
    src = np.random.PCG64(5).random_raw(size // 8).view(np.uint8)
    pin = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    pin.numpy()[:] = src
    for name, buf in (("pageable", src), ("pinned", pin.numpy())):
        chunkers.ChunkBuffers([buf], opts)
        ts = []
        for _ in range(10):
            t0 = time.perf_counter()
            chunkers.ChunkBuffers([buf], opts)
            ts.append(time.perf_counter() - t0)
        tc = []
        t = torch.from_numpy(buf) if name == "pageable" else pin
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            d[:size].copy_(t, non_blocking=True)
            torch.cuda.synchronize()
            tc.append(time.perf_counter() - t0)
        print(f"{size >> 20:5d} MiB {name:8s}: cdc_chunk per call ms min {min(ts) * 1e3:.2f} med "
              f"{statistics.median(ts) * 1e3:.2f} max {max(ts) * 1e3:.2f} ({size / min(ts) / 2**30:.1f} GiB/s best); "
              f"torch H2D ms min {min(tc) * 1e3:.2f} med {statistics.median(tc) * 1e3:.2f}", flush=True)
