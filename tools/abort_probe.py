"""Debug helper (round 5): run one launch group on the GPU and report a
bounded wait that gave up (g_ts[kTsAbort..], see cdc_kernels.hip SpinGuard).
Usage: python tools/abort_probe.py [size_mib] [resolve_mode]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from datagen import random_bytes  # noqa: E402
from plakar_amd import _lib, chunkers, device  # noqa: E402

K_SCAN = 0
K_RES = 4 * 4096
K_CLK = K_RES + 8 * 16384
K_CLKN = K_CLK + 4 * 4096
K_HW = K_CLKN + 1
K_ABORT = K_HW + 4096
K_SLOTS = K_ABORT + 4
KINDS = {1: "task flags", 2: "junction (later segment's chain)", 3: "previous segment's exit", 4: "look-back",
         5: "look-back slow path", 6: "last segment: every INCLUSIVE"}


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    mode = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    _lib.ensure_init()
    L = _lib.lib()
    L.cdc_debug_timestamps.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
    device.set_resolve_mode(mode)
    t = torch.from_numpy(random_bytes(mib << 20, 1)).cuda()
    b = device.DeviceBatch([t], chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20))
    import time
    t0 = time.time()
    b.launch()
    torch.cuda.synchronize()
    print(f"launch + sync {time.time() - t0:.3f} s", flush=True)
    w = b.workspace.cpu().numpy().view(np.uint32)
    ones = (w == 1).astype(np.int8)
    # the longest run of u32 == 1: the task flags (k_chunk)
    best, cur, end = 0, 0, 0
    for i, v in enumerate(ones):
        cur = cur + 1 if v else 0
        if cur > best:
            best, end = cur, i
    print(f"longest run of u32 == 1 in the workspace: {best} (ends at word {end}); "
          f"the 12 words before it: {w[max(0, end - best - 11):end - best + 1].tolist()}", flush=True)
    r = b.res.cpu().numpy()
    print("result row (ncuts, consumed, status, needed):", r[0].tolist(), flush=True)
    ts = np.zeros(K_SLOTS, dtype=np.uint64)
    assert L.cdc_debug_timestamps(ts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), K_SLOTS) == 0
    kind, a, bb, when = (int(x) for x in ts[K_ABORT:K_ABORT + 4])
    print("abort:", KINDS.get(kind, kind), a, bb, when, flush=True)


if __name__ == "__main__":
    main()
