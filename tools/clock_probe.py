"""Shader clock over a cold run: the scan's workgroup 0 records its span in the
100-MHz counter and in the shader-clock counter (B.debug & 64, a ring of 4096
launches), so the clock each pass ran at is d(memtime) / d(realtime) x 100 MHz.

    python tools/clock_probe.py [--passes 600] [--streams 2] [--bins 25]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

K_CLK = 4 * 4096 + 8 * 16384
K_SLOTS = K_CLK + 4 * 4096 + 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=600)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--bins", type=int, default=25)
    ap.add_argument("--workload", default="c1")
    args = ap.parse_args()
    os.environ["CDC_DEBUG_PHASE"] = "64"
    import torch

    from bench import WORKLOADS, make_buffers
    from plakar_amd import _lib, chunkers, device

    _lib.ensure_init()
    L = _lib.lib()
    L.cdc_debug_timestamps.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
    L.cdc_debug_timestamps.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    wl = WORKLOADS[args.workload]
    bufs = make_buffers(torch, wl, 0, dev, wl["size"])
    opts = chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20)
    batches = [device.DeviceBatch(bufs, opts, final=True) for _ in range(args.streams)]
    streams = [torch.cuda.Stream(dev) for _ in range(args.streams)]
    torch.cuda.synchronize()
    for i in range(args.passes):
        batches[i % args.streams].launch(streams[i % args.streams])
    torch.cuda.synchronize()
    ts = np.zeros(K_SLOTS, dtype=np.uint64)
    assert L.cdc_debug_timestamps(ts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), K_SLOTS) == 0
    n = int(ts[K_SLOTS - 1])
    rec = ts[K_CLK:K_CLK + 4 * min(n, 4096)].astype(np.int64).reshape(-1, 4)
    dur = (rec[:, 2] - rec[:, 0]) / 100.0  # us
    ghz = (rec[:, 3] - rec[:, 1]) / np.maximum(rec[:, 2] - rec[:, 0], 1) / 10.0
    t0 = rec[0, 0]
    print(f"{n} scan launches recorded; streams {args.streams}")
    print("passes       t_ms   wg0_us   sclk_GHz(avg min max)")
    for b0 in range(0, len(rec), args.bins):
        sl = slice(b0, b0 + args.bins)
        print(f"{b0:5d}-{min(len(rec), b0 + args.bins) - 1:<5d} {(rec[b0, 0] - t0) / 1e5:6.2f} {dur[sl].mean():8.1f}   "
              f"{ghz[sl].mean():.3f} {ghz[sl].min():.3f} {ghz[sl].max():.3f}")


if __name__ == "__main__":
    main()
