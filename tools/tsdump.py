"""Per-phase device timestamps of one launch group (debug build knob).

    CDC_DEBUG_PHASE=16 python tools/tsdump.py [--size-mib 1024] [--workload c1]

Runs the device path with B.debug & 16, which makes the kernels record
s_memrealtime (100 MHz) at phase boundaries, then prints where the time of
the last launch went: scan workgroups, then per-segment walk phases, then
k_emit phases.  Times are in us, relative to the first scan workgroup start.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

K_SCAN, K_W1 = 0, 4 * 4096
K_MAXSEGS = 16384
K_W2 = K_W1 + 8 * K_MAXSEGS
K_EMIT = K_W2 + 8 * K_MAXSEGS
K_SLOTS = K_EMIT + 16


def pct(a, qs=(0, 50, 90, 100)):
    if len(a) == 0:
        return "-"
    return " ".join(f"p{q}={np.percentile(a, q):7.1f}" for q in qs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-mib", type=int, default=1024)
    ap.add_argument("--workload", default="c1")
    ap.add_argument("--warm", type=int, default=300, help="launches before the recorded one (clock ramp)")
    args = ap.parse_args()
    os.environ.setdefault("CDC_DEBUG_PHASE", "16")
    import torch

    from bench import WORKLOADS, make_buffers
    from plakar_amd import _lib, chunkers, device

    _lib.ensure_init()
    L = _lib.lib()
    L.cdc_debug_timestamps.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
    L.cdc_debug_timestamps.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    bufs = make_buffers(torch, WORKLOADS[args.workload], 0, dev, args.size_mib << 20)
    b = device.DeviceBatch(bufs, chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20))
    for _ in range(max(1, args.warm)):
        b.launch()
    torch.cuda.synchronize()
    ts = np.zeros(K_SLOTS, dtype=np.uint64)
    assert L.cdc_debug_timestamps(ts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), K_SLOTS) == 0
    ts = ts.astype(np.int64)
    scan = ts[K_SCAN:K_W1].reshape(-1, 4)
    scan = scan[scan[:, 0] > 0]
    t0 = scan[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # 100 MHz
    print(f"scan WGs {len(scan)}: start {pct(us(scan[:, 0]))}")
    print(f"  fill done {pct(us(scan[:, 1]))}")
    print(f"  wave0 end {pct(us(scan[:, 2]))}")
    idx = np.nonzero(ts[K_SCAN:K_W1].reshape(-1, 4)[:, 0] > 0)[0]
    for x in range(8):  # blockIdx % 8 ~ XCD
        sel = (idx % 8) == x
        print(f"    blk%8={x}: end {pct(us(scan[sel, 2]), (0, 50, 100))}")
    nseg = int(np.count_nonzero(ts[K_W1:K_W2].reshape(-1, 8)[:, 3]))
    w1 = ts[K_W1:K_W2].reshape(-1, 8)[:nseg]
    w2 = ts[K_W2:K_EMIT].reshape(-1, 8)[:nseg]
    print(f"walk1 segs {nseg}: start {pct(us(w1[:, 0]))}")
    print(f"  fill done {pct(us(w1[:, 1]))}")
    print(f"  1st node / preload done {pct(us(w1[:, 2]))}")
    if w1[:, 5].max() > 0:
        print(f"  1st spec loop done  {pct(us(w1[:, 7]))}")
        print(f"  1st spec round done {pct(us(w1[:, 5]))}   rounds {pct(w1[:, 6])}")
    print(f"  end       {pct(us(w1[:, 3]))}")
    print(f"  per-wave (end - fill) {pct((w1[:, 3] - w1[:, 1]) / 100.0)}  nodes {pct(w1[:, 4])}")
    ok = w2[:, 3] > 0
    print(f"walk2 start {pct(us(w2[:, 0]))}")
    print(f"  fill done {pct(us(w2[:, 1]))}")
    print(f"  end       {pct(us(w2[ok, 3]))}")
    print(f"  per-wave (end - fill) {pct((w2[ok, 3] - w2[ok, 1]) / 100.0)}  steps {pct(w2[ok, 4])}")
    e = ts[K_EMIT:K_SLOTS]
    names = ["start", "ph1 done", "ph2 done", "ph3 loads", "ph3 scan", "end"]
    print("emit " + "  ".join(f"{n}={us(e[i]):.1f}" for i, n in enumerate(names)) +
          f"  nontrivial={e[8]} intervals={e[9]}")


if __name__ == "__main__":
    main()
