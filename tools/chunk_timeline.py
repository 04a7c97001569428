"""Round 5: where a k_chunk launch's time goes (CDC_DEBUG_PHASE=16 stamps).

After --warm launches (single stream), one launch of C1 (1 GiB random) with
s_memrealtime stamps (100 MHz): per scan task (start, end, wave, where), per
resolution segment (start, graph built, speculative exit, look-back done,
INCLUSIVE).  Prints percentiles relative to the first task's start.  With
CDC_RESOLVE_MODE=0 the scan tasks are k_scan's (no per-task stamps) and the
segments k_resolve's.
Usage: CDC_DEBUG_PHASE=16 python tools/chunk_timeline.py [--warm N] [--mib M]"""
import argparse
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

K_RES = 4 * 4096
K_CLK = K_RES + 8 * 16384
K_CLKN = K_CLK + 4 * 4096
K_HW = K_CLKN + 1
K_ABORT = K_HW + 4096
K_TASK = K_ABORT + 4
K_SLOTS = K_TASK + 4 * 8192


def pct(x, qs=(0, 10, 50, 90, 100)):
    x = np.asarray(x, dtype=np.float64)
    if x.size == 0:
        return "-"
    return " ".join(f"p{q}={np.percentile(x, q):.1f}" for q in qs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", type=int, default=20)
    ap.add_argument("--mib", type=int, default=1024)
    args = ap.parse_args()
    _lib.ensure_init()
    L = _lib.lib()
    L.cdc_debug_timestamps.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
    t = torch.from_numpy(random_bytes(args.mib << 20, 1)).cuda()
    b = device.DeviceBatch([t], chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * (args.warm + 1))]
    for k in range(args.warm + 1):
        ev[2 * k].record()
        b.launch()
        ev[2 * k + 1].record()
    torch.cuda.synchronize()
    ms = [ev[2 * k].elapsed_time(ev[2 * k + 1]) for k in range(args.warm + 1)]
    print(f"launches (ms, single stream): first {ms[0]:.3f}  last 5 {[round(x, 3) for x in ms[-5:]]}")
    ts = np.zeros(K_SLOTS, dtype=np.uint64)
    assert L.cdc_debug_timestamps(ts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), K_SLOTS) == 0
    ts = ts.astype(np.int64)
    tk = ts[K_TASK:K_TASK + 4 * 8192].reshape(-1, 4)
    tk = tk[tk[:, 0] > 0]
    r = ts[K_RES:K_RES + 8 * 16384].reshape(-1, 8)
    r = r[r[:, 4] > 0]
    if len(tk):
        t0 = tk[:, 0].min()
    elif len(r):
        t0 = r[:, 0].min()
    else:
        print("no stamps")
        return
    us = lambda x: (x - t0) / 100.0
    if len(tk):
        print(f"scan tasks {len(tk)}: start {pct(us(tk[:, 0]))}")
        print(f"  end {pct(us(tk[:, 1]))}")
        print(f"  duration {pct((tk[:, 1] - tk[:, 0]) / 100.0)}")
        for tier in range(3):
            sel = (tk[:, 2] // 4) == tier
            if sel.any():
                print(f"  tier {tier} (waves {4 * tier}-{4 * tier + 3}): {int(sel.sum())} tasks, end {pct(us(tk[sel, 1]))}")
    if len(r) == 0:
        print(f"no segment stamps; last scan task end {us(tk[:, 1].max()) if len(tk) else float('nan'):.1f} us")
        return
    print(f"segments {len(r)}: start {pct(us(r[:, 0]))}")
    third = len(r) // 3
    for k in range(3):
        sel = slice(k * third, (k + 1) * third if k < 2 else len(r))
        rr = r[sel]
        print(f"  segments {k}/3: start {pct(us(rr[:, 0]), (50, 100))}  built {pct(us(rr[:, 1]), (50, 100))}  "
              f"inclusive {pct(us(rr[:, 4]), (50, 100))}")
    print(f"  graph built {pct(us(r[:, 1]))}   (built - start) {pct((r[:, 1] - r[:, 0]) / 100.0)}")
    print(f"  spec exit {pct(us(r[:, 2]))}   (- built) {pct((r[:, 2] - r[:, 1]) / 100.0)}")
    lb = r[1:, 3]
    print(f"  look-back done {pct(us(lb))}   (- spec) {pct((lb - r[1:, 2]) / 100.0)}")
    print(f"  inclusive {pct(us(r[:, 4]))}   per wave (end - start) {pct((r[:, 4] - r[:, 0]) / 100.0)}")
    last = r[:, 4].max()
    print(f"last INCLUSIVE at {us(last):.1f} us; last scan task end {us(tk[:, 1].max()) if len(tk) else float('nan'):.1f} us")
    a = ts[K_ABORT:K_ABORT + 4]
    if a[0]:
        print("ABORT:", a.tolist())


if __name__ == "__main__":
    main()
