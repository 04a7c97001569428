"""Per-phase device timestamps of one launch group (debug build knob).

    CDC_DEBUG_PHASE=16 python tools/tsdump.py [--size-mib 1024] [--workload c1]

Runs the device path with B.debug & 16, which makes the kernels record
s_memrealtime (100 MHz) at phase boundaries, then prints where the time of
the last launch went: scan workgroups, then the per-segment phases of k_resolve.  Times are in us, relative to the first scan workgroup start.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

K_SCAN, K_RES = 0, 4 * 4096
K_HW = K_RES + 8 * 16384 + 4 * 4096 + 1
K_SLOTS = K_HW + 4096


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
    scan = ts[K_SCAN:K_RES].reshape(-1, 4)
    scan = scan[scan[:, 0] > 0]
    r0 = ts[K_RES:K_RES + 8 * 16384].reshape(-1, 8)
    t0 = scan[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # 100 MHz
    print(f"scan WGs {len(scan)}: start {pct(us(scan[:, 0]))}")
    print(f"  fill done {pct(us(scan[:, 1]))}")
    print(f"  wave0 end {pct(us(scan[:, 2]))}")
    print(f"  wave1 end {pct(us(scan[:, 3]))}   |wave0 - wave1| {pct(np.abs(scan[:, 2] - scan[:, 3]) / 100.0)}")
    print(f"  duration (wave0 end - start) {pct((scan[:, 2] - scan[:, 0]) / 100.0)}")
    hw = ts[K_HW:K_HW + len(scan)]
    xcc = (hw >> 32) & 0xF
    hwid = hw & 0xFFFFFFFF
    cu = (hwid >> 8) & 0xF
    se = (hwid >> 13) & 0x7
    sh = (hwid >> 12) & 0x1
    end = us(scan[:, 2])
    for x in range(8):
        sel = xcc == x
        if sel.any():
            print(f"    xcc {x}: {int(sel.sum())} WGs, end {pct(end[sel], (0, 50, 100))}")
    for e in range(int(se.max()) + 1):
        sel = se == e
        if sel.any():
            print(f"    se {e}: {int(sel.sum())} WGs, end {pct(end[sel], (0, 50, 100))}")
    order = np.argsort(end)
    print("  earliest WGs (blk xcc se sh cu end):", [(int(i), int(xcc[i]), int(se[i]), int(sh[i]), int(cu[i]), round(float(end[i]), 1)) for i in order[:6]])
    print("  latest WGs:", [(int(i), int(xcc[i]), int(se[i]), int(sh[i]), int(cu[i]), round(float(end[i]), 1)) for i in order[-6:]])
    idx = np.nonzero(ts[K_SCAN:K_RES].reshape(-1, 4)[:, 0] > 0)[0]
    for x in range(8):  # blockIdx % 8 ~ XCD
        sel = (idx % 8) == x
        print(f"    blk%8={x}: end {pct(us(scan[sel, 2]), (0, 50, 100))}")
    r = ts[K_RES:K_RES + 8 * 16384].reshape(-1, 8)
    nseg = int(np.count_nonzero(r[:, 4]))
    r = r[:nseg]
    print(f"k_resolve segs {nseg}: start {pct(us(r[:, 0]))}")
    print(f"  graph built {pct(us(r[:, 1]))}   (built - start) {pct((r[:, 1] - r[:, 0]) / 100.0)}")
    print(f"  spec exit published {pct(us(r[:, 2]))}   (- built) {pct((r[:, 2] - r[:, 1]) / 100.0)}")
    lb = r[1:, 3]
    print(f"  look-back done {pct(us(lb))}   (- spec) {pct((lb - r[1:, 2]) / 100.0)}")
    print(f"  inclusive published {pct(us(r[:, 4]))}   per wave (end - start) {pct((r[:, 4] - r[:, 0]) / 100.0)}")
    if os.environ.get("CDC_DEBUG_PHASE") == "48":
        print(f"  graph: records+list {pct((r[:, 5] - r[:, 0]) / 100.0)}  slot0 {pct((r[:, 6] - r[:, 5]) / 100.0)}"
              f"  slot1 {pct((r[r[:, 7] > 0, 7] - r[r[:, 7] > 0, 6]) / 100.0)} ({int((r[:, 7] > 0).sum())} segs)")
        return
    slow = np.argsort(r[:, 2] - r[:, 0])[-4:]
    print("  slowest speculative chains (segment: us, exact calls, listed): " +
          ", ".join(f"{i}: {(r[i, 2] - r[i, 0]) / 100.0:.1f}, {r[i, 6]}, {r[i, 5]}" for i in slow))
    slow8 = np.argsort(r[:, 2])[-8:]
    print("  latest spec exits (segment: start, build us, walk us, exact, listed, exit at): " +
          "; ".join(f"{i}: {us(r[i, 0]):.1f}, {(r[i, 1] - r[i, 0]) / 100.0:.1f}, {(r[i, 2] - r[i, 1]) / 100.0:.1f}, "
                    f"{r[i, 6]}, {r[i, 5]}, {us(r[i, 2]):.1f}" for i in slow8))
    ex = r[:, 6] > 0
    if ex.any():
        print(f"  walk us with exact calls {pct((r[ex, 2] - r[ex, 1]) / 100.0)} ({int(ex.sum())} segs); "
              f"without {pct((r[~ex, 2] - r[~ex, 1]) / 100.0)}")
    lbs = np.argsort(r[:, 3])[-4:]
    print("  latest look-backs (segment: done at us): " + ", ".join(f"{i}: {us(r[i, 3]):.1f}" for i in lbs))
    print(f"  listed nodes {pct(r[:, 5])}   exact next_node() calls {pct(r[:, 6])}   junction nodes {pct(r[:, 7])}")


if __name__ == "__main__":
    main()
