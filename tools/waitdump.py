"""Scan diagnostics of a build-time variant library (PLAKAR_CDC_LIB):
the isolated scan / pass time after `--warm` single-stream launches, and,
for a -DCDC_DIAG_WAITS build, the share of each wave's task spent in the
per-stage DMA waits (shader cycles, s_memtime).

    PLAKAR_CDC_LIB=plakar_amd/_lib/var_waits.so python tools/waitdump.py --warm 5
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
K_RES = 4 * 4096
K_SLOTS = K_RES + 8 * 16384 + 4 * 4096 + 1 + 4096


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", type=int, default=5)
    ap.add_argument("--timed", type=int, default=20)
    ap.add_argument("--workload", default="c1")
    ap.add_argument("--waits", action="store_true")
    ap.add_argument("--save", default=None, help="write the per-task records (.npy)")
    args = ap.parse_args()
    import torch

    from bench import WORKLOADS, make_buffers
    from plakar_amd import _lib, chunkers, device

    _lib.ensure_init()
    L = _lib.lib()
    L.cdc_debug_timestamps.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
    L.cdc_debug_timestamps.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    wl = WORKLOADS[args.workload]
    bufs = make_buffers(torch, wl, 0, dev, wl["size"] if "size" in wl else 1 << 30)
    b = device.DeviceBatch(bufs, chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20))
    for _ in range(max(1, args.warm)):
        b.launch()
    torch.cuda.synchronize()
    L.cdc_profile_collect(None, None, None, None)
    L.cdc_profile_enable(1)
    for _ in range(args.timed):
        b.launch()
    torch.cuda.synchronize()
    L.cdc_profile_enable(0)
    s, p = ctypes.c_double(), ctypes.c_double()
    n, by = ctypes.c_uint64(), ctypes.c_uint64()
    L.cdc_profile_collect(ctypes.byref(s), ctypes.byref(p), ctypes.byref(n), ctypes.byref(by))
    print(f"warm {args.warm}: scan {s.value / n.value * 1e3:.1f} us, pass {p.value / n.value * 1e3:.1f} us "
          f"({n.value} launches, {by.value / n.value / 2**30:.3f} GiB each)")
    if args.waits:
        ts = np.zeros(K_SLOTS, dtype=np.uint64)
        assert L.cdc_debug_timestamps(ts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), K_SLOTS) == 0
        r = ts[K_RES:K_RES + 8 * 16384].astype(np.int64).reshape(-1, 8)
        r = r[r[:, 1] > 0]
        if args.save:
            np.save(args.save, r)
        w, t = r[:, 0], r[:, 1]
        f = w / t
        print(f"  tasks {len(r)}: task cycles p50 {np.median(t):.0f} p90 {np.percentile(t, 90):.0f}; "
              f"DMA-wait cycles p50 {np.median(w):.0f}; wait share p10 {np.percentile(f, 10):.3f} "
              f"p50 {np.median(f):.3f} p90 {np.percentile(f, 90):.3f}")
        hw = r[:, 4]
        fields = {"wave_slot": hw & 0xF, "simd": (hw >> 4) & 3, "cu": (hw >> 8) & 0xF, "se": (hw >> 13) & 7,
                  "xcc": r[:, 5] & 0xF, "wave": r[:, 7], "rechecks": np.minimum(r[:, 6] // 4, 8) * 4}
        t0 = r[:, 2] - r[:, 2].min()
        print(f"  start spread (10 ns): p50 {np.median(t0):.0f} p90 {np.percentile(t0, 90):.0f} "
              f"max {t0.max()}; end p50 {np.median(r[:, 3] - r[:, 2].min()):.0f} max {(r[:, 3] - r[:, 2].min()).max()}")
        for name, v in fields.items():
            rows = []
            for k in np.unique(v):
                m = v == k
                rows.append(f"{k}:{np.median(t[m]) / 1e3:.0f}/{np.percentile(t[m], 90) / 1e3:.0f}K(n{m.sum()})")
            print(f"  by {name}: " + " ".join(rows))
        # rank of the wave's start within its SIMD (by s_memrealtime) in its workgroup
        cyc_by_rank = {}
        key = (r[:, 5] & 0xF) * 4096 + ((hw >> 8) & 0xFF) * 8 + ((hw >> 4) & 3)
        for k in np.unique(key):
            idx = np.where(key == k)[0]
            order = idx[np.argsort(r[idx, 2], kind="stable")]
            for j, i in enumerate(order):
                cyc_by_rank.setdefault(j, []).append(t[i])
        print("  by start rank on its SIMD: " + " ".join(
            f"{j}:{np.median(v) / 1e3:.0f}/{np.percentile(v, 90) / 1e3:.0f}K(n{len(v)})" for j, v in sorted(cyc_by_rank.items())))

if __name__ == "__main__":
    main()
