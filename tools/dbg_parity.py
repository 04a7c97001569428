"""Debug helper: GPU vs oracle on one buffer under several scan-lane sizes and
debug modes.  python tools/dbg_parity.py [size_mib] [seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

from datagen import random_bytes
from oracle_ref import Oracle
from plakar_amd import _lib, chunkers, device

size = int(sys.argv[1]) << 20 if len(sys.argv) > 1 else 64 << 20
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
_lib.ensure_init()
opts = chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20)
data = random_bytes(size, seed)
ref = Oracle().chunk(data, _lib.default_gear())
t = torch.from_numpy(data).cuda()
for lane in ["", "512", "1024", "2048", "5632", "8192"]:
    for mode in [0, 1]:
        if lane:
            os.environ["CDC_SCAN_LANE_BYTES"] = lane
        device.set_debug_mode(mode)
        (c,) = device.chunk_device([t], opts)
        got = c.cpu().numpy().astype(np.uint64)
        ok = got.shape == ref.shape and bool((got == ref).all())
        first = None
        if not ok:
            n = min(len(got), len(ref))
            bad = np.nonzero((got[:n] != ref[:n]).any(axis=1))[0]
            first = (int(bad[0]), got[bad[0]].tolist(), ref[bad[0]].tolist()) if bad.size else ("len", len(got), len(ref))
        print(f"lane={lane or 'auto':5s} mode={mode} n={len(got)} ref={len(ref)} ok={ok} first_bad={first}", flush=True)
device.set_debug_mode(0)
