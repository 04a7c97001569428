"""Candidate-index records of one launch group (diagnostic).

    [PLAKAR_CDC_LIB=<variant.so>] python tools/dump_records.py <out.npy> [size_mib]

Chunks one random buffer with DeviceBatch and saves the run records (the
first region of the workspace, cdc_kernels.hip make_plan: off_runs = 0), then
prints the count distribution (bits 0-7 of each record)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from datagen import random_bytes  # noqa: E402
from plakar_amd import _lib, chunkers, device  # noqa: E402

out = sys.argv[1]
mib = int(sys.argv[2]) if len(sys.argv) > 2 else 256
_lib.ensure_init()
a = random_bytes(mib << 20, 7)
t = torch.from_numpy(a).cuda()
b = device.DeviceBatch([t], chunkers.ChunkerOpts(MinSize=65536, NormalSize=1 << 20, MaxSize=4 << 20))
b.launch()
cuts, _ = b.results()
ws = b.workspace.cpu().numpy()
nruns = 0
# records: u64 per run; the plan's scan lane sets the run count: infer from the cut list's size
recs = ws.view(np.uint64)
# the records region ends where the next region starts (256-B aligned); find the count by the lane length
lane = _lib.lib().cdc_debug_scan_lane() if hasattr(_lib.lib(), "cdc_debug_scan_lane") else None
np.save(out, recs[: (mib << 20) // 512 + 64])
cnt = (recs[: (mib << 20) // 512] & np.uint64(0xFF)).astype(np.int64)
print(out, "chunks", cuts[0].shape[0], "records>0", int((cnt > 0).sum()), "sum count", int(cnt.sum()),
      "dense(>4)", int((cnt > 4).sum()), "max", int(cnt.max()))
