"""Pipelined stress: thousands of launch groups over two streams (bench.py's
pattern: one group's resolution beside the next group's scan), every pass's
cut lists and result rows compared on the device with the oracle's.

A race in the resolver's hand-offs (speculative exits, LOCAL / INCLUSIVE
statuses, the look-back windows, the per-launch tickets and zeroed granules)
would show as one wrong pass among many; a one-pass test can miss it.  The
adaptive MaskL index switches kernels between groups on the low-entropy
buffer (k_scan, k_maskl_probe, k_scan_f), so those transitions are stressed
too.  PARITY UNPINNED w.r.t. the Go module.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from datagen import gear_table, low_entropy, random_bytes  # noqa: E402
from plakar_amd import _lib, chunkers, device  # noqa: E402

pytestmark = pytest.mark.gpu

DEF = dict(min_size=65536, normal_size=1 << 20, max_size=4 << 20)


@pytest.fixture(autouse=True)
def _restore():
    yield
    device.set_maskl_index_mode(1)
    _lib.ensure_init(gear=_lib.default_gear())


def _run(oracle, arrays, p, gear, passes):
    _lib.ensure_init(gear=gear)
    device.set_maskl_index_mode(1)
    refs = [torch.from_numpy(oracle.chunk(a, gear, **p).astype(np.int64)).cuda() for a in arrays]
    ts = [torch.from_numpy(a).cuda() for a in arrays]
    opts = chunkers.ChunkerOpts(MinSize=p["min_size"], NormalSize=p["normal_size"], MaxSize=p["max_size"])
    batches = [device.DeviceBatch(ts, opts) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    errs = [torch.zeros((), dtype=torch.int64, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    for i in range(passes):
        k = i % 2
        b, s = batches[k], streams[k]
        with torch.cuda.stream(s):
            b.res.zero_()  # nothing of the previous pass on this workspace can pass for this one
            for c in b.cuts:
                c.zero_()
            b.launch(s)
            for j, r in enumerate(refs):
                n = r.shape[0]
                row = b.res[j]
                bad = (row[0] != n) | (row[1] != ts[j].numel()) | (row[2] != 0)
                c = b.cuts[j][:n]
                bad = bad | (c[:, 0] != r[:, 0]).any() | ((c[:, 1] & 0xFFFFFFFF) != r[:, 1]).any()
                errs[k] += bad.to(torch.int64)
    torch.cuda.synchronize()
    # the check itself catches a wrong list: one more pass against a reference
    # whose last row is off by one
    bad_ref = refs[0].clone()
    bad_ref[-1, 1] += 1
    b = batches[0]
    b.launch(streams[0])
    torch.cuda.synchronize()
    c = b.cuts[0][:bad_ref.shape[0]]
    assert bool(((c[:, 0] != bad_ref[:, 0]).any() | ((c[:, 1] & 0xFFFFFFFF) != bad_ref[:, 1]).any()).item())
    return [int(e) for e in errs]


def test_pipelined_passes_all_exact(oracle):
    """2,000 passes of a C1-like, a C3-like and four small buffers."""
    arrays = [random_bytes(192 << 20, 11), low_entropy(96 << 20, 12), random_bytes(3 << 20, 13),
              np.zeros(5 << 20, np.uint8), random_bytes(65537, 14), low_entropy(7 << 20, 15, 0.05)]
    errs = _run(oracle, arrays, DEF, _lib.default_gear(), 2000)
    assert errs == [0, 0], f"wrong (pass, buffer) results per stream: {errs}"


def test_pipelined_small_chunks(oracle):
    """Small chunks (many cuts per segment, long look-back chains): 1,000
    passes, random Gear table, 4 KiB / 16 KiB / 64 KiB."""
    p = dict(min_size=4096, normal_size=16384, max_size=65536)
    arrays = [random_bytes(64 << 20, 21), low_entropy(32 << 20, 22, 0.02), random_bytes(1 << 20, 23)]
    errs = _run(oracle, arrays, p, gear_table(24), 1000)
    assert errs == [0, 0], f"wrong (pass, buffer) results per stream: {errs}"
