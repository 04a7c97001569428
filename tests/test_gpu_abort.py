"""The device-abort path: a bounded wait that gives up surfaces as an error.

SURVEY.md section 5: a chunker failure must reach the caller as an error
(the reference's backup aborts on one, /root/reference/snapshot/backup.go:98-101),
never as a hung device.  Every spin of k_resolve is bounded (SpinGuard,
cdc_kernels.hip).  Debug mode 2 (cdc_set_debug_mode) makes one wait
unsatisfiable -- segment 0 of the launch group's first buffer never publishes
its speculative exit -- and shortens the spin limit to 200 us, so segment 1's
wait for it gives up.  The checks: every result row of the launch group reports
CDC_E_DEVICE, the host API returns the error instead of hanging, the abort
record names the wait that gave up, and the next launch on the same device is
bit-exact against the oracle again (the scan kernel clears the abort word).
"""
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from datagen import low_entropy, random_bytes  # noqa: E402
from plakar_amd import _lib, chunkers, device  # noqa: E402
from test_gpu_parity import DEF, _opts, _placeholder, assert_same, gpu_chunk  # noqa: E402

pytestmark = pytest.mark.gpu

CDC_E_DEVICE = -4
# g_ts slots (cdc_kernels.hip): kTsRes = 4 * 4096, kTsClk = kTsRes + 8 * 16384,
# kTsClkN = kTsClk + 4 * 4096, kTsHw = kTsClkN + 1, kTsAbort = kTsHw + 4096
K_TS_ABORT = 4 * 4096 + 8 * 16384 + 4 * 4096 + 1 + 4096
# kinds of waits (cdc_kernels.hip): 3 the junction's wait for the previous
# segment's exit (the withheld one), 4 / 5 a look-back waiting on it
K_WAITS = (3, 4, 5)


def _device_batch(arrays):
    _lib.ensure_init(gear=_placeholder(), cut_convention=0)
    ts = []
    for a in arrays:
        t = torch.empty(a.size, dtype=torch.uint8, device="cuda")
        t.copy_(torch.from_numpy(np.ascontiguousarray(a)))
        ts.append(t)
    return device.DeviceBatch(ts, _opts(DEF))


def _abort_record():
    import ctypes
    n = K_TS_ABORT + 4
    buf = (ctypes.c_uint64 * n)()
    _lib.check(_lib.lib().cdc_debug_timestamps(buf, n), "timestamps")
    return [int(buf[K_TS_ABORT + i]) for i in range(4)]


@pytest.mark.parametrize("maskl_mode", [1, 2], ids=["k_scan", "k_scan_f"])
def test_forced_abort_reports_device_error(oracle, maskl_mode):
    data = [random_bytes(16 << 20, 90), low_entropy(6 << 20, 91), random_bytes(1 << 20, 92),
            np.zeros(0, dtype=np.uint8)]
    device.set_maskl_index_mode(maskl_mode)
    device.set_debug_mode(2)
    try:
        b = _device_batch(data)
        t0 = time.time()
        b.launch()
        torch.cuda.synchronize()
        dt = time.time() - t0
        rows = b.res.cpu().numpy()
        assert (rows[:, 2] == CDC_E_DEVICE).all(), f"rows {rows[:, 2]}"
        assert dt < 5.0, f"the aborted launch took {dt:.2f} s"
        with pytest.raises(_lib.CdcError) as e:
            b.results()
        assert e.value.status == CDC_E_DEVICE
        rec = _abort_record()
        assert rec[0] in K_WAITS and rec[3] > 0, f"abort record {rec}"
        # the host batch API (cdc_chunk) returns the error, it does not hang
        t0 = time.time()
        with pytest.raises(_lib.CdcError) as e:
            chunkers.ChunkBuffers([data[0]], _opts(DEF))
        assert e.value.status == CDC_E_DEVICE
        assert time.time() - t0 < 10.0
    finally:
        device.set_debug_mode(0)
        device.set_maskl_index_mode(1)
    # the next launch on the same device: clean abort word, bit-exact
    gear = _placeholder()
    got, res = gpu_chunk(data, DEF, gear=gear)
    assert (res.numpy()[:, 2] == 0).all()
    for g, a in zip(got, data):
        assert_same(g, oracle.chunk(a, gear, **DEF), "after the abort")


def test_abort_needs_two_segments(oracle):
    """A launch group whose first buffer has one segment has no wait to
    withhold: debug mode 2 then changes nothing (bit-exact)."""
    data = [random_bytes(512 << 10, 93)]
    gear = _placeholder()
    device.set_debug_mode(2)
    try:
        got, res = gpu_chunk(data, DEF, gear=gear)
    finally:
        device.set_debug_mode(0)
    assert_same(got[0], oracle.chunk(data[0], gear, **DEF), "one segment")
