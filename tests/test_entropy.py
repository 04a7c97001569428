"""Device entropy() (cdc_chunk_entropy_device_async, k_chunk_entropy) against
the host restatement of snapshot/backup.go:548-569 with Go's math.Log2
(plakar_amd.hashing.entropy_rows / entropy_from_freq): equal floats, row by
row (the device folds the 256 terms in the reference's bin order).  Go itself
is absent here, so agreement with Go's own floats stays unpinned, as for the
host path."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from datagen import low_entropy, random_bytes  # noqa: E402
from plakar_amd import hashing  # noqa: E402

pytestmark = pytest.mark.gpu


def _rows():
    rng = np.random.default_rng(5)
    rows = []
    # histograms of real chunk shapes: uniform bytes, low entropy, text-like
    for n in (1, 2, 3, 255, 256, 257, 4096, 65536, 1 << 20, (1 << 24) + 12345):
        rows.append(np.bincount(random_bytes(n, n).astype(np.int64), minlength=256))
        rows.append(np.bincount(low_entropy(n, n + 1).astype(np.int64), minlength=256))
    # a single bin (p = 1: Log2 = 0), two equal bins (p = 1/2: frac == 0.5),
    # powers of two everywhere, one byte among many
    for b in (0, 7, 255):
        r = np.zeros(256, np.int64)
        r[b] = 1000
        rows.append(r)
    r = np.zeros(256, np.int64)
    r[[3, 200]] = 4096
    rows.append(r)
    rows.append(np.full(256, 64, np.int64))
    r = np.zeros(256, np.int64)
    r[0], r[1] = (1 << 26) - 1, 1
    rows.append(r)
    rows.append(np.zeros(256, np.int64))  # an empty chunk: 0
    # random sparse and dense rows, bins spanning the Sqrt2/2 split
    for _ in range(300):
        k = int(rng.integers(1, 257))
        r = np.zeros(256, np.int64)
        r[rng.choice(256, k, replace=False)] = rng.integers(1, 1 << int(rng.integers(1, 20)), k)
        rows.append(r)
    return np.stack(rows)


def test_device_entropy_equals_host_restatement():
    rows = _rows()
    lens = rows.sum(1)
    want = hashing.entropy_rows(rows, lens)
    got = hashing.chunk_entropy_device(torch.from_numpy(rows.astype(np.int32)).cuda()).cpu().numpy()
    torch.cuda.synchronize()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5]}: {got[bad[:5]]} vs {want[bad[:5]]}"
    for i in range(0, len(rows), 37):  # the scalar form too
        assert got[i] == hashing.entropy_from_freq(rows[i].tolist(), int(lens[i]))


def test_device_entropy_empty_input():
    out = hashing.chunk_entropy_device(torch.zeros((0, 256), dtype=torch.int32, device="cuda"))
    assert out.shape == (0,)
