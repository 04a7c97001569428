"""Deterministic synthetic inputs (BASELINE.json configs), independent of numpy's
Generator API changes: PCG64.random_raw is a fixed algorithm."""
import numpy as np


def random_bytes(n, seed):
    """Uniform random bytes (C0/C1/C2/C4 content)."""
    words = np.random.PCG64(seed).random_raw((n + 7) // 8)
    return words.view(np.uint8)[:n].copy()


def low_entropy(n, seed, frac=0.01):
    """C3: zeros with ~frac of the positions (uniform, with replacement) set to
    uniform random bytes."""
    k = int(n * frac)
    raw = np.random.PCG64(seed).random_raw(2 * k)
    pos = (raw[:k] % np.uint64(n)).astype(np.int64)
    vals = (raw[k:] & np.uint64(0xFF)).astype(np.uint8)
    out = np.zeros(n, dtype=np.uint8)
    out[pos] = vals
    return out


def zipf_sizes(count, seed, s=1.1, unit=4096, kmax=32768):
    """C4: file sizes from a bounded Zipf(s) over {unit * k, k = 1..kmax}."""
    k = np.arange(1, kmax + 1, dtype=np.float64)
    p = k ** -s
    cdf = np.cumsum(p) / p.sum()
    u = (np.random.PCG64(seed).random_raw(count) >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    idx = np.searchsorted(cdf, u)
    return ((idx + 1) * unit).astype(np.int64)


def gear_table(seed):
    """Alternative Gear tables for parity tests (the real v0.0.8 table is unknown)."""
    return [int(x) for x in np.random.PCG64(seed).random_raw(256)]
