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


def _bits_mask(rng, bits, top):
    """`bits` distinct random bits below `top`."""
    return int(sum(1 << int(b) for b in rng.choice(top, size=bits, replace=False)))


def draw_masks(rng, default):
    """Random (MaskS, MaskL) for the randomised parity tests: `default` (the
    FastCDC pair), MaskL drawn from MaskS's bits (nested), mostly shared bits
    plus one of MaskL's own, or independent masks."""
    kind = rng.integers(0, 4)
    if kind == 0:
        return default
    top = int(rng.integers(20, 64))
    ms = _bits_mask(rng, int(rng.integers(9, 16)), top)
    bits = [b for b in range(64) if ms >> b & 1]
    if kind == 1:
        ml = int(sum(1 << int(b) for b in rng.choice(bits, size=max(1, len(bits) - 3), replace=False)))
    elif kind == 2:
        ml = int(sum(1 << int(b) for b in rng.choice(bits, size=max(1, len(bits) - 4), replace=False)))
        ml |= 1 << int(rng.integers(0, top))
    else:
        ml = _bits_mask(rng, int(rng.integers(6, 13)), int(rng.integers(16, 64)))
    return ms, ml
