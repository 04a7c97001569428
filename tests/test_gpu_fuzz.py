"""Randomised GPU parity: the HIP path (through the C ABI) against the CPU
oracle on seeded random configurations, bit-exact.

Each case draws from its seed: the Gear table (the placeholder or a random
one), the masks (FastCDC's, or random ones: some k_scan_f can fuse, some it
cannot), Min / Normal / Max within Validate's bounds, the cut convention, the
MaskL index mode, and a launch group of 1-5 buffers (sizes 0 B to 12 MiB,
unaligned starts) of random, low-entropy, zero, periodic or mixed bytes.  The
oracle (oracle/fastcdc_oracle.c) restates (*FastCDC).Algorithm and the Next
loop; PARITY UNPINNED w.r.t. the Go module.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from datagen import draw_masks, gear_table, low_entropy, random_bytes  # noqa: E402
from oracle_ref import DEFAULT_MASK_L, DEFAULT_MASK_S  # noqa: E402
from plakar_amd import _lib, chunkers, device  # noqa: E402

pytestmark = pytest.mark.gpu

import os  # noqa: E402

N_CASES = int(os.environ.get("FUZZ_CASES", "128"))  # a longer sweep: FUZZ_CASES=2000
N_STREAM = int(os.environ.get("FUZZ_STREAM_CASES", "32"))


@pytest.fixture(autouse=True)
def _restore():
    yield
    device.set_maskl_index_mode(1)
    _lib.ensure_init(gear=_lib.default_gear())


def _masks(rng):
    return draw_masks(rng, (DEFAULT_MASK_S, DEFAULT_MASK_L))


def _params(rng):
    mn = 64 << int(rng.integers(0, 11))
    nm = mn << int(rng.integers(1, 5))
    mx = nm << int(rng.integers(1, 4))
    return dict(min_size=mn, normal_size=min(nm, 1 << 30), max_size=min(mx, 1 << 30))


def _data(rng, n, seed):
    kind = int(rng.integers(0, 5))
    if n == 0:
        return np.zeros(0, np.uint8)
    if kind == 0:
        return random_bytes(n, seed)
    if kind == 1:
        return low_entropy(n, seed, float(rng.choice([0.001, 0.005, 0.01, 0.05])))
    if kind == 2:
        return np.zeros(n, np.uint8)
    if kind == 3:  # a random block repeated
        blk = random_bytes(int(rng.integers(1, 4097)), seed)
        return np.resize(blk, n)
    parts, left, k = [], n, 0
    while left > 0:
        m = min(left, int(rng.integers(1, max(2, n // 3) + 1)))
        parts.append(_data(rng, m, seed * 7 + k))
        left -= m
        k += 1
    return np.concatenate(parts)


def _size(rng):
    r = rng.random()
    if r < 0.1:
        return int(rng.integers(0, 200))
    return int(np.exp(rng.uniform(np.log(200), np.log(12 << 20))))


@pytest.mark.parametrize("seed", range(N_CASES))
def test_random_configuration(oracle, seed):
    rng = np.random.default_rng(np.random.PCG64(1000 + seed))
    gear = _lib.default_gear() if rng.random() < 0.3 else gear_table(2000 + seed)
    ms, ml = _masks(rng)
    p = _params(rng)
    assert oracle.validate(p["min_size"], p["normal_size"], p["max_size"]) == 0, p
    cut_adj = int(rng.integers(0, 2))
    mode = int(rng.integers(0, 4))
    nb = int(rng.integers(1, 6))
    datas = [_data(rng, _size(rng), 3000 + 16 * seed + i) for i in range(nb)]
    offs = [int(rng.integers(0, 16)) for _ in range(nb)]
    what = (f"seed {seed}: masks {ms:#x}/{ml:#x} {p} cut_adj {cut_adj} mode {mode} "
            f"sizes {[d.size for d in datas]} offsets {offs}")

    _lib.ensure_init(gear=gear, mask_s=ms, mask_l=ml, cut_convention=cut_adj)
    device.set_maskl_index_mode(mode)
    ts = []
    for a, off in zip(datas, offs):
        t = torch.empty(a.size + off + 16, dtype=torch.uint8, device="cuda")
        t[off:off + a.size].copy_(torch.from_numpy(a))
        ts.append(t[off:off + a.size])
    b = device.DeviceBatch(ts, chunkers.ChunkerOpts(MinSize=p["min_size"], NormalSize=p["normal_size"],
                                                     MaxSize=p["max_size"]))
    for rep in range(2):  # the second launch reuses the workspace
        b.launch()
        cuts, res = b.results()
        for i, (a, c) in enumerate(zip(datas, cuts)):
            got = c.cpu().numpy().astype(np.uint64)
            ref = oracle.chunk(a, gear, mask_s=ms, mask_l=ml, cut_adj=cut_adj, **p)
            assert got.shape == ref.shape, f"{what}: buffer {i} rep {rep}: {got.shape[0]} chunks vs {ref.shape[0]}"
            bad = np.nonzero((got != ref).any(axis=1))[0]
            assert bad.size == 0, f"{what}: buffer {i} rep {rep}: chunk {bad[0]}: {got[bad[0]]} vs {ref[bad[0]]}"
            assert int(res[i, 1]) == a.size, f"{what}: buffer {i} consumed {int(res[i, 1])}"


@pytest.mark.parametrize("seed", range(N_STREAM))
def test_random_stream_windows(oracle, seed):
    """A stream chunked as non-final windows (each resumed at the last
    window's `consumed`, the Peek(MaxSize) carry of the Go chunker's Next)
    gives the whole stream's cuts, for random configurations and windows of
    MaxSize + 1 .. 4 MaxSize bytes."""
    rng = np.random.default_rng(np.random.PCG64(5000 + seed))
    gear = _lib.default_gear() if rng.random() < 0.3 else gear_table(6000 + seed)
    ms, ml = _masks(rng)
    p = _params(rng)
    cut_adj = int(rng.integers(0, 2))
    device.set_maskl_index_mode(int(rng.integers(0, 4)))
    data = _data(rng, int(rng.integers(1, min(24 << 20, 100 * p["max_size"]))), 7000 + seed)  # <= ~100 windows
    _lib.ensure_init(gear=gear, mask_s=ms, mask_l=ml, cut_convention=cut_adj)
    ref = oracle.chunk(data, gear, mask_s=ms, mask_l=ml, cut_adj=cut_adj, **p)
    opts = chunkers.ChunkerOpts(MinSize=p["min_size"], NormalSize=p["normal_size"], MaxSize=p["max_size"])
    got, off = [], 0
    while off < data.size:
        w = min(p["max_size"] + int(rng.integers(1, 3 * p["max_size"] + 2)), data.size - off)
        fin = off + w == data.size
        t = torch.from_numpy(np.ascontiguousarray(data[off:off + w])).cuda()
        b = device.DeviceBatch([t], opts, final=fin)
        b.launch()
        (c,), res = b.results()
        c = c.cpu().numpy().astype(np.uint64)
        c[:, 0] += np.uint64(off)
        got.append(c)
        consumed = int(res[0, 1])
        assert fin or consumed > 0, f"seed {seed}: window at {off} consumed nothing"
        off = off + w if fin else off + consumed
    got = np.concatenate(got) if got else np.zeros((0, 2), np.uint64)
    what = f"seed {seed}: masks {ms:#x}/{ml:#x} {p} cut_adj {cut_adj} size {data.size}"
    assert got.shape == ref.shape, f"{what}: {got.shape[0]} chunks vs {ref.shape[0]}"
    bad = np.nonzero((got != ref).any(axis=1))[0]
    assert bad.size == 0, f"{what}: chunk {bad[0]}: {got[bad[0]]} vs {ref[bad[0]]}"


@pytest.mark.parametrize("seed", range(24))
def test_random_host_buffers(oracle, seed, monkeypatch):
    """cdc_chunk (host buffers in, cut lists out, through the two-slot staging
    pipeline) on random configurations: 1-40 buffers, launch-group budgets of
    16 MiB-1 GiB, and buffers above CDC_HOST_MAXBUF_MB chunked as streams of
    windows."""
    rng = np.random.default_rng(np.random.PCG64(8000 + seed))
    gear = _lib.default_gear() if rng.random() < 0.3 else gear_table(8100 + seed)
    ms, ml = _masks(rng)
    p = _params(rng)
    cut_adj = int(rng.integers(0, 2))
    monkeypatch.setenv("CDC_HOST_GROUP_MB", str(int(rng.choice([16, 64, 1024]))))
    monkeypatch.setenv("CDC_HOST_MAXBUF_MB", str(int(rng.choice([16, 64, 16384]))))
    device.set_maskl_index_mode(int(rng.integers(0, 4)))
    nb = int(rng.integers(1, 41))
    sizes = [_size(rng) if rng.random() < 0.9 else int(rng.integers(16 << 20, 40 << 20)) for _ in range(nb)]
    datas = [_data(rng, n, 8200 + 64 * seed + i) for i, n in enumerate(sizes)]
    _lib.ensure_init(gear=gear, mask_s=ms, mask_l=ml, cut_convention=cut_adj)
    res = chunkers.ChunkBuffers(datas, chunkers.ChunkerOpts(MinSize=p["min_size"], NormalSize=p["normal_size"],
                                                             MaxSize=p["max_size"]))
    what = f"seed {seed}: masks {ms:#x}/{ml:#x} {p} cut_adj {cut_adj} sizes {sizes}"
    for i, a in enumerate(datas):
        ref = oracle.chunk(a, gear, mask_s=ms, mask_l=ml, cut_adj=cut_adj, **p)
        got = np.asarray(res[i]).astype(np.uint64).reshape(-1, 2)
        assert got.shape == ref.shape, f"{what}: buffer {i}: {got.shape[0]} chunks vs {ref.shape[0]}"
        bad = np.nonzero((got != ref).any(axis=1))[0]
        assert bad.size == 0, f"{what}: buffer {i}: chunk {bad[0]}: {got[bad[0]]} vs {ref[bad[0]]}"


class _RaggedReader:
    """An io.Reader that returns 1..k bytes per read (no readinto)."""

    def __init__(self, data, rng):
        self.b = data.tobytes()
        self.o = 0
        self.rng = rng

    def read(self, n):
        k = min(n, int(self.rng.integers(1, 1 << int(self.rng.integers(1, 22)))))
        out = self.b[self.o:self.o + k]
        self.o += len(out)
        return out


@pytest.mark.parametrize("seed", range(16))
def test_random_streaming_next(oracle, seed):
    """NewChunker(...).Next() over a ragged reader (1 B - 2 MiB per read),
    random configurations and window sizes: the chunks are the oracle's, byte
    for byte, then (nil, EOF)."""
    rng = np.random.default_rng(np.random.PCG64(6600 + seed))
    gear = _lib.default_gear() if rng.random() < 0.3 else gear_table(6700 + seed)
    ms, ml = _masks(rng)
    p = _params(rng)
    cut_adj = int(rng.integers(0, 2))
    device.set_maskl_index_mode(int(rng.integers(0, 4)))
    data = _data(rng, int(rng.integers(0, 12 << 20)), 6800 + seed)
    window = int(rng.choice([0, 1, 3 << 20, 2 * p["max_size"] + 4096 + int(rng.integers(0, 1 << 20))]))
    _lib.ensure_init(gear=gear, mask_s=ms, mask_l=ml, cut_convention=cut_adj)
    ref = oracle.chunk(data, gear, mask_s=ms, mask_l=ml, cut_adj=cut_adj, **p)
    opts = chunkers.ChunkerOpts(MinSize=p["min_size"], NormalSize=p["normal_size"], MaxSize=p["max_size"])
    chk = chunkers.NewChunker("fastcdc", _RaggedReader(data, rng), opts, window_bytes=window)
    what = f"seed {seed}: masks {ms:#x}/{ml:#x} {p} cut_adj {cut_adj} size {data.size} window {window}"
    off, k = 0, 0
    while True:
        chunk, err = chk.Next()
        if err is chunkers.EOF:
            assert chunk is None, what
            break
        assert k < ref.shape[0], f"{what}: more chunks than the oracle's {ref.shape[0]}"
        assert (int(ref[k, 0]), int(ref[k, 1])) == (off, len(chunk)), f"{what}: chunk {k}"
        assert chunk == data[off:off + len(chunk)].tobytes(), f"{what}: chunk {k} bytes"
        off += len(chunk)
        k += 1
    assert k == ref.shape[0] and off == data.size, what
    chk.close()
