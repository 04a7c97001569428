"""Per-chunk digests: SHA-256 and byte histogram of
every chunk on the device vs hashlib / numpy, the reference's hashing config
mirror, and the entropy formula of snapshot/backup.go:548-569.

SHA-256 parity is pinned by the FIPS 180-4 known answers (and hashlib, the
CPython restatement of the same standard); the histogram is exact integer
counting.  GPU tests are marked `gpu`.
"""
import hashlib
import math

import numpy as np
import pytest

from datagen import random_bytes

# FIPS 180-4 / NIST CSRC SHA-256 examples
KATS = [
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    (b"abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu",
     "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"),
    (b"a" * 1000000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
]


def test_kats_pin_hashlib():
    """The oracle (hashlib) agrees with the FIPS 180-4 known answers."""
    for msg, hexd in KATS:
        assert hashlib.sha256(msg).hexdigest() == hexd


def test_hashing_configuration_mirror():
    from plakar_amd import hashing
    c = hashing.DefaultConfiguration()
    assert (c.Algorithm, c.Bits) == ("SHA256", 256)
    c2, err = hashing.LookupDefaultConfiguration("BLAKE3")
    assert c2 is None and str(err) == "unknown hashing algorithm: BLAKE3"


def _entropy_direct(data):
    """snapshot/backup.go:548-569 restated over the bytes."""
    if len(data) == 0:
        return 0.0, [0.0] * 256
    freq = [0.0] * 256
    for b in data:
        freq[b] += 1
    e = 0.0
    size = float(len(data))
    for f in freq:
        if f > 0:
            p = f / size
            e -= p * math.log2(p)
    return e, freq


def test_entropy_from_histogram_matches_reference_formula():
    from plakar_amd import hashing
    for n, seed in [(0, 0), (1, 1), (255, 2), (4096, 3)]:
        data = random_bytes(n, seed)
        e, freq = _entropy_direct(data.tobytes())
        hist = np.bincount(data, minlength=256) if n else np.zeros(256, np.int64)
        assert hashing.entropy_from_freq(hist.tolist(), n) == e  # same terms, same order: bit-identical
        assert [float(x) for x in hist] == freq


# ------------------------------------------------------------------ GPU parity
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _run(buf, cuts):
    torch = _gpu()
    from plakar_amd import _lib, hashing
    _lib.ensure_init()
    t = torch.from_numpy(np.ascontiguousarray(buf)).cuda()
    c = torch.tensor(np.asarray(cuts, dtype=np.int64).reshape(-1, 2), device="cuda")
    d, h = hashing.chunk_digests(t, c)
    torch.cuda.synchronize()
    return d.cpu().numpy(), h.cpu().numpy()


def _check(buf, cuts, d, h):
    for i, (o, n) in enumerate(cuts):
        part = buf[o:o + n].tobytes()
        assert bytes(d[i]) == hashlib.sha256(part).digest(), f"chunk {i} ({o}, {n})"
        assert (h[i] == np.bincount(np.frombuffer(part, np.uint8), minlength=256)).all(), f"histogram {i}"


@pytest.mark.gpu
def test_gpu_digest_kats():
    msgs = [m for m, _ in KATS]
    buf = np.frombuffer(b"".join(msgs), np.uint8).copy()
    cuts, o = [], 0
    for m in msgs:
        cuts.append((o, len(m)))
        o += len(m)
    d, h = _run(buf, cuts)
    for i, (_, hexd) in enumerate(KATS):
        assert bytes(d[i]).hex() == hexd
    _check(buf, cuts, d, h)


@pytest.mark.gpu
def test_gpu_digest_padding_boundaries_and_alignment():
    """Lengths around the one/two final-block boundary (55/56, 63/64, ...) at
    every byte alignment of the chunk start."""
    buf = random_bytes(1 << 20, 11)
    lens = [0, 1, 3, 4, 5, 54, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 1000, 4095, 4096, 65537]
    cuts, o = [], 0
    for k, n in enumerate(lens * 4):
        o += k % 7  # gaps: every alignment
        cuts.append((o, n))
        o += n
    assert o < buf.size
    d, h = _run(buf, cuts)
    _check(buf, cuts, d, h)


@pytest.mark.gpu
def test_gpu_digest_of_device_cut_list():
    """The device path's own cut list of 48 MiB of random bytes, digests and
    histograms straight from device memory (count bounded by the result row),
    checked chunk by chunk; and the processChunk records."""
    torch = _gpu()
    from plakar_amd import _lib, chunkers, device, hashing
    _lib.ensure_init()
    data = random_bytes(48 << 20, 12)
    t = torch.from_numpy(data).cuda()
    b = device.DeviceBatch([t], chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20))
    b.launch()
    d, h = hashing.chunk_digests(t, b.cuts[0], result=b.res[0])
    torch.cuda.synchronize()
    (cuts,), res = b.results()
    n = cuts.shape[0]
    cl = cuts.cpu().numpy()
    dd, hh = d[:n].cpu().numpy(), h[:n].cpu().numpy()
    _check(data, [(int(o), int(m)) for o, m in cl], dd, hh)
    recs = hashing.chunk_records(t, cuts)
    o, m = int(cl[0][0]), int(cl[0][1])
    e, freq = _entropy_direct(data[o:o + m].tobytes())
    assert recs[0].Checksum == hashlib.sha256(data[o:o + m].tobytes()).digest()
    assert recs[0].Length == m and recs[0].Entropy == e
    assert recs[0].Distribution == [f / m for f in freq]


@pytest.mark.gpu
def test_gpu_digest_batch_many_buffers():
    """One launch group over several buffers (the batched entry point), with
    per-buffer counts bounded on the device."""
    torch = _gpu()
    from plakar_amd import _lib, hashing
    _lib.ensure_init()
    bufs, cut_lists, res, refs = [], [], [], []
    for k in range(5):
        data = random_bytes(200000 + 7919 * k, 40 + k)
        cuts, o = [], k
        while o + 3000 < data.size:
            n = int((o * 2654435761) % 9000)
            n = min(n, data.size - o)
            cuts.append((o, n))
            o += n + 1
        cuts.append((0, 0))
        keep = len(cuts) - 3 if k % 2 else len(cuts)  # the result row bounds the count on odd buffers
        bufs.append(torch.from_numpy(data).cuda())
        cut_lists.append(torch.tensor(np.asarray(cuts, np.int64), device="cuda"))
        res.append(torch.tensor([keep, 0, 0, 0], dtype=torch.int64, device="cuda"))
        refs.append((data, cuts[:keep]))
    outs = hashing.chunk_digests_batch(bufs, cut_lists, res)
    torch.cuda.synchronize()
    for (data, cuts), (d, h) in zip(refs, outs):
        _check(data, cuts, d[:len(cuts)].cpu().numpy(), h[:len(cuts)].cpu().numpy())
