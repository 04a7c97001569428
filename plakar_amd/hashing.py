"""Mirror of plakar's hashing package and of the per-chunk work of
snapshot/backup.go processChunk, on the device.

    hashing/hashing.go:9-29      Configuration, DefaultConfiguration,
                                 LookupDefaultConfiguration
    snapshot/backup.go:548-569   entropy(data) -> (entropy, freq[256])
    snapshot/backup.go:594-629   processChunk: chunk SHA-256, entropy, the
                                 normalised byte distribution -> objects.Chunk

chunk_digests() runs the HIP kernel of libplakar_cdc.so
(cdc_chunk_digests_device_async): one SHA-256 and one 256-bin histogram per
chunk of a device cut list.  The float64 entropy is computed here, on the host,
with the reference's formula and summation order, from the exact integer
histogram, with Go's math.Log2 restated (go_log2: math/log2.go's frexp
split over the fdlibm log that math/log.go implements).  Go is not available
here, so bit-identity with Go's floats is unpinned.
"""
import ctypes
import math
from dataclasses import dataclass, field
from typing import List

import numpy as np
import torch

from . import _lib
from ._lib import check, lib


@dataclass
class Configuration:
    """hashing.Configuration (hashing/hashing.go:9-12)."""
    Algorithm: str
    Bits: int


def LookupDefaultConfiguration(algorithm):
    """hashing.LookupDefaultConfiguration (hashing/hashing.go:19-29)."""
    if algorithm == "SHA256":
        return Configuration("SHA256", 256), None
    return None, ValueError(f"unknown hashing algorithm: {algorithm}")


def DefaultConfiguration():
    """hashing.DefaultConfiguration (hashing/hashing.go:14-17)."""
    return LookupDefaultConfiguration("SHA256")[0]


def chunk_digests(data, cuts, result=None, hist=True, stream=None):
    """SHA-256 (and byte histogram) of every chunk of a device buffer.

    data: contiguous uint8 CUDA tensor; cuts: (n, 2) int64 CUDA tensor of
    (offset, length) as the device path returns them (or its raw cdc_cut
    storage); result: optional int64 CUDA tensor row (ncuts, consumed,
    status, needed) bounding the count on the device.  Returns (digests
    uint8 (n, 32), histograms int32 (n, 256) or None) on the device;
    asynchronous on `stream` like the rest of the device path.
    """
    if data.dtype != torch.uint8 or not data.is_cuda or not data.is_contiguous():
        raise ValueError("expected a contiguous uint8 CUDA tensor")
    if cuts.dtype != torch.int64 or cuts.dim() != 2 or cuts.shape[1] != 2 or not cuts.is_contiguous():
        raise ValueError("expected an (n, 2) contiguous int64 cut tensor")
    n = cuts.shape[0]
    dev = data.device
    digests = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    h = torch.empty((n, 256), dtype=torch.int32, device=dev) if hist else None
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    check(lib().cdc_chunk_digests_device_async(
        dev.index, ctypes.c_void_p(data.data_ptr()), data.numel(), ctypes.c_void_p(cuts.data_ptr()), n,
        ctypes.c_void_p(result.data_ptr() if result is not None else 0), ctypes.c_void_p(digests.data_ptr()),
        ctypes.c_void_p(h.data_ptr() if h is not None else 0), ctypes.c_void_p(stream.cuda_stream)), "digests")
    return digests, h


def chunk_digests_batch(datas, cut_lists, results=None, hist=True, stream=None):
    """chunk_digests() for several buffers in one launch group (every chunk of
    every buffer hashes in parallel: a launch lasts as long as its longest
    chunk, so batching is what gives throughput).  Returns a list of
    (digests, histograms) per buffer."""
    n = len(datas)
    if n == 0:
        return []
    dev = datas[0].device
    for t, c in zip(datas, cut_lists):
        if t.dtype != torch.uint8 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("expected contiguous uint8 CUDA tensors")
        if c.dtype != torch.int64 or c.dim() != 2 or c.shape[1] != 2 or not c.is_contiguous():
            raise ValueError("expected (n, 2) contiguous int64 cut tensors")
    outs = [(torch.empty((c.shape[0], 32), dtype=torch.uint8, device=dev),
             torch.empty((c.shape[0], 256), dtype=torch.int32, device=dev) if hist else None) for c in cut_lists]
    V = ctypes.c_void_p
    arr = lambda xs: (V * n)(*xs)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    check(lib().cdc_chunk_digests_device_batch_async(
        dev.index, arr([t.data_ptr() for t in datas]), (ctypes.c_uint64 * n)(*[t.numel() for t in datas]), n,
        arr([c.data_ptr() for c in cut_lists]), (ctypes.c_uint64 * n)(*[c.shape[0] for c in cut_lists]),
        arr([r.data_ptr() for r in results]) if results is not None else None,
        arr([o[0].data_ptr() for o in outs]), arr([o[1].data_ptr() for o in outs]) if hist else None,
        V(stream.cuda_stream)), "digests")
    return outs


def chunk_digests_hybrid(datas, cut_lists, results=None, hist=True, stream=None, host_threads=16,
                         host_min_len=0):
    """chunk_digests_batch() with the longest chunks' SHA-256 on host cores
    (cdc_chunk_digests_hybrid): a device chain costs ~2 us per 64-B block, a
    host core with the SHA extensions ~35 ns, and one device launch lasts as
    long as its longest chunk.  Synchronous.  Returns (outs, host_chunks,
    host_bytes), outs as chunk_digests_batch's."""
    n = len(datas)
    if n == 0:
        return [], 0, 0
    if n > 32:
        raise ValueError("at most 32 buffers")
    dev = datas[0].device
    for t, c in zip(datas, cut_lists):
        if t.dtype != torch.uint8 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("expected contiguous uint8 CUDA tensors")
        if c.dtype != torch.int64 or c.dim() != 2 or c.shape[1] != 2 or not c.is_contiguous():
            raise ValueError("expected (n, 2) contiguous int64 cut tensors")
    outs = [(torch.empty((c.shape[0], 32), dtype=torch.uint8, device=dev),
             torch.empty((c.shape[0], 256), dtype=torch.int32, device=dev) if hist else None) for c in cut_lists]
    V = ctypes.c_void_p
    arr = lambda xs: (V * n)(*xs)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    hc, hb = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().cdc_chunk_digests_hybrid(
        dev.index, arr([t.data_ptr() for t in datas]), (ctypes.c_uint64 * n)(*[t.numel() for t in datas]), n,
        arr([c.data_ptr() for c in cut_lists]), (ctypes.c_uint64 * n)(*[c.shape[0] for c in cut_lists]),
        arr([r.data_ptr() for r in results]) if results is not None else None,
        arr([o[0].data_ptr() for o in outs]), arr([o[1].data_ptr() for o in outs]) if hist else None,
        int(host_threads), int(host_min_len), V(stream.cuda_stream), ctypes.byref(hc), ctypes.byref(hb)),
        "hybrid digests")
    return outs, int(hc.value), int(hb.value)


def chunk_entropy_device(hist, stream=None):
    """entropy() per histogram row on the device (cdc_chunk_entropy_device_async):
    hist is a (n, 256) int32/uint32 CUDA tensor as chunk_digests returns it;
    returns a float64 (n,) CUDA tensor, bit-equal to entropy_rows."""
    assert hist.is_cuda and hist.dim() == 2 and hist.shape[1] == 256 and hist.element_size() == 4
    _lib.ensure_init()
    hist = hist.contiguous()
    out = torch.empty(hist.shape[0], dtype=torch.float64, device=hist.device)
    if stream is None:
        stream = torch.cuda.current_stream(hist.device)
    check(lib().cdc_chunk_entropy_device_async(hist.device.index, ctypes.c_void_p(hist.data_ptr()), hist.shape[0],
                                               ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream.cuda_stream)),
          "entropy")
    return out


# --------------------------------------------------------------------- Go Log2
# fdlibm e_log.c constants (Go math/log.go uses the same algorithm)
_LN2_HI = 6.93147180369123816490e-01
_LN2_LO = 1.90821492927058770002e-10
_LG = (6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01,
       2.222219843214978396e-01, 1.818357216161805012e-01, 1.531383769920937332e-01,
       1.479819860511658591e-01)
_SQRT2_2 = math.sqrt(2.0) / 2.0
_INV_LN2 = float.fromhex("0x1.71547652b82fep+0")  # Go constant 1/Ln2, rounded once


def _go_log_reduced(f1, ki):
    """Go's log(x) for x = f1 * 2**ki, f1 in [0.5, 1) (frexp form), x > 0 finite."""
    if f1 < _SQRT2_2:
        f1 *= 2.0
        ki -= 1
    f = f1 - 1.0
    k = float(ki)
    s = f / (2.0 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (_LG[0] + s4 * (_LG[2] + s4 * (_LG[4] + s4 * _LG[6])))
    t2 = s4 * (_LG[1] + s4 * (_LG[3] + s4 * _LG[5]))
    r = t1 + t2
    hfsq = 0.5 * f * f
    return k * _LN2_HI - ((hfsq - (s * (hfsq + r) + k * _LN2_LO)) - f)


def go_log2(x):
    """math.Log2 as Go defines it for finite x > 0: frac, exp := Frexp(x);
    frac == 0.5 -> exp - 1; else Log(frac) * (1/Ln2) + exp."""
    frac, exp = math.frexp(x)
    if frac == 0.5:
        return float(exp - 1)
    return _go_log_reduced(*math.frexp(frac)) * _INV_LN2 + float(exp)


def go_log2_array(x):
    """go_log2 over a float64 array (elementwise IEEE operations in the same
    order; numpy ufuncs do not contract into FMAs)."""
    x = np.asarray(x, dtype=np.float64)
    frac, exp = np.frexp(x)
    f1, ki = np.frexp(frac)  # frac in [0.5, 1): f1 == frac, ki == 0
    small = f1 < _SQRT2_2
    f1 = np.where(small, f1 * 2.0, f1)
    k = (ki - small.astype(np.int64)).astype(np.float64)
    f = f1 - 1.0
    s = f / (2.0 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (_LG[0] + s4 * (_LG[2] + s4 * (_LG[4] + s4 * _LG[6])))
    t2 = s4 * (_LG[1] + s4 * (_LG[3] + s4 * _LG[5]))
    r = t1 + t2
    hfsq = 0.5 * f * f
    lg = k * _LN2_HI - ((hfsq - (s * (hfsq + r) + k * _LN2_LO)) - f)
    out = lg * _INV_LN2 + exp.astype(np.float64)
    return np.where(frac == 0.5, (exp - 1).astype(np.float64), out)


def entropy_rows(hist, lengths):
    """entropy() of backup.go:548-569 for every row of an integer histogram
    (n, 256) with row sums `lengths`: -sum_b p_b log2 p_b over the bins with
    p_b > 0, accumulated left to right.  Returns float64 (n,)."""
    hist = np.asarray(hist, dtype=np.float64)
    lengths = np.asarray(lengths, dtype=np.float64)
    n = hist.shape[0]
    out = np.zeros(n, dtype=np.float64)
    nz = lengths > 0
    if not nz.any():
        return out
    h = hist[nz]
    p = h / lengths[nz, None]
    pos = h > 0
    terms = np.zeros_like(p)
    terms[pos] = p[pos] * go_log2_array(p[pos])
    # e = 0; e -= t_0; e -= t_1; ...  == cumulative sum of -t, in bin order
    out[nz] = np.cumsum(-terms, axis=1)[:, -1]
    return out


def entropy_from_freq(freq, size):
    """entropy() of snapshot/backup.go:548-569 from its frequency table: the
    same float64 terms in the same order (bins 0..255), with Go's Log2."""
    if size == 0:
        return 0.0
    e = 0.0
    data_size = float(size)
    for f in freq:
        if f > 0:
            p = float(f) / data_size
            e -= p * go_log2(p)
    return e


@dataclass(slots=True)
class Chunk:
    """objects.Chunk (objects/objects.go:73-79).  Slotted: a backup makes one
    per chunk (tens of thousands per run), and a slotted instance is made and
    freed in about half the time of one with a __dict__."""
    Checksum: bytes
    Length: int
    Entropy: float
    Distribution: List[float] = field(default_factory=list)


def chunk_records(data, cuts, result=None):
    """processChunk's per-chunk records (snapshot/backup.go:594-629) for every
    chunk of a device cut list: Checksum and the histogram on the device,
    Entropy and Distribution (freq / len) on the host."""
    digests, hist = chunk_digests(data, cuts, result)
    torch.cuda.synchronize(data.device)
    lens = cuts[:, 1].cpu().tolist()
    dg = digests.cpu().numpy()
    hs = hist.cpu().numpy()
    out = []
    for i, n in enumerate(lens):
        freq = hs[i].tolist()
        dist = [float(f) / n for f in freq] if n > 0 else [0.0] * 256
        out.append(Chunk(bytes(dg[i]), int(n), entropy_from_freq(freq, n), dist))
    return out


__all__ = ["Configuration", "LookupDefaultConfiguration", "DefaultConfiguration", "chunk_digests",
           "chunk_digests_batch", "go_log2", "go_log2_array", "entropy_rows",
           "entropy_from_freq", "Chunk", "chunk_records", "_lib"]
