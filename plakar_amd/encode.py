"""Encode on the device: plakar's (*Repository).Encode (repository/repository.go:
212-236) for a batch of blobs -- the LZ4 frame of compression.DeflateLZ4Stream
(compression/compression.go:94-106), then the AES-256-GCM stream of
encryption.EncryptStream (encryption/symmetric.go:72-163) when a key is
configured.  Every call goes through the C ABI (cdc_encode_device)."""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check, ensure_init, lib

RANDOM_BYTES = 56  # per blob: subkey 32, subkey nonce 12, data nonce 12
_URANDOM_SPLIT = 256 << 10  # above this, os.urandom in parallel pieces
_urandom_pool = None


def _urandom(n):
    """os.urandom(n); a large draw (a batch of ~20 K blobs needs 1.2 MB, ~4 ms
    from one thread) in four pieces on threads (getrandom releases the GIL):
    the same kernel CSPRNG, ~2x sooner."""
    global _urandom_pool
    if n <= _URANDOM_SPLIT:
        return os.urandom(n)
    if _urandom_pool is None:
        from concurrent.futures import ThreadPoolExecutor
        _urandom_pool = ThreadPoolExecutor(4, thread_name_prefix="plakar-urandom")
    k = 4
    sizes = [n // k + (1 if i < n % k else 0) for i in range(k)]
    return b"".join(_urandom_pool.map(os.urandom, sizes))


def encode_bound(n, compress=True, encrypt=True):
    return int(lib().cdc_encode_bound(int(n), int(bool(compress)), int(bool(encrypt))))


def encode_device(base, offsets, lens, out, key=None, compress=True, random=None, device=0, stream=None):
    """Encode blobs that live in the device tensor `base` (uint8) at the given
    byte offsets/lengths (sequences or numpy arrays) into the device tensor
    `out`; returns the n + 1 output offsets (int64 numpy array)."""
    import torch
    ensure_init()
    n = len(lens)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    offs_a = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64).reshape(-1))
    lens_a = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64).reshape(-1))
    if offs_a.size != n:
        raise ValueError("offsets and lens differ in length")
    oo_a = np.zeros(n + 1, dtype=np.uint64)
    offs, lns, oo = (a.ctypes.data_as(u64p) if a.size else (ctypes.c_uint64 * 1)() for a in (offs_a, lens_a, oo_a))
    if key is not None:
        key = bytes(key)
        if len(key) != 32:
            raise ValueError("the repository key is 32 bytes (AES-256)")
        if random is None:
            random = _urandom(RANDOM_BYTES * n)
        if len(random) != RANDOM_BYTES * n:
            raise ValueError(f"random: {RANDOM_BYTES} bytes per blob")
    st = stream if stream is not None else torch.cuda.current_stream(device)
    check(lib().cdc_encode_device(int(device), ctypes.c_void_p(base.data_ptr()), offs, lns, n, int(bool(compress)),
                                  key, bytes(random) if key is not None else None, ctypes.c_void_p(out.data_ptr()),
                                  out.numel(), oo, ctypes.c_void_p(st.cuda_stream)), "cdc_encode_device")
    return oo_a.astype(np.int64)


def encode_blobs(blobs, key=None, compress=True, random=None, device=0):
    """Encode host byte buffers (numpy uint8 arrays or bytes): a list of the
    encoded bytes, blob by blob."""
    import torch
    arrs = [np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else np.asarray(b, np.uint8).ravel()
            for b in blobs]
    lens = [a.size for a in arrs]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) if arrs else np.zeros(1, np.uint64)
    dev = torch.device("cuda", device)
    base = torch.empty(max(int(offs[-1]), 1), dtype=torch.uint8, device=dev)
    if arrs and offs[-1]:
        base[:int(offs[-1])].copy_(torch.from_numpy(np.concatenate(arrs)))
    cap = sum(encode_bound(n, compress, key is not None) for n in lens)
    out = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
    oo = encode_device(base, offs[:-1], lens, out, key=key, compress=compress, random=random, device=device)
    host = out[:int(oo[-1])].cpu().numpy()
    return [host[oo[i]:oo[i + 1]].tobytes() for i in range(len(lens))]


class DeviceEncoder:
    """(*Repository).Encode with the repository's configuration: compression
    "LZ4" (compression.DefaultConfiguration) or None, and the encryption key
    (None: no encryption).  `encode_many` encodes a whole batch of blobs in
    one device call; calling the object encodes one blob, like Encode."""

    def __init__(self, key=None, compression="LZ4", device=0):
        if compression not in (None, "LZ4"):
            raise ValueError(f"unsupported compression {compression!r} (the device path implements LZ4)")
        self.key = None if key is None else bytes(key)
        self.compress = compression == "LZ4"
        self.device = device

    def encode_many(self, blobs):
        return encode_blobs(blobs, key=self.key, compress=self.compress, device=self.device)

    def __call__(self, blob):
        return self.encode_many([blob])[0]
