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


def _urandom_now(n):
    """os.urandom(n); a large draw in four pieces on threads (getrandom
    releases the GIL): the same kernel CSPRNG, ~2x sooner."""
    global _urandom_pool
    if n <= _URANDOM_SPLIT:
        return os.urandom(n)
    if _urandom_pool is None:
        from concurrent.futures import ThreadPoolExecutor
        _urandom_pool = ThreadPoolExecutor(4, thread_name_prefix="plakar-urandom")
    k = 4
    sizes = [n // k + (1 if i < n % k else 0) for i in range(k)]
    return b"".join(_urandom_pool.map(os.urandom, sizes))


class _Reservoir:
    """OS random bytes drawn ahead of the calls that use them: a background
    thread keeps up to `target` bytes of os.urandom output ready (in 256-KiB
    pieces), and each Encode call takes fresh bytes from it (never the same
    bytes twice), the rest drawn at once when the reservoir runs short.  The
    source is the same kernel CSPRNG; only the time of the draw moves off the
    call (a batch of ~20 K blobs needs 1.2 MB, 2-4.5 ms of getrandom).
    DESIGN.md 5.7."""

    PIECE = 256 << 10

    def __init__(self, target=4 << 20):
        import collections
        import threading
        self.target = target
        self.pieces = collections.deque()  # bytes objects, consumed from the left
        self.have = 0
        self.mu = threading.Lock()
        self.want = threading.Event()
        self.thread = None
        self.tl = threading.local()  # each thread's reusable output buffer (take_into)
        self.pid = os.getpid()
        # a fork while the filler holds mu must not leave the child's lock held
        os.register_at_fork(after_in_child=self._reset_lock)

    def _reset_lock(self):
        import threading
        self.mu = threading.Lock()

    def _after_fork(self):
        """A forked child must never use bytes its parent may also use (GCM
        nonce reuse): drop them and start its own filler.  Called under mu."""
        import threading
        if self.pid != os.getpid():
            self.pieces.clear()
            self.have = 0
            self.thread = None
            self.want = threading.Event()
            self.pid = os.getpid()

    def _fill(self):
        while True:
            self.want.wait()
            with self.mu:
                if self.have >= self.target:
                    self.want.clear()
                    continue
            piece = os.urandom(self.PIECE)
            with self.mu:
                if self.pid != os.getpid():
                    return
                self.pieces.append(piece)
                self.have += len(piece)

    def take_into(self, n):
        """n fresh bytes in this thread's reusable buffer (no allocation once
        it has grown: a fresh 1.2-MB bytes object costs ~1 ms of page faults);
        returned as a ctypes char array over it, valid until this thread's
        next call (cdc_encode_device copies the bytes before it returns)."""
        import ctypes
        import threading
        buf = getattr(self.tl, "buf", None)
        if buf is None or len(buf) < n:
            buf = self.tl.buf = bytearray(max(n, 1))
        mv = memoryview(buf)
        got = 0
        with self.mu:
            self._after_fork()
            while got < n and self.pieces:
                p = self.pieces.popleft()
                k = min(len(p), n - got)
                mv[got:got + k] = p[:k] if k < len(p) else p
                if k < len(p):
                    self.pieces.appendleft(p[k:])
                got += k
                self.have -= k
            if self.thread is None:
                self.thread = threading.Thread(target=self._fill, name="plakar-urandom-reservoir", daemon=True)
                self.thread.start()
        self.want.set()
        if got < n:
            mv[got:n] = _urandom_now(n - got)
        mv.release()
        return (ctypes.c_char * n).from_buffer(buf)

    def take(self, n):
        parts, got = [], 0
        with self.mu:
            self._after_fork()
            while got < n and self.pieces:
                p = self.pieces.popleft()
                k = min(len(p), n - got)
                parts.append(p[:k] if k < len(p) else p)
                if k < len(p):
                    self.pieces.appendleft(p[k:])
                got += k
                self.have -= k
            if self.thread is None:
                import threading
                self.thread = threading.Thread(target=self._fill, name="plakar-urandom-reservoir", daemon=True)
                self.thread.start()
        self.want.set()
        if got < n:
            parts.append(_urandom_now(n - got))
        return b"".join(parts)


_reservoir = _Reservoir()


def _urandom(n):
    """n fresh OS random bytes for Encode's subkeys and nonces."""
    return _reservoir.take(n)


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
        if random is None:  # fresh OS random bytes, drawn ahead (the reservoir)
            random = _reservoir.take_into(RANDOM_BYTES * n)
        elif len(random) != RANDOM_BYTES * n:
            raise ValueError(f"random: {RANDOM_BYTES} bytes per blob")
        else:
            random = bytes(random)
    st = stream if stream is not None else torch.cuda.current_stream(device)
    check(lib().cdc_encode_device(int(device), ctypes.c_void_p(base.data_ptr()), offs, lns, n, int(bool(compress)),
                                  key, random if key is not None else None, ctypes.c_void_p(out.data_ptr()),
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
