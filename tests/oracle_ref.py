"""ctypes wrapper of the CPU oracle (oracle/fastcdc_oracle.c).

TEST INFRASTRUCTURE: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg only, as the checker.  Never imported by plakar_amd/.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")

DEFAULT_MASK_S = 0x0003590703530000
DEFAULT_MASK_L = 0x0000D90003530000


class _Params(ctypes.Structure):
    _fields_ = [("gear", ctypes.POINTER(ctypes.c_uint64)), ("mask_s", ctypes.c_uint64),
                ("mask_l", ctypes.c_uint64), ("min_size", ctypes.c_uint64),
                ("normal_size", ctypes.c_uint64), ("max_size", ctypes.c_uint64),
                ("cut_adj", ctypes.c_uint32)]


class Oracle:
    def __init__(self):
        src = os.path.join(ROOT, "oracle", "fastcdc_oracle.c")
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
        L = ctypes.CDLL(LIB)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.oracle_chunk.restype = ctypes.c_uint64
        L.oracle_chunk.argtypes = [ctypes.POINTER(_Params), ctypes.c_void_p, ctypes.c_uint64,
                                   u64p, u32p, ctypes.c_uint64]
        L.oracle_chunkify.restype = ctypes.c_uint64
        L.oracle_chunkify.argtypes = L.oracle_chunk.argtypes
        L.oracle_fastcdc_algorithm.restype = ctypes.c_uint64
        L.oracle_fastcdc_algorithm.argtypes = [ctypes.POINTER(_Params), ctypes.c_void_p,
                                               ctypes.c_uint64]
        L.oracle_fastcdc_validate.restype = ctypes.c_int
        L.oracle_fastcdc_validate.argtypes = [ctypes.c_uint64] * 3
        L.oracle_hashed_bytes.restype = ctypes.c_uint64
        L.oracle_hashed_bytes.argtypes = [ctypes.POINTER(_Params), u32p, ctypes.c_uint64]
        self.L = L

    @staticmethod
    def _params(gear, min_size, normal_size, max_size, mask_s, mask_l, cut_adj):
        g = (ctypes.c_uint64 * 256)(*[int(x) & 0xFFFFFFFFFFFFFFFF for x in gear])
        p = _Params(ctypes.cast(g, ctypes.POINTER(ctypes.c_uint64)), mask_s, mask_l, min_size,
                    normal_size, max_size, cut_adj)
        return p, g

    def chunk(self, data, gear, min_size=65536, normal_size=1 << 20, max_size=4 << 20,
              mask_s=DEFAULT_MASK_S, mask_l=DEFAULT_MASK_L, cut_adj=0, chunkify=False):
        """Drain (*Chunker).Next over `data`: returns a uint64 array (n, 2) of
        (offset, length) rows."""
        a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data, dtype=np.uint8)
        p, g = self._params(gear, min_size, normal_size, max_size, mask_s, mask_l, cut_adj)
        cap = a.size // max(min_size, 1) + 4
        offs = np.zeros(cap, dtype=np.uint64)
        lens = np.zeros(cap, dtype=np.uint32)
        fn = self.L.oracle_chunkify if chunkify else self.L.oracle_chunk
        n = fn(ctypes.byref(p), a.ctypes.data if a.size else None, a.size,
               offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
               lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), cap)
        assert n <= cap
        out = np.zeros((n, 2), dtype=np.uint64)
        out[:, 0] = offs[:n]
        out[:, 1] = lens[:n]
        return out

    def algorithm(self, data, gear, min_size, normal_size, max_size, mask_s=DEFAULT_MASK_S,
                  mask_l=DEFAULT_MASK_L, cut_adj=0):
        a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8), dtype=np.uint8)
        p, g = self._params(gear, min_size, normal_size, max_size, mask_s, mask_l, cut_adj)
        return int(self.L.oracle_fastcdc_algorithm(ctypes.byref(p), a.ctypes.data, a.size))

    def validate(self, min_size, normal_size, max_size):
        return self.L.oracle_fastcdc_validate(min_size, normal_size, max_size)

    def hashed_bytes(self, cuts, min_size):
        lens = np.ascontiguousarray(cuts[:, 1], dtype=np.uint32)
        p, g = self._params([0] * 256, min_size, min_size + 1, min_size + 2, 1, 1, 0)
        return int(self.L.oracle_hashed_bytes(ctypes.byref(p),
                                              lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                              lens.size))


def py_algorithm(data, gear, min_size, normal_size, max_size, mask_s=DEFAULT_MASK_S,
                 mask_l=DEFAULT_MASK_L, cut_adj=0):
    """Pure-Python restatement of (*FastCDC).Algorithm (small inputs only); an
    independent second statement used to check the C oracle."""
    n = len(data)
    if n <= min_size:
        return n
    if n >= max_size:
        n = max_size
    elif n <= normal_size:
        normal_size = n
    fp = 0
    M = 0xFFFFFFFFFFFFFFFF
    i = min_size
    while i < normal_size:
        fp = ((fp << 1) + gear[data[i]]) & M
        if fp & mask_s == 0:
            return i + cut_adj
        i += 1
    while i < n:
        fp = ((fp << 1) + gear[data[i]]) & M
        if fp & mask_l == 0:
            return i + cut_adj
        i += 1
    return i


def py_chunk(data, gear, min_size, normal_size, max_size, **kw):
    out, p = [], 0
    while p < len(data):
        n = min(len(data) - p, max_size)
        cut = py_algorithm(bytes(data[p:p + n]), gear, min_size, normal_size, max_size, **kw)
        out.append((p, cut))
        p += cut
    return out
