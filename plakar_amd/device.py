"""Device-resident chunking of torch uint8 tensors already in HBM.

This is the path bench.py measures: inputs resident on the GPU, cut lists
written to device memory by the kernels of libplakar_cdc.so.  torch provides
device memory and streams only; the chunking itself is the HIP library.
"""
import ctypes

import torch

from . import _lib
from ._lib import check, ensure_init, lib


def _opts_c(opts):
    return _lib.cdc_opts(opts.MinSize, opts.NormalSize, opts.MaxSize, 0)


class DeviceBatch:
    """Preallocated device chunking of a fixed list of device buffers.

    launch() enqueues the kernels on a stream (async, allocation-free, graph-
    capturable); results() synchronises and returns, per buffer, an int64
    tensor (n, 2) of (offset, length) on the device.
    """

    def __init__(self, tensors, opts, final=True, device=None):
        ensure_init()
        if not tensors:
            raise ValueError("no buffers")
        self.tensors = list(tensors)
        for t in self.tensors:
            if t.dtype != torch.uint8 or not t.is_cuda or not t.is_contiguous():
                raise ValueError("expected contiguous uint8 CUDA tensors")
        self.device = self.tensors[0].device.index if device is None else device
        self.opts = opts
        self.final = 1 if final else 0
        self._o = _opts_c(opts)
        n = len(self.tensors)
        self.n = n
        self.lens = (ctypes.c_uint64 * n)(*[t.numel() for t in self.tensors])
        ws = ctypes.c_uint64()
        check(lib().cdc_device_batch_workspace_size(self.lens, n, ctypes.byref(self._o),
                                                    ctypes.byref(ws)), "workspace size")
        dev = torch.device("cuda", self.device)
        self.workspace = torch.empty(max(int(ws.value), 256), dtype=torch.uint8, device=dev)
        self.caps = [t.numel() // opts.MinSize + 2 for t in self.tensors]
        self.cuts = [torch.empty((c, 2), dtype=torch.int64, device=dev) for c in self.caps]
        self.res = torch.zeros((n, 4), dtype=torch.int64, device=dev)
        self._data = (ctypes.c_void_p * n)(*[t.data_ptr() for t in self.tensors])
        self._cuts = (ctypes.c_void_p * n)(*[c.data_ptr() for c in self.cuts])
        self._caps = (ctypes.c_uint64 * n)(*self.caps)
        rsz = self.res.element_size() * 4
        self._res = (ctypes.c_void_p * n)(*[self.res.data_ptr() + i * rsz for i in range(n)])

    def launch(self, stream=None):
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        check(lib().cdc_chunk_device_batch_async(
            self.device, self._data, self.lens, self.n, self.final, ctypes.byref(self._o),
            self._cuts, self._caps, self._res, ctypes.c_void_p(self.workspace.data_ptr()),
            self.workspace.numel(), ctypes.c_void_p(stream.cuda_stream)), "chunk_device")

    def results(self):
        """Synchronise and return (list of (n_i, 2) int64 device tensors, result rows)."""
        torch.cuda.synchronize(self.device)
        r = self.res.cpu()
        out = []
        for i in range(self.n):
            ncuts, consumed, status, needed = (int(x) for x in r[i])
            check(status, f"buffer {i}")
            c = self.cuts[i][:ncuts].clone()
            c[:, 1] &= 0xFFFFFFFF
            out.append(c)
        return out, r


def chunk_device(tensors, opts, final=True):
    """One-shot helper: chunk device-resident uint8 tensors, return cut tensors."""
    b = DeviceBatch(tensors, opts, final=final)
    b.launch()
    cuts, _ = b.results()
    return cuts


def set_debug_mode(mode):
    """0 = fast path, 1 = sequential single-wave resolver (cross-check)."""
    lib().cdc_set_debug_mode(int(mode))


def set_maskl_index_mode(mode):
    """0 = never build the MaskL index, 1 = adaptive (default), 2 = every
    launch group in the fused pass (k_scan_f), 3 = every launch group by
    k_scan_l. Cut points do not depend on it."""
    check(lib().cdc_set_maskl_index_mode(int(mode)))


def maskl_state(device=0):
    """Adaptive MaskL state (diagnostics): (1 while the next launch groups
    build the MaskL index because a recent group asked for MaskL candidates,
    else 0; launch groups issued on the device)."""
    hint, groups = ctypes.c_uint32(), ctypes.c_uint64()
    check(lib().cdc_debug_maskl_state(int(device), ctypes.byref(hint), ctypes.byref(groups)))
    return hint.value, groups.value
