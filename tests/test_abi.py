"""The C-ABI library loads and exports every symbol include/plakar_cdc.h
declares; pure (device-free) entry points behave.  No GPU compute here."""
import ctypes
import json
import os
import re

import pytest

from plakar_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "plakar_cdc.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(cdc_[a-z0-9_]+)\s*\(", src))
    return sorted(n for n in names if not n.endswith("_fn"))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    syms = _declared_symbols()
    assert len(syms) >= 24
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # and the Python binding declares a signature for each of them
    assert set(syms) <= set(_lib.SIGNATURES), set(syms) - set(_lib.SIGNATURES)


def test_abi_version_and_defaults():
    L = _lib.lib()
    assert L.cdc_abi_version() == 1
    assert L.cdc_default_mask_s() == 0x0003590703530000
    assert L.cdc_default_mask_l() == 0x0000D90003530000
    o = _lib.cdc_opts()
    L.cdc_default_opts(ctypes.byref(o))
    assert (o.min_size, o.normal_size, o.max_size) == (65536, 1 << 20, 4 << 20)


def test_maskl_index_mode_setter():
    """Device-free knob: valid modes 0-3, anything else CDC_E_INVALID."""
    L = _lib.lib()
    assert L.cdc_set_maskl_index_mode(4) == _lib.CDC_E_INVALID
    assert L.cdc_set_maskl_index_mode(-1) == _lib.CDC_E_INVALID
    for m in (0, 2, 3, 1):
        assert L.cdc_set_maskl_index_mode(m) == 0


def test_default_gear_is_the_committed_placeholder():
    with open(os.path.join(ROOT, "tests", "golden", "gear_placeholder.json")) as f:
        fx = [int(x, 16) for x in json.load(f)["gear"]]
    assert _lib.default_gear() == fx


@pytest.mark.parametrize("algo,sizes,status", [
    ("fastcdc", (65536, 1 << 20, 4 << 20), _lib.CDC_OK),
    ("FASTCDC", (65536, 1 << 20, 4 << 20), _lib.CDC_OK),   # lower-cased like repository.go:288
    ("ultracdc", (65536, 1 << 20, 4 << 20), _lib.CDC_E_UNSUPPORTED),
    ("rabin", (65536, 1 << 20, 4 << 20), _lib.CDC_E_UNSUPPORTED),
    ("fastcdc", (65536, 32, 4 << 20), _lib.CDC_E_NORMAL_SIZE),
    ("fastcdc", (32, 1 << 20, 4 << 20), _lib.CDC_E_MIN_SIZE),
    ("fastcdc", (1 << 20, 1 << 20, 4 << 20), _lib.CDC_E_MIN_SIZE),
    ("fastcdc", (65536, 1 << 20, 1 << 20), _lib.CDC_E_MAX_SIZE),
    ("fastcdc", (65536, 1 << 20, (1 << 30) + 1), _lib.CDC_E_MAX_SIZE),
])
def test_validate(algo, sizes, status):
    o = _lib.cdc_opts(*sizes, 0)
    assert _lib.lib().cdc_validate(algo.encode(), ctypes.byref(o)) == status


def test_strerror_covers_all_codes():
    L = _lib.lib()
    for name in dir(_lib):
        if name.startswith("CDC_"):
            code = getattr(_lib, name)
            assert L.cdc_strerror(code).decode() != "unknown status", name


def test_workspace_size_is_device_free():
    ws = ctypes.c_uint64()
    o = _lib.cdc_opts(65536, 1 << 20, 4 << 20, 0)
    assert _lib.lib().cdc_device_workspace_size(1 << 30, ctypes.byref(o), ctypes.byref(ws)) == 0
    assert 0 < ws.value < (64 << 20)


def test_compute_entry_points_fail_loudly_without_init():
    """No CPU fallback: before cdc_init (or without a GPU) chunking returns an error."""
    L = _lib.lib()
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    o = _lib.cdc_opts(65536, 1 << 20, 4 << 20, 0)
    buf = (ctypes.c_uint8 * 100)()
    b = (_lib.cdc_buf * 1)(_lib.cdc_buf(ctypes.cast(buf, ctypes.c_void_p), 100))
    counts = (ctypes.c_uint64 * 1)()
    st = L.cdc_chunk(b, 1, ctypes.byref(o), None, 0, counts, None)
    assert st in (_lib.CDC_E_NOT_INIT, _lib.CDC_E_NO_DEVICE)
    assert L.cdc_init(0, None, 0, 0, 0) == _lib.CDC_E_NO_DEVICE


def test_host_sha256_matches_hashlib():
    """The library's host SHA-256 (the packfile index checksum and the backup
    pipeline's object checksums): the SHA-extension path and the portable
    path agree with hashlib at every padding boundary and on long inputs."""
    import ctypes
    import hashlib

    import numpy as np
    from plakar_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, size=(1 << 20) + 333, dtype=np.uint8)
    out = (ctypes.c_uint8 * 32)()
    sizes = list(range(0, 200)) + [447, 448, 511, 512, 513, 4095, 4096, 65537, (1 << 20) + 333]
    for force in (0, 1):
        for n in sizes:
            assert L.cdc_sha256(data.ctypes.data, n, force, out) == 0
            assert bytes(out) == hashlib.sha256(data[:n].tobytes()).digest(), (n, force)
    assert L.cdc_sha256(None, 1, 0, out) == _lib.CDC_E_INVALID
    assert L.cdc_sha256_accelerated() in (0, 1)
