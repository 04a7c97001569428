"""Runs the C-level boundary test (tests/c/abi_threads.c, built by
__graft_entry__.build()): a read-callback chunker, cdc_chunk from 8 threads at
once and the pinned file arena, every result compared with the oracle."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "abi_threads")


def test_c_boundary_threads_callback_files():
    assert os.path.exists(EXE), "build it with __graft_entry__.build()"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=180)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.strip().endswith("OK")
