"""Encode's OS random bytes drawn ahead (plakar_amd.encode._Reservoir): every
call gets fresh bytes -- never bytes another call, or a forked child, also
got -- since the subkeys and GCM nonces of EncryptStream
(encryption/symmetric.go:72-163, crypto/rand there) come from them."""
import os
import time

from plakar_amd import encode


def _fresh():
    r = encode._Reservoir(target=1 << 20)
    r.take(1)  # starts the filler
    t0 = time.monotonic()
    while r.have < r.target and time.monotonic() - t0 < 10:  # a loaded host may be slow to fill
        time.sleep(0.05)
    return r


def test_takes_are_fresh_and_sized():
    r = _fresh()
    seen = set()
    for n in (56, 1000, 300_000, 1 << 20, 3 << 20):  # inside, across and past the reservoir
        a = bytes(r.take_into(n))
        b = r.take(n)
        assert len(a) == n and len(b) == n
        for x in (a, b):
            for i in range(0, n - 32, max(32, n // 64)):
                k = x[i:i + 32]
                assert k not in seen
                seen.add(k)


def test_forked_child_never_reuses_the_parents_bytes():
    r = _fresh()
    assert r.have > 0
    rd, wr = os.pipe()
    pid = os.fork()
    if pid == 0:
        try:
            os.close(rd)
            os.write(wr, bytes(r.take_into(64)))
        finally:
            os._exit(0)
    os.close(wr)
    child = b""
    while len(child) < 64:
        part = os.read(rd, 64)
        if not part:
            break
        child += part
    os.close(rd)
    os.waitpid(pid, 0)
    parent = r.take(r.have)  # everything the parent still holds
    assert len(child) == 64 and child not in parent
