"""Dump Encode frames that liblz4 rejects (debugging aid): python tools/enc_debug.py <outdir>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import crypto_ref as ref  # noqa: E402
from datagen import low_entropy  # noqa: E402
from plakar_amd import _lib, encode  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
_lib.ensure_init()
sizes = [0, 1, 15, 16, 17, 4095, 16384, 16385, 65535, 65536, 65537, (1 << 20) + 13, 4 << 20]
blobs = [low_entropy(n, 600 + i).tobytes() for i, n in enumerate(sizes)]
outs = encode.encode_blobs(blobs, key=None, compress=True)
for i, (b, o) in enumerate(zip(blobs, outs)):
    try:
        ok = ref.lz4f_decompress(o) == b
        err = "" if ok else "content differs"
    except ValueError as e:
        ok, err = False, str(e)
    print(i, len(b), len(o), "ok" if ok else "FAIL " + err)
    if not ok:
        open(f"{out}/blob{i}.bin", "wb").write(b)
        open(f"{out}/frame{i}.bin", "wb").write(o)
