"""CPU tests of the oracle restatement: golden vectors, a second (pure-Python)
restatement, and the chunker contract's properties.  No GPU."""
import json
import os

import numpy as np
import pytest

from datagen import draw_masks, gear_table, low_entropy, random_bytes
from oracle_ref import DEFAULT_MASK_L, DEFAULT_MASK_S, py_algorithm, py_chunk

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden():
    with open(os.path.join(GOLDEN, "golden_vectors.json")) as f:
        return json.load(f)


def _inputs():
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden
    return make_golden


@pytest.mark.parametrize("case", _golden()["cases"], ids=lambda c: c["name"])
def test_oracle_matches_golden(oracle, case):
    mg = _inputs()
    data = mg.make_input(case["input"])
    import hashlib
    assert hashlib.sha256(data.tobytes()).hexdigest() == case["input_sha256"], "input generator drifted"
    cuts = oracle.chunk(data, mg.gear_for(case["gear"]), cut_adj=case["cut_adj"], **case["params"])
    assert [int(x) for x in cuts[:, 1]] == case["lengths"]
    assert int(cuts[:, 1].sum()) == data.size


def test_chunkify_routing_golden(oracle):
    mg = _inputs()
    g = _golden()
    for r in g["chunkify"]:
        data = random_bytes(r["size"], 99)
        cuts = oracle.chunk(data, mg.placeholder_gear(), chunkify=True, **mg.DEF)
        assert [int(x) for x in cuts[:, 1]] == r["lengths"]
    # snapshot/backup.go:631-644: empty -> one empty chunk; < MinSize -> one chunk
    assert g["chunkify"][0]["lengths"] == [0]
    assert g["chunkify"][1]["lengths"] == [1]
    assert g["chunkify"][2]["lengths"] == [65535]
    assert g["chunkify"][3]["lengths"] == [65536]


def test_placeholder_gear_fixture_matches_generator():
    mg = _inputs()
    with open(os.path.join(GOLDEN, "gear_placeholder.json")) as f:
        fx = [int(x, 16) for x in json.load(f)["gear"]]
    assert fx == mg.placeholder_gear()


PARAMS = [
    dict(min_size=64, normal_size=256, max_size=1024),
    dict(min_size=64, normal_size=100, max_size=130),   # Normal - Min < W - 1: truncated window crosses Normal
    dict(min_size=128, normal_size=4096, max_size=4097),
    dict(min_size=1000, normal_size=3000, max_size=10000),
]


@pytest.mark.parametrize("params", PARAMS)
@pytest.mark.parametrize("cut_adj", [0, 1])
@pytest.mark.parametrize("kind", ["random", "low_entropy", "zeros"])
def test_oracle_matches_python_restatement(oracle, params, cut_adj, kind):
    n = 40000
    data = {"random": lambda: random_bytes(n, 1), "low_entropy": lambda: low_entropy(n, 2, 0.03),
            "zeros": lambda: np.zeros(n, np.uint8)}[kind]()
    for gseed in (1, 2):
        gear = gear_table(gseed)
        if kind == "zeros" and gseed == 2:
            gear[0] = 0  # dense: every all-zero window hits
        c = oracle.chunk(data, gear, cut_adj=cut_adj, **params)
        ref = py_chunk(data.tobytes(), gear, cut_adj=cut_adj, **params)
        assert [tuple(map(int, r)) for r in c] == ref


def test_algorithm_edge_windows(oracle):
    """(*FastCDC).Algorithm at n <= Min, n == Max, n in (Min, Normal], (Normal, Max)."""
    gear = gear_table(3)
    p = dict(min_size=64, normal_size=256, max_size=1024)
    data = random_bytes(4096, 3).tobytes()
    for n in [0, 1, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025, 4096]:
        d = data[:n]
        assert oracle.algorithm(d, gear, **p) == py_algorithm(d, gear, **p), n
    assert oracle.algorithm(data[:64], gear, **p) == 64   # n <= Min: whole window


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_contract_properties(oracle, seed):
    """Every chunk >= Min except the last; every chunk <= Max; lengths sum to n;
    offsets are the prefix sums."""
    p = dict(min_size=4096, normal_size=16384, max_size=65536)
    data = np.concatenate([random_bytes(1 << 20, seed), np.zeros(300000, np.uint8),
                           low_entropy(500000, seed, 0.01)])
    for gear in (gear_table(seed), gear_table(seed + 10)):
        c = oracle.chunk(data, gear, **p)
        lens = c[:, 1].astype(np.int64)
        assert lens.sum() == data.size
        assert (lens[:-1] >= p["min_size"]).all() and (lens <= p["max_size"]).all()
        assert (c[1:, 0] == np.cumsum(lens)[:-1]).all() and c[0, 0] == 0


def test_validate_bounds(oracle):
    assert oracle.validate(65536, 1 << 20, 4 << 20) == 0
    assert oracle.validate(65536, 63, 4 << 20) == -1
    assert oracle.validate(63, 1 << 20, 4 << 20) == -2
    assert oracle.validate(1 << 20, 1 << 20, 4 << 20) == -2
    assert oracle.validate(65536, 1 << 20, 1 << 20) == -3
    assert oracle.validate(65536, 1 << 20, (1 << 30) + 1) == -3


@pytest.mark.parametrize("seed", range(12))
def test_oracle_random_masks_match_python(oracle, seed):
    """Random masks (the ones tests/test_gpu_fuzz.py draws: nested, mostly
    shared, independent) and parameters: the C oracle and the pure-Python
    restatement agree, so the GPU fuzz cases are checked against a restatement
    that is itself cross-checked."""
    rng = np.random.default_rng(np.random.PCG64(9000 + seed))
    ms, ml = draw_masks(rng, (DEFAULT_MASK_S, DEFAULT_MASK_L))
    mn = 64 << int(rng.integers(0, 4))
    p = dict(min_size=mn, normal_size=mn << int(rng.integers(1, 4)), max_size=0)
    p["max_size"] = p["normal_size"] << int(rng.integers(1, 3))
    data = np.concatenate([random_bytes(12000, seed), low_entropy(12000, seed + 1, 0.02),
                           np.zeros(4000, np.uint8)])
    gear = gear_table(9100 + seed)
    cut_adj = int(rng.integers(0, 2))
    c = oracle.chunk(data, gear, mask_s=ms, mask_l=ml, cut_adj=cut_adj, **p)
    ref = py_chunk(data.tobytes(), gear, mask_s=ms, mask_l=ml, cut_adj=cut_adj, **p)
    assert [tuple(map(int, r)) for r in c] == ref, f"masks {ms:#x}/{ml:#x} {p}"
