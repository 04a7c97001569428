"""Mirror of plakar chunking/chunking_test.go:8-36 (the only reference test on
this path), run against the Python mirror of the package."""
from plakar_amd.chunkers import ChunkerOpts
from plakar_amd.chunking import DefaultConfiguration


def test_default_algorithm():
    expected = "FASTCDC"
    result = DefaultConfiguration().Algorithm
    assert result == expected, f"DefaultAlgorithm failed: expected {expected}, got {result}"


def test_default_configuration():
    expected = ChunkerOpts(MinSize=64 * 1024, NormalSize=1 * 1024 * 1024, MaxSize=4 * 1024 * 1024)
    result = DefaultConfiguration()
    assert int(result.MinSize) == expected.MinSize
    assert int(result.NormalSize) == expected.NormalSize
    assert int(result.MaxSize) == expected.MaxSize
