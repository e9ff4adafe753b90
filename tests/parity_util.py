"""Bit-level comparison helpers shared by the parity tests (CPU-importable: no GPU marker)."""
import numpy as np


def bits(a):
    """float32 bit patterns of `a`; every NaN maps to one pattern (payloads are not part of
    the contract)."""
    a = np.array(a, np.float32)  # keeps 0-d inputs 0-d (ascontiguousarray would make them 1-d)
    b = a.view(np.uint32).copy()
    b[np.isnan(a)] = 0x7FC00000
    return b


def assert_bits_equal(x, y, what):
    """x and y hold the same float32 bits.  Scalars (0-d) and arrays of any shape: the
    message names the count and the first mismatch with both values."""
    bx, by = bits(x), bits(y)
    assert bx.shape == by.shape, f"{what}: shape {bx.shape} vs {by.shape}"
    if bx.ndim == 0:
        assert bx == by, f"{what}: {np.float32(x)!r} ({int(bx):#010x}) vs {np.float32(y)!r} ({int(by):#010x})"
        return
    bad = np.nonzero(bx != by)
    if len(bad[0]):
        at = tuple(int(i[0]) for i in bad)
        xa, ya = np.asarray(x, np.float32), np.asarray(y, np.float32)
        raise AssertionError(f"{what}: {len(bad[0])} mismatches, first at {at}: {xa[at]!r} vs {ya[at]!r}")
