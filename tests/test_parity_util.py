"""CPU unit tests of the parity helpers (tests/parity_util.py)."""
import numpy as np
import pytest

from tests.parity_util import assert_bits_equal, bits


def test_scalar_mismatch_reports_both_values():
    # the round-2 failure: a 0-d cost mismatch raised IndexError and lost the report
    with pytest.raises(AssertionError) as e:
        assert_bits_equal(np.float32(24.0085), np.float32(33.0305), "harness cost")
    msg = str(e.value)
    assert "harness cost" in msg and "24.0085" in msg and "33.0305" in msg


def test_scalar_and_array_equal_pass():
    assert_bits_equal(np.float32(1.5), np.float32(1.5), "scalar")
    assert_bits_equal(np.arange(6, dtype=np.float32).reshape(2, 3), np.arange(6, dtype=np.float32).reshape(2, 3), "2d")


def test_array_mismatch_names_first_index():
    a = np.zeros((3, 4), np.float32)
    b = a.copy()
    b[1, 2] = 7.0
    b[2, 0] = 1.0
    with pytest.raises(AssertionError) as e:
        assert_bits_equal(a, b, "path")
    assert "2 mismatches" in str(e.value) and "(1, 2)" in str(e.value)


def test_bits_distinguish_signed_zero_and_unify_nans():
    assert bits(np.float32(0.0)) != bits(np.float32(-0.0))
    n1 = np.array([np.nan], np.float32)
    n2 = np.array([0x7FC00001], np.uint32).view(np.float32)
    assert_bits_equal(n1, n2, "nan payloads")


def test_shape_mismatch():
    with pytest.raises(AssertionError, match="shape"):
        assert_bits_equal(np.zeros(3, np.float32), np.zeros(4, np.float32), "len")
