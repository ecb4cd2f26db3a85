"""TCP host engine's reduce-on-receive through the native multi-threaded reduce
(host_engine._native_reduce): bit-identical to the numpy path it replaces, for every built-in
dtype the runtime takes, incl. NaN propagation and integer wrap-around; unaligned frames and
custom operators fall back to numpy.  Reference: the reduce-on-receive hot loop,
J/operand/DoubleOperand.java:196."""
import os

import numpy as np
import pytest

from mp4x import Operators
from mp4x.ops import native
from mp4x.parallel.host_engine import _native_reduce, _reduce_segment

pytestmark = pytest.mark.skipif(not os.path.exists(native.HOST_LIB), reason="host library not built")

N = (1 << 18) + 37


@pytest.mark.parametrize("dt,ops", [(np.float64, Operators.Double), (np.float32, Operators.Float),
                                    (np.int64, Operators.Long), (np.int32, Operators.Int),
                                    (np.int16, Operators.Short), (np.int8, Operators.Byte)])
@pytest.mark.parametrize("name", ["SUM", "MAX", "MIN", "PROD"])
def test_native_matches_numpy(dt, ops, name):
    rng = np.random.default_rng(7)
    if np.issubdtype(dt, np.floating):
        a = rng.standard_normal(N).astype(dt)
        b = rng.standard_normal(N).astype(dt)
        a[::1001] = np.nan
        b[5::997] = np.nan
    else:
        info = np.iinfo(dt)
        a = rng.integers(info.min, info.max, N, dtype=dt, endpoint=True)
        b = rng.integers(info.min, info.max, N, dtype=dt, endpoint=True)
    op = getattr(ops, name)
    want = a.copy()
    with np.errstate(over="ignore", invalid="ignore"):
        op.reduce_into(want, b)
    got = a.copy()
    assert _native_reduce(got, b, op)
    np.testing.assert_array_equal(got.view(np.uint8), want.view(np.uint8))


def test_unaligned_frame_falls_back():
    a = np.arange(N, dtype=np.float64)
    raw = bytearray(N * 8 + 3)
    b = np.frombuffer(raw, dtype=np.float64, count=N, offset=3)   # a frame at an odd byte offset
    assert not _native_reduce(a.copy(), b, Operators.Double.SUM)
    out = a.copy()
    _reduce_segment(out, 0, N, b, Operators.Double.SUM)          # numpy path, same answer
    np.testing.assert_array_equal(out, a + b)


def test_custom_and_mismatched_dtype_fall_back():
    a = np.ones(N)
    assert not _native_reduce(a, np.ones(N, np.float32), Operators.Double.SUM)
    assert not _native_reduce(a, np.ones(N), Operators.Float.SUM)
