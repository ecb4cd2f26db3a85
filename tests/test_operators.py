"""Port of the reference unit test (src/test/java/com/fenbi/mp4j/operator/OperatorsTest.java:32-121)
plus vectorised-vs-scalar property checks."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from mp4x import Operators
from mp4x.operators import OpCode, DType, CustomOperator, IDoubleOperator


def test_double():
    D = Operators.Double
    assert D.SUM.apply(1.0, 2.0) == 3.0
    assert D.MAX.apply(1.0, 2.0) == 2.0
    assert D.MIN.apply(1.0, 2.0) == 1.0
    assert D.PROD.apply(1.0, 2.0) == 2.0
    a, b = D.compositeDouble(1.9, 1), D.compositeDouble(1.8, 2)
    assert _bits(D.FLOAT_MAX_LOC.apply(a, b)) == _bits(a)
    assert _bits(D.FLOAT_MIN_LOC.apply(a, b)) == _bits(b)
    assert D.getIntLoc(a) == 1 and abs(D.getFloatVal(a) - 1.9) < 1e-6


def _bits(x):
    return np.array([x]).view(np.uint64)[0]


def test_float():
    F = Operators.Float
    assert F.SUM.apply(1.0, 2.0) == 3.0
    assert F.MAX.apply(1.0, 2.0) == 2.0
    assert F.MIN.apply(1.0, 2.0) == 1.0
    assert F.PROD.apply(1.0, 2.0) == 2.0


def test_long():
    L = Operators.Long
    assert L.SUM.apply(1, 2) == 3
    assert L.MAX.apply(1, 2) == 2
    assert L.MIN.apply(1, 2) == 1
    assert L.PROD.apply(1, 2) == 2
    assert L.INT_MAX_LOC.apply(L.compositeLong(19, 1), L.compositeLong(18, 2)) == L.compositeLong(19, 1)
    assert L.INT_MIN_LOC.apply(L.compositeLong(19, 1), L.compositeLong(18, 2)) == L.compositeLong(18, 2)
    assert L.BITS_AND.apply(-1, 1234) == 1234
    assert L.BITS_AND.apply(-1, -14343434) == -14343434
    assert L.BITS_OR.apply(-1, -14343434) == -1        # 0xffffffffffffffffL
    assert L.BITS_OR.apply(1234, 3456) == 3538
    assert L.BITS_XOR.apply(1234, 3456) == 2386
    assert L.getIntVal(L.compositeLong(-7, 3)) == -7 and L.getIntLoc(L.compositeLong(-7, 3)) == 3


def test_int():
    I = Operators.Int
    assert I.SUM.apply(1, 2) == 3
    assert I.MAX.apply(1, 2) == 2
    assert I.MIN.apply(1, 2) == 1
    assert I.PROD.apply(1, 2) == 2
    assert I.BITS_AND.apply(-1, 1234) == 1234
    assert I.BITS_AND.apply(-1, -14343434) == -14343434
    assert I.BITS_OR.apply(-1, -14343434) == -1        # 0xffffffff as Java int
    assert I.BITS_OR.apply(1234, 3456) == 3538
    assert I.BITS_XOR.apply(1234, 3456) == 2386
    assert I.SUM.apply(2**31 - 1, 1) == -2**31          # Java int overflow wraps


def test_short():
    S = Operators.Short
    assert S.SUM.apply(1, 2) == 3
    assert S.MAX.apply(1, 2) == 2
    assert S.MIN.apply(1, 2) == 1
    assert S.PROD.apply(1, 2) == 2
    assert S.BITS_AND.apply(-1, 1234) == 1234
    assert S.BITS_AND.apply(-1, -1434) == -1434
    assert S.BITS_OR.apply(-1, -1434) == -1
    assert S.BITS_OR.apply(1234, 3456) == 3538
    assert S.BITS_XOR.apply(1234, 3456) == 2386
    assert S.SUM.apply(32767, 1) == -32768


def test_byte():
    B = Operators.Byte
    assert B.SUM.apply(1, 2) == 3
    assert B.MAX.apply(1, 2) == 2
    assert B.MIN.apply(1, 2) == 1
    assert B.PROD.apply(1, 2) == 2
    assert B.BITS_AND.apply(-1, 12) == 12
    assert B.BITS_AND.apply(-1, -14) == -14
    assert B.BITS_OR.apply(-1, -14) == -1
    assert B.BITS_OR.apply(2, 1) == 3
    assert B.BITS_XOR.apply(-1, -1) == 0
    assert B.SUM.apply(127, 1) == -128


def test_loc_tie_prefers_first_argument():
    D = Operators.Double
    a, b = D.compositeDouble(2.5, 7), D.compositeDouble(2.5, 9)
    assert D.getIntLoc(D.FLOAT_MAX_LOC.apply(a, b)) == 7
    assert D.getIntLoc(D.FLOAT_MIN_LOC.apply(a, b)) == 7
    L = Operators.Long
    assert L.getIntLoc(L.INT_MAX_LOC.apply(L.compositeLong(5, 1), L.compositeLong(5, 2))) == 1


def test_operator_pickles_to_singleton():
    import pickle
    assert pickle.loads(pickle.dumps(Operators.Int.BITS_XOR)) is Operators.Int.BITS_XOR


def test_custom_operator():
    op = IDoubleOperator(lambda a, b: a * 10 + b)
    acc = np.array([1.0, 2.0])
    op.reduce_into(acc, np.array([3.0, 4.0]))
    assert acc.tolist() == [13.0, 24.0]
    v = CustomOperator(lambda a, b: np.maximum(a, b) * 2, vectorized=True)
    acc = np.array([1.0, 5.0])
    v.reduce_into(acc, np.array([3.0, 4.0]))
    assert acc.tolist() == [6.0, 10.0]


@settings(max_examples=60, deadline=None)
@given(st.lists(st.integers(-2**31, 2**31 - 1), min_size=1, max_size=50),
       st.lists(st.integers(-2**31, 2**31 - 1), min_size=1, max_size=50))
def test_vectorised_matches_scalar_int(xs, ys):
    n = min(len(xs), len(ys))
    a = np.array(xs[:n], dtype=np.int32)
    b = np.array(ys[:n], dtype=np.int32)
    for op in (Operators.Int.SUM, Operators.Int.PROD, Operators.Int.MAX, Operators.Int.BITS_XOR):
        acc = a.copy()
        with np.errstate(over="ignore"):
            op.reduce_into(acc, b)
        assert acc.tolist() == [op.apply(int(x), int(y)) for x, y in zip(a, b)]
