"""Reduction operators, collective / container enums.

Behavioural parity with the reference's ``Operators`` table
(/root/reference/src/main/java/com/fenbi/mp4j/operator/Operators.java:29-353):

* Double: SUM MAX MIN PROD FLOAT_MAX_LOC FLOAT_MIN_LOC (+ compositeDouble /
  getFloatVal / getIntLoc helpers, :57-89)
* Float:  SUM MAX MIN PROD (:91-117)
* Long:   SUM MAX MIN BITS_AND BITS_OR BITS_XOR PROD INT_MAX_LOC INT_MIN_LOC
  (+ compositeLong / getIntVal / getIntLoc, :119-202)
* Int / Short / Byte: SUM MAX MIN BITS_AND BITS_OR BITS_XOR PROD (:204-351)

Integer arithmetic wraps like Java (two's complement), ``*_LOC`` ties prefer
the first (local) argument (``>=`` / ``<=``).

Design (not a translation): an :class:`Operator` is an immutable descriptor
``(dtype, op-code)``.  The op-code is shared with the native kernels
(``csrc/include/mp4x/ops.h``) so the same object drives

* the host path — vectorised numpy ``reduce_into(acc, x)``,
* the device path — the hand-written HIP reduce kernels (K1/K2) or an RCCL
  reduction where RCCL supports the (dtype, op) pair,
* scalar ``apply(a, b)`` (the reference's ``IXxxOperator.apply``).

User defined operators (the reference's anonymous ``IDoubleOperator`` etc.)
are :class:`CustomOperator` instances wrapping a Python callable; they run on
the host path or, if marked ``vectorized``, on torch tensors for the device
path.
"""
from __future__ import annotations

import enum
import struct
from typing import Any, Callable, Optional

import numpy as np


class Collective(enum.Enum):
    """Reference: ``J/operator/Collective.java:29-36``."""
    GATHER = 0
    SCATTER = 1
    ALL_GATHER = 2
    BROADCAST = 3
    REDUCE_SCATTER = 4
    REDUCE = 5
    ALL_REDUCE = 6


class Container(enum.Enum):
    """Reference: ``J/operator/Container.java:29-31``."""
    ARRAY = 0
    MAP = 1


class OpCode(enum.IntEnum):
    """Must match ``enum mp4x_op`` in csrc/include/mp4x/ops.h."""
    SUM = 0
    MAX = 1
    MIN = 2
    PROD = 3
    BAND = 4
    BOR = 5
    BXOR = 6
    FMAXLOC = 7   # f64 word = (f32 value in hi 32 bits, int32 loc in lo 32 bits)
    FMINLOC = 8
    IMAXLOC = 9   # i64 word = (int32 value in hi 32 bits, int32 loc in lo 32 bits)
    IMINLOC = 10


class DType(enum.IntEnum):
    """Must match ``enum mp4x_dtype`` in csrc/include/mp4x/ops.h."""
    F64 = 0
    F32 = 1
    I64 = 2
    I32 = 3
    I16 = 4
    I8 = 5
    BF16 = 6
    F16 = 7
    U8 = 8


NP_DTYPE = {
    DType.F64: np.dtype(np.float64), DType.F32: np.dtype(np.float32),
    DType.I64: np.dtype(np.int64), DType.I32: np.dtype(np.int32),
    DType.I16: np.dtype(np.int16), DType.I8: np.dtype(np.int8),
    DType.F16: np.dtype(np.float16), DType.U8: np.dtype(np.uint8),
}

_DTYPE_BY_NP = {v: k for k, v in NP_DTYPE.items()}


def dtype_of_numpy(dt) -> DType:
    return _DTYPE_BY_NP[np.dtype(dt)]


_TORCH_DT = None


def dtype_of_torch(t) -> DType:
    global _TORCH_DT
    if _TORCH_DT is None:    # built once: this is on every device collective's path
        import torch
        _TORCH_DT = {
            torch.float64: DType.F64, torch.float32: DType.F32, torch.int64: DType.I64,
            torch.int32: DType.I32, torch.int16: DType.I16, torch.int8: DType.I8,
            torch.bfloat16: DType.BF16, torch.float16: DType.F16, torch.uint8: DType.U8,
        }
    return _TORCH_DT[t]


def torch_dtype_of(dt: DType):
    import torch
    return {
        DType.F64: torch.float64, DType.F32: torch.float32, DType.I64: torch.int64,
        DType.I32: torch.int32, DType.I16: torch.int16, DType.I8: torch.int8,
        DType.BF16: torch.bfloat16, DType.F16: torch.float16, DType.U8: torch.uint8,
    }[dt]


# --------------------------------------------------------------------------- helpers
def _hi32_as_f32(u64: np.ndarray) -> np.ndarray:
    return (u64 >> np.uint64(32)).astype(np.uint32).view(np.float32)


def _hi32_as_i32(u64: np.ndarray) -> np.ndarray:
    return (u64 >> np.uint64(32)).astype(np.uint32).view(np.int32)


class Operator:
    """A predefined reduction ``(dtype, op)``.

    ``reduce_into(acc, x)`` computes ``acc[i] = op(acc[i], x[i])`` in place —
    local value first, incoming value second, exactly the argument order of the
    reference's fused recv+reduce loop (``J/operand/DoubleOperand.java:196``).
    """

    __slots__ = ("dtype", "code", "name", "commutative")

    def __init__(self, dtype: DType, code: OpCode, name: str):
        self.dtype = dtype
        self.code = code
        self.name = name
        # *_LOC ops are commutative except for exact-tie ordering; all ops here are associative.
        self.commutative = True

    is_custom = False
    vectorized = True

    def __repr__(self):
        return f"Operators.{self.dtype.name}.{self.name}"

    def __reduce__(self):
        return (_lookup_operator, (int(self.dtype), int(self.code)))

    # --- vectorised host implementation -----------------------------------
    def reduce_into(self, acc: np.ndarray, x: np.ndarray) -> np.ndarray:
        c = self.code
        if c == OpCode.SUM:
            np.add(acc, x, out=acc)
        elif c == OpCode.MAX:
            np.maximum(acc, x, out=acc)
        elif c == OpCode.MIN:
            np.minimum(acc, x, out=acc)
        elif c == OpCode.PROD:
            np.multiply(acc, x, out=acc)
        elif c == OpCode.BAND:
            np.bitwise_and(acc, x, out=acc)
        elif c == OpCode.BOR:
            np.bitwise_or(acc, x, out=acc)
        elif c == OpCode.BXOR:
            np.bitwise_xor(acc, x, out=acc)
        else:
            ua = acc.view(np.uint64)
            ux = np.ascontiguousarray(x).view(np.uint64)
            if c in (OpCode.FMAXLOC, OpCode.FMINLOC):
                va, vx = _hi32_as_f32(ua), _hi32_as_f32(ux)
            else:
                va, vx = _hi32_as_i32(ua), _hi32_as_i32(ux)
            keep = (va >= vx) if c in (OpCode.FMAXLOC, OpCode.IMAXLOC) else (va <= vx)
            np.copyto(ua, ux, where=~keep)
        return acc

    def reduce_many(self, acc: np.ndarray, xs) -> np.ndarray:
        for x in xs:
            self.reduce_into(acc, x)
        return acc

    # --- scalar (the reference's IXxxOperator.apply) ----------------------
    def apply(self, a, b):
        npdt = NP_DTYPE[self.dtype]
        if self.code in (OpCode.FMAXLOC, OpCode.FMINLOC, OpCode.IMAXLOC, OpCode.IMINLOC):
            aa = np.array([a], dtype=npdt)
            bb = np.array([b], dtype=npdt)
        else:
            aa = np.array([_wrap(a, npdt)], dtype=npdt)
            bb = np.array([_wrap(b, npdt)], dtype=npdt)
        with np.errstate(over="ignore", invalid="ignore"):
            self.reduce_into(aa, bb)
        return aa[0].item()

    __call__ = apply


def _wrap(v, npdt):
    """Java-like narrowing of a Python int into the dtype's range."""
    if npdt.kind == "i" and isinstance(v, (int, np.integer)):
        bits = npdt.itemsize * 8
        v = int(v) & ((1 << bits) - 1)
        if v >= 1 << (bits - 1):
            v -= 1 << bits
    return v


class CustomOperator:
    """User operator (reference: anonymous ``I<Type>Operator`` / ``IObjectOperator``).

    ``fn(a, b)`` is applied elementwise (host path).  With ``vectorized=True`` it
    is called once per block with two arrays/tensors and must return the
    reduced block (works on numpy arrays and on device tensors).
    """

    is_custom = True
    commutative = False

    def __init__(self, fn: Callable[[Any, Any], Any], dtype: Optional[DType] = None,
                 vectorized: bool = False, name: str = "custom"):
        self.fn = fn
        self.dtype = dtype
        self.vectorized = vectorized
        self.name = name
        self.code = None

    def apply(self, a, b):
        return self.fn(a, b)

    __call__ = apply

    def reduce_into(self, acc, x):
        if self.vectorized:
            r = self.fn(acc, x)
            acc[...] = r
            return acc
        if isinstance(acc, np.ndarray):
            for i in range(len(acc)):
                acc[i] = self.fn(acc[i], x[i])
        else:  # python list of objects
            for i in range(len(acc)):
                acc[i] = self.fn(acc[i], x[i])
        return acc

    def __repr__(self):
        return f"CustomOperator({self.name})"


# Reference interface names, for users porting code: IDoubleOperator(fn) etc.
def IDoubleOperator(fn):
    return CustomOperator(fn, DType.F64)


def IFloatOperator(fn):
    return CustomOperator(fn, DType.F32)


def ILongOperator(fn):
    return CustomOperator(fn, DType.I64)


def IIntOperator(fn):
    return CustomOperator(fn, DType.I32)


def IShortOperator(fn):
    return CustomOperator(fn, DType.I16)


def IByteOperator(fn):
    return CustomOperator(fn, DType.I8)


def IStringOperator(fn):
    return CustomOperator(fn, None, name="string")


def IObjectOperator(fn):
    return CustomOperator(fn, None, name="object")


# --------------------------------------------------------------------------- table
_REGISTRY = {}


def _mk(dtype: DType, code: OpCode, name: str) -> Operator:
    op = Operator(dtype, code, name)
    _REGISTRY[(int(dtype), int(code))] = op
    return op


def _lookup_operator(dtype: int, code: int) -> Operator:
    return _REGISTRY[(dtype, code)]


def lookup(dtype: DType, code: OpCode) -> Operator:
    """Return the operator for (dtype, code), creating it for extra dtypes (bf16/f16/u8)."""
    key = (int(dtype), int(code))
    if key not in _REGISTRY:
        _mk(DType(dtype), OpCode(code), OpCode(code).name)
    return _REGISTRY[key]


class Operators:
    """Namespace mirroring ``com.fenbi.mp4j.operator.Operators``."""

    class Double:
        SUM = _mk(DType.F64, OpCode.SUM, "SUM")
        MAX = _mk(DType.F64, OpCode.MAX, "MAX")
        MIN = _mk(DType.F64, OpCode.MIN, "MIN")
        PROD = _mk(DType.F64, OpCode.PROD, "PROD")
        FLOAT_MAX_LOC = _mk(DType.F64, OpCode.FMAXLOC, "FLOAT_MAX_LOC")
        FLOAT_MIN_LOC = _mk(DType.F64, OpCode.FMINLOC, "FLOAT_MIN_LOC")

        @staticmethod
        def compositeDouble(val: float, loc: int) -> float:
            """Pack (float32 value, int32 loc) into one double's raw bits (Operators.java:76-81)."""
            hi = struct.unpack("<I", struct.pack("<f", val))[0]
            bits = (hi << 32) | (loc & 0xFFFFFFFF)
            return struct.unpack("<d", struct.pack("<Q", bits))[0]

        @staticmethod
        def getFloatVal(composite: float) -> float:
            bits = struct.unpack("<Q", struct.pack("<d", composite))[0]
            return struct.unpack("<f", struct.pack("<I", bits >> 32))[0]

        @staticmethod
        def getIntLoc(composite: float) -> int:
            bits = struct.unpack("<Q", struct.pack("<d", composite))[0]
            return struct.unpack("<i", struct.pack("<I", bits & 0xFFFFFFFF))[0]

    class Float:
        SUM = _mk(DType.F32, OpCode.SUM, "SUM")
        MAX = _mk(DType.F32, OpCode.MAX, "MAX")
        MIN = _mk(DType.F32, OpCode.MIN, "MIN")
        PROD = _mk(DType.F32, OpCode.PROD, "PROD")

    class Long:
        SUM = _mk(DType.I64, OpCode.SUM, "SUM")
        MAX = _mk(DType.I64, OpCode.MAX, "MAX")
        MIN = _mk(DType.I64, OpCode.MIN, "MIN")
        BITS_AND = _mk(DType.I64, OpCode.BAND, "BITS_AND")
        BITS_OR = _mk(DType.I64, OpCode.BOR, "BITS_OR")
        BITS_XOR = _mk(DType.I64, OpCode.BXOR, "BITS_XOR")
        PROD = _mk(DType.I64, OpCode.PROD, "PROD")
        INT_MAX_LOC = _mk(DType.I64, OpCode.IMAXLOC, "INT_MAX_LOC")
        INT_MIN_LOC = _mk(DType.I64, OpCode.IMINLOC, "INT_MIN_LOC")

        @staticmethod
        def compositeLong(val: int, loc: int) -> int:
            bits = ((val & 0xFFFFFFFF) << 32) | (loc & 0xFFFFFFFF)
            return _wrap(bits, np.dtype(np.int64))

        @staticmethod
        def getIntVal(composite: int) -> int:
            return _wrap((composite >> 32) & 0xFFFFFFFF, np.dtype(np.int32))

        @staticmethod
        def getIntLoc(composite: int) -> int:
            return _wrap(composite & 0xFFFFFFFF, np.dtype(np.int32))

    class Int:
        SUM = _mk(DType.I32, OpCode.SUM, "SUM")
        MAX = _mk(DType.I32, OpCode.MAX, "MAX")
        MIN = _mk(DType.I32, OpCode.MIN, "MIN")
        BITS_AND = _mk(DType.I32, OpCode.BAND, "BITS_AND")
        BITS_OR = _mk(DType.I32, OpCode.BOR, "BITS_OR")
        BITS_XOR = _mk(DType.I32, OpCode.BXOR, "BITS_XOR")
        PROD = _mk(DType.I32, OpCode.PROD, "PROD")

    class Short:
        SUM = _mk(DType.I16, OpCode.SUM, "SUM")
        MAX = _mk(DType.I16, OpCode.MAX, "MAX")
        MIN = _mk(DType.I16, OpCode.MIN, "MIN")
        BITS_AND = _mk(DType.I16, OpCode.BAND, "BITS_AND")
        BITS_OR = _mk(DType.I16, OpCode.BOR, "BITS_OR")
        BITS_XOR = _mk(DType.I16, OpCode.BXOR, "BITS_XOR")
        PROD = _mk(DType.I16, OpCode.PROD, "PROD")

    class Byte:
        SUM = _mk(DType.I8, OpCode.SUM, "SUM")
        MAX = _mk(DType.I8, OpCode.MAX, "MAX")
        MIN = _mk(DType.I8, OpCode.MIN, "MIN")
        BITS_AND = _mk(DType.I8, OpCode.BAND, "BITS_AND")
        BITS_OR = _mk(DType.I8, OpCode.BOR, "BITS_OR")
        BITS_XOR = _mk(DType.I8, OpCode.BXOR, "BITS_XOR")
        PROD = _mk(DType.I8, OpCode.PROD, "PROD")

    # Device-only dtypes (new in mp4x; the reference has no 16-bit floats).
    class BFloat16:
        SUM = _mk(DType.BF16, OpCode.SUM, "SUM")
        MAX = _mk(DType.BF16, OpCode.MAX, "MAX")
        MIN = _mk(DType.BF16, OpCode.MIN, "MIN")
        PROD = _mk(DType.BF16, OpCode.PROD, "PROD")

    class Half:
        SUM = _mk(DType.F16, OpCode.SUM, "SUM")
        MAX = _mk(DType.F16, OpCode.MAX, "MAX")
        MIN = _mk(DType.F16, OpCode.MIN, "MIN")
        PROD = _mk(DType.F16, OpCode.PROD, "PROD")


def for_dtype(op: Operator, dtype: DType) -> Operator:
    """Same op-code re-targeted at another dtype (e.g. SUM for bf16 tensors)."""
    if op.is_custom or op.dtype == dtype:
        return op
    return lookup(dtype, op.code)
