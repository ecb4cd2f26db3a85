"""Operand descriptors — what element type a collective moves, and how.

Reference: ``Operands`` factory (/root/reference/src/main/java/com/fenbi/mp4j/operand/Operands.java:33-111)
and the stateful ``Operand`` base (J/operand/Operand.java:44-79).

In the reference an operand is a mutable object that also *is* the codec
(Kryo serializers per collective).  Here an operand is an immutable
descriptor — element kind, compression flag / codec, optional object
serializer — and the engines pick the data path from it:

* primitive kinds → contiguous numpy arrays (host) or torch tensors (device);
  payloads go over the wire as raw bytes, reductions are vectorised;
* ``STRING`` / ``OBJECT`` → Python lists, serialised by the operand's
  :class:`Serializer` (pickle by default; user-supplied like Kryo's
  ``Serializer<T>``).

``compress=True`` is the reference's Kryo ``DeflateSerializer`` wrapper
(J/operand/DoubleOperand.java:267-277): lossless zlib on the host wire, lossless
zero suppression (kernel K6b, ``codec="zs"``) for device-tensor allreduce.  On the
device path the lossy block-scaled fp8 / bf16 wire codecs (kernel K6) are
selected with ``codec="fp8"`` / ``codec="bf16"``.
"""
from __future__ import annotations

import pickle
from typing import Any, Optional

import numpy as np

from .operators import DType, NP_DTYPE


def _dumps(obj) -> bytes:
    try:
        return pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
    except (pickle.PicklingError, AttributeError, TypeError):
        import cloudpickle   # local classes / lambdas (the reference's Kryo handles any class)
        return cloudpickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)


class Serializer:
    """Host object serializer (reference: Kryo ``Serializer<T>``).

    The default implementation uses pickle; override ``write``/``read`` for a
    compact custom format.  Only data produced by the job's own ranks is ever
    deserialised.
    """

    def write(self, obj: Any) -> bytes:
        return _dumps(obj)

    def read(self, data: bytes) -> Any:
        return pickle.loads(data)

    # list helpers (one frame per list keeps the wire format simple)
    def write_list(self, objs) -> bytes:
        return pickle.dumps([self.write(o) for o in objs], protocol=pickle.HIGHEST_PROTOCOL) \
            if type(self) is not Serializer else _dumps(list(objs))

    def read_list(self, data: bytes):
        if type(self) is Serializer:
            return pickle.loads(data)
        return [self.read(b) for b in pickle.loads(data)]


class StringSerializer(Serializer):
    def write(self, obj):
        return obj.encode("utf-8")

    def read(self, data):
        return bytes(data).decode("utf-8")


DEFAULT_SERIALIZER = Serializer()


class KryoUtils:
    """Reference: J/utils/KryoUtils.java:33-46 — default serializer per class."""

    @staticmethod
    def getDefaultSerializer(cls=None) -> Serializer:
        if cls is str:
            return StringSerializer()
        return DEFAULT_SERIALIZER


class Operand:
    """Immutable element descriptor."""

    __slots__ = ("kind", "dtype", "compress", "serializer", "elem_type", "codec")

    def __init__(self, kind: str, dtype: Optional[DType], compress: bool = False,
                 serializer: Optional[Serializer] = None, elem_type=None, codec: Optional[str] = None):
        self.kind = kind
        self.dtype = dtype
        self.compress = bool(compress)
        self.serializer = serializer
        self.elem_type = elem_type
        if codec not in (None, "none", "zlib", "fp8", "bf16", "zs"):
            raise ValueError(f"unknown codec {codec!r}")
        self.codec = None if codec == "none" else codec

    @property
    def is_primitive(self) -> bool:
        return self.dtype is not None

    @property
    def np_dtype(self):
        return NP_DTYPE.get(self.dtype)

    def isCompress(self) -> bool:
        return self.compress

    def __repr__(self):
        extra = ", compress" if self.compress else ""
        if self.codec:
            extra += f", codec={self.codec}"
        return f"Operand({self.kind}{extra})"

    def __reduce__(self):
        return (Operand, (self.kind, self.dtype, self.compress, self.serializer, self.elem_type, self.codec))

    # scalar boxing used by broadcast/reduce/allreduce of a single value
    def box(self, value):
        if self.is_primitive:
            return np.array([value], dtype=self.np_dtype)
        return [value]

    def unbox(self, arr):
        v = arr[0]
        return v.item() if isinstance(v, np.generic) else v


class Operands:
    """Factory mirroring ``com.fenbi.mp4j.operand.Operands``."""

    @staticmethod
    def DOUBLE_OPERAND(compress: bool = False) -> Operand:
        return Operand("double", DType.F64, compress)

    @staticmethod
    def FLOAT_OPERAND(compress: bool = False, codec: Optional[str] = None) -> Operand:
        return Operand("float", DType.F32, compress, codec=codec)

    @staticmethod
    def LONG_OPERAND(compress: bool = False) -> Operand:
        return Operand("long", DType.I64, compress)

    @staticmethod
    def INT_OPERAND(compress: bool = False) -> Operand:
        return Operand("int", DType.I32, compress)

    @staticmethod
    def SHORT_OPERAND(compress: bool = False) -> Operand:
        return Operand("short", DType.I16, compress)

    @staticmethod
    def BYTE_OPERAND(compress: bool = False) -> Operand:
        return Operand("byte", DType.I8, compress)

    @staticmethod
    def STRING_OPERAND(compress: bool = False) -> Operand:
        return Operand("string", None, compress, StringSerializer(), str)

    @staticmethod
    def OBJECT_OPERAND(serializer: Optional[Serializer] = None, elem_type=None, compress: bool = False) -> Operand:
        return Operand("object", None, compress, serializer or DEFAULT_SERIALIZER, elem_type)

    # ---- new device dtypes -------------------------------------------------
    @staticmethod
    def BF16_OPERAND(codec: Optional[str] = None) -> Operand:
        return Operand("bf16", DType.BF16, False, codec=codec)

    @staticmethod
    def HALF_OPERAND(codec: Optional[str] = None) -> Operand:
        return Operand("half", DType.F16, False, codec=codec)


def operand_for_numpy(arr: np.ndarray) -> Operand:
    from .operators import dtype_of_numpy
    dt = dtype_of_numpy(arr.dtype)
    return Operand(dt.name.lower(), dt)
