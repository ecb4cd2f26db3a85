"""Key hashing for the sparse ``Map<String, T>`` collectives.

* :func:`java_string_hash` reproduces ``java.lang.String.hashCode`` (31-based
  polynomial over UTF-16 code units, int32 wrap) so that key ownership in
  ``reduceScatterMap``/``allreduceMap`` partitions is bit-compatible with the
  reference's ``key.hashCode() % p`` (ProcessCommSlave.java:2059-2072).
* :func:`key_ids` maps string keys to stable 64-bit ids (xxh64) for the GPU
  sparse path, where keys travel as int64 and strings stay on the host.
"""
from __future__ import annotations

from typing import Iterable, List

import numpy as np

try:
    import xxhash as _xxhash
except Exception:  # pragma: no cover - xxhash is in the image, keep a fallback anyway
    _xxhash = None


def java_string_hash(s: str) -> int:
    h = 0
    b = s.encode("utf-16-be")
    for i in range(0, len(b), 2):
        h = (31 * h + ((b[i] << 8) | b[i + 1])) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def owner_of(key: str, p: int) -> int:
    """Reference partition rule: ``idx = hashCode % p`` (Java remainder), negatives wrapped."""
    h = java_string_hash(key)
    idx = abs(h) % p
    if h < 0 and idx != 0:
        idx = p - idx
    return idx


def partition_keys(keys: Iterable[str], p: int) -> List[int]:
    return [owner_of(k, p) for k in keys]


def key_id(key: str) -> int:
    if _xxhash is not None:
        v = _xxhash.xxh64_intdigest(key.encode("utf-8"))
    else:  # FNV-1a 64
        v = 0xCBF29CE484222325
        for c in key.encode("utf-8"):
            v = ((v ^ c) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    # keep ids non-negative int64 (bit 63 cleared) so sorting as int64 is stable
    return v & 0x7FFFFFFFFFFFFFFF


def key_ids(keys: Iterable[str]) -> np.ndarray:
    return np.fromiter((key_id(k) for k in keys), dtype=np.int64)
