"""Per-collective tracing and metrics.

The reference only logs ad-hoc ``System.currentTimeMillis()`` deltas
(J/check/checkdouble/ProcessAllReduceCheck.java:64-66).  mp4x keeps, per communicator and
per operation name: call count, bytes, host wall time and the algorithm the engine picked.
With ``MP4X_TRACE=1`` every collective is also

* bracketed by a roctx range (``libroctx64``, visible in ``rocprofv3 --marker-trace``), and
* timed on the device with a hipEvent pair (GPU tensors) — read with :meth:`Tracer.report`.

``MP4X_TRACE_LOG=1`` additionally logs one line per call (rank-prefixed).
"""
from __future__ import annotations

import ctypes
import logging
import os
import threading
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict

LOG = logging.getLogger("mp4x.trace")

_roctx = None
_roctx_tried = False


def _roctx_lib():
    global _roctx, _roctx_tried
    if not _roctx_tried:
        _roctx_tried = True
        for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx


class Tracer:
    def __init__(self, rank: int = 0):
        self.rank = rank
        self.enabled = os.environ.get("MP4X_TRACE", "0") == "1"
        self.log_calls = os.environ.get("MP4X_TRACE_LOG", "0") == "1"
        self.calls: Dict[str, int] = defaultdict(int)
        self.bytes: Dict[str, int] = defaultdict(int)
        self.wall: Dict[str, float] = defaultdict(float)
        self.algos: Dict[str, int] = defaultdict(int)
        self._events = []
        self._lock = threading.Lock()

    def count(self, name: str, nbytes: int = 0) -> None:
        """Counters only (the untraced fast path: no context manager, no roctx, no events)."""
        with self._lock:
            self.calls[name] += 1
            self.bytes[name] += int(nbytes)

    @contextmanager
    def span(self, name: str, nbytes: int = 0, device_tensor=None):
        with self._lock:
            self.calls[name] += 1
            self.bytes[name] += int(nbytes)
        if not self.enabled:
            yield
            return
        lib = _roctx_lib()
        if lib is not None:
            lib.roctxRangePushA(f"mp4x.{name}".encode())
        ev = None
        if device_tensor is not None:
            import torch
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            dt = time.perf_counter() - t0
            if ev is not None:
                ev[1].record()
                self._events.append((name, ev))
            with self._lock:
                self.wall[name] += dt
            if lib is not None:
                lib.roctxRangePop()
            if self.log_calls:
                LOG.info("[rank=%d] %s %d B %.3f ms", self.rank, name, nbytes, dt * 1e3)

    def note_algo(self, name: str):
        with self._lock:
            self.algos[name] += 1

    def report(self) -> Dict[str, dict]:
        dev: Dict[str, float] = defaultdict(float)
        for name, (a, b) in self._events:
            b.synchronize()
            dev[name] += a.elapsed_time(b)
        out = {}
        for k in self.calls:
            out[k] = {"calls": self.calls[k], "bytes": self.bytes[k], "host_ms": self.wall[k] * 1e3}
            if k in dev:
                out[k]["device_ms"] = dev[k]
        if self.algos:
            out["_algorithms"] = dict(self.algos)
        return out
