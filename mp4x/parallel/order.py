"""The per-communicator stream-order guard (VERDICT r5 Next #1; native half in
csrc/runtime/order.hip).

One communicator's device collectives execute in the order they were issued, on every rank,
whatever streams the caller issued them on — the total order the reference gets from one send
queue and one receive queue per process (/root/reference/src/main/java/com/fenbi/mp4j/comm/
ProcessCommSlave.java:84-127) and the barrier closing every collective (:1367).  The IPC kernels'
protocols rely on it (the latency tier's double-buffered slots, the epoch flags): two calls of
one instance must never run concurrently on a rank.

Every launch of the communicator — each IPC form, the native latency fast paths, each RCCL call
through :class:`~mp4x.parallel.coll.TorchColl` — first calls :meth:`CommOrder.enter` with the
stream it is about to use.  On the stream of the previous launch that is one comparison; on
another stream the new stream first waits for an event recorded on the previous one.

Contract (DESIGN.md "Stream order"): a stream passed to a collective stays alive until the
communicator's next collective is issued (torch's pooled streams always do); inside one graph
capture every collective of the communicator is captured on one stream (a switch raises).

``MP4X_TEST_NO_STREAM_ORDER=1`` turns the join off — for tests that show the guard has teeth
(tests/test_stream_order_gpu.py); never for a job.
"""
from __future__ import annotations

import ctypes
import os

from ..ops import native

native.register_signatures({
    "mp4x_order_enter": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "mp4x_order_enter_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "mp4x_order_release": (ctypes.c_int, [ctypes.c_void_p]),
})

STREAM_SWITCH = 1005      # MP4X_E_STREAM_SWITCH (csrc/include/mp4x/ops.h)


class StreamOrder(ctypes.Structure):
    """ctypes layout of ``mp4x::StreamOrder`` (csrc/runtime/ipc_common.hpp)."""
    _fields_ = [("last", ctypes.c_void_p), ("ev", ctypes.c_void_p), ("cap_stream", ctypes.c_void_p),
                ("cap_id", ctypes.c_uint64), ("switches", ctypes.c_uint64), ("have_last", ctypes.c_int32),
                ("cap_have", ctypes.c_int32), ("disabled", ctypes.c_int32), ("pad", ctypes.c_int32)]


def disabled_by_env() -> bool:
    return os.environ.get("MP4X_TEST_NO_STREAM_ORDER", "0") == "1"


class CommOrder:
    """One communicator's guard: the native state plus its Python entry.  The latency fast paths
    get :attr:`addr` in their native state (``FastAr.order``) and call the guard themselves."""

    def __init__(self):
        self.s = StreamOrder()
        self.s.disabled = int(disabled_by_env())
        self.addr = ctypes.addressof(self.s)
        self._enter = None

    def enter(self, stream: int) -> None:
        """Order ``stream`` (a raw hipStream_t; 0 = the null stream) after the communicator's
        previous launch.  Raises on a stream switch inside one graph capture."""
        s = self.s
        cap = native.capturing_now()
        if not cap and s.have_last and (s.last or 0) == stream:
            return
        f = self._enter
        if f is None:
            f = self._enter = native.hip().mp4x_order_enter_ex
        rc = f(self.addr, stream, 1 if cap else 0)
        if rc:
            if rc == STREAM_SWITCH:
                from ..exceptions import Mp4jException
                raise Mp4jException("a communicator's collectives inside one graph capture must all be captured on "
                                    "ONE stream (stream order, DESIGN.md): capture them on one stream, or join the "
                                    "streams before capturing")
            native.check(rc, "mp4x_order_enter")

    @property
    def switches(self) -> int:
        """Stream switches joined so far."""
        return int(self.s.switches)

    def release(self) -> None:
        """Free the guard's event (the communicator's streams were drained)."""
        if self.s.ev:
            native.soft_check(native.hip().mp4x_order_release(self.addr), "mp4x_order_release")
