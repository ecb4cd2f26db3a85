"""Shared-memory data plane for ranks that share a host (host arrays).

The reference moves every message over a fresh TCP connection even between processes on
the same machine (ProcessCommSlave.java:391-425).  When every rank's advertised address is
the same host, mp4x maps ONE /dev/shm segment (a 4 KiB header + one slot per rank) into all
ranks and runs the collectives in C++ (csrc/host/host_ops.cpp): copies and rank-ordered
reductions at memory bandwidth, OpenMP-parallel, a process-shared atomic barrier between
phases.  Rank 0 creates the segment and unlinks it as soon as everyone attached, so no
/dev/shm file outlives the job.

Used by ProcessComm's host path for primitive arrays >= ``MP4X_SHM_MIN_BYTES`` (default 0:
every size) with built-in operators; ``MP4X_SHM=0`` disables it.  A peer process that exits
is noticed by the barrier within ~0.1 s (its /proc entry is polled while waiting), so a
crashed rank fails the job fast, as a closed TCP connection does on the mesh.
"""
from __future__ import annotations

import ctypes
import os
import uuid
from multiprocessing import shared_memory

import numpy as np

from ..exceptions import TransportError
from ..ops import native
from ..ops.native import check as _native_check
from ..utils.cpus import usable_cpus

_BARRIER_ERRORS = {-1: "barrier timed out (MP4X_SHM_TIMEOUT)", -2: "barrier aborted by a peer",
                   -3: "a peer process exited (connection closed)"}


def _check(rc: int, where: str) -> None:
    if rc in _BARRIER_ERRORS:
        raise TransportError(f"{where}: shared-memory {_BARRIER_ERRORS[rc]}")
    _native_check(rc, where)


def _untrack(shm: shared_memory.SharedMemory) -> None:
    try:   # attaching processes must not unlink the segment at exit (Python 3.10 resource_tracker)
        from multiprocessing import resource_tracker
        resource_tracker.unregister(shm._name, "shared_memory")
    except Exception:
        pass


class ShmEngine:
    def __init__(self, comm, slot_bytes: int = None, threads: int = None):
        self.comm = comm
        self.rank, self.p = comm.rank, comm.slaveNum
        self.lib = native.host()
        self.slot = int(slot_bytes or int(os.environ.get("MP4X_SHM_SLOT_BYTES", 16 << 20)))
        self.slot = (self.slot + 4095) // 4096 * 4096
        size = 4096 + self.p * self.slot
        key = f"mp4x/shm/{comm.addresses[0]}"
        if self.rank == 0:
            name = f"mp4x_{os.getpid()}_{uuid.uuid4().hex[:8]}"
            self.shm = shared_memory.SharedMemory(name=name, create=True, size=size)
            self.shm.buf[:4096] = bytes(4096)
            comm.server.call("kv_set", key, name.encode())
        else:
            name = comm.server.call("kv_get", key, 120.0).decode()
            self.shm = shared_memory.SharedMemory(name=name)
            _untrack(self.shm)
        comm.server.call("barrier", self.rank)     # everyone attached
        if self.rank == 0:
            self.shm.unlink()                      # mapping stays valid; no leak on crash
        self._base = ctypes.c_char.from_buffer(self.shm.buf)
        nt = int(threads or int(os.environ.get("MP4X_HOST_THREADS", 0)) or max(1, usable_cpus() // self.p))
        timeout = float(os.environ.get("MP4X_SHM_TIMEOUT", 300.0))
        self.h = self.lib.mp4x_shm_attach(ctypes.addressof(self._base), self.rank, self.p, self.slot, nt, timeout)
        # every rank published its pid: from now on a barrier wait notices a peer process that
        # exited (fail fast, like a closed TCP connection) instead of sleeping until the timeout
        _check(self.lib.mp4x_shm_barrier(self.h), "shm attach barrier")
        self.watching = bool(self.lib.mp4x_shm_watch_peers(self.h))

    @staticmethod
    def _ptr(a: np.ndarray, off_elems: int = 0) -> int:
        return a.ctypes.data + off_elems * a.itemsize

    def allreduce(self, buf: np.ndarray, frm: int, to: int, dtype: int, op: int):
        _check(self.lib.mp4x_shm_allreduce(self.h, dtype, op, self._ptr(buf, frm), to - frm), "shm_allreduce")

    def reduce_scatter(self, buf: np.ndarray, froms, tos, dtype: int, op: int):
        f = (ctypes.c_int64 * self.p)(*froms)
        t = (ctypes.c_int64 * self.p)(*tos)
        _check(self.lib.mp4x_shm_reduce_scatter(self.h, dtype, op, self._ptr(buf), f, t), "shm_reduce_scatter")

    def allgather(self, buf: np.ndarray, froms, tos):
        f = (ctypes.c_int64 * self.p)(*froms)
        t = (ctypes.c_int64 * self.p)(*tos)
        _check(self.lib.mp4x_shm_allgather(self.h, buf.itemsize, self._ptr(buf), f, t), "shm_allgather")

    def broadcast(self, buf: np.ndarray, frm: int, to: int, root: int):
        _check(self.lib.mp4x_shm_broadcast(self.h, buf.itemsize, self._ptr(buf), frm, to, root), "shm_broadcast")

    def close(self):
        if getattr(self, "h", None):
            self.lib.mp4x_shm_detach(self.h)
            self.h = None
        try:
            del self._base
            self.shm.close()
        except Exception:
            pass


def same_host(addresses) -> bool:
    hosts = {a.rsplit("###", 1)[0] for a in addresses}
    return len(hosts) == 1
