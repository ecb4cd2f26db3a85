"""Library-owned, peer-mappable device allocations of any size (``ProcessCommSlave.memAlloc``).

The ncclMemAlloc analogue of mp4x (native side: csrc/runtime/vmm.hip).  A buffer is a run of
physical chunks (``hipMemCreate``, ``MP4X_VMM_CHUNK`` bytes each, default 512 MiB — far below
the 2 GiB size at which an IPC open of one allocation hangs on this ROCm,
profiles/r2/ipc_open_probe.jsonl) mapped back to back into one reserved VA range.  Every chunk
is exported as a POSIX fd (dmabuf); the fds travel to the same-node peers over an abstract
unix socket (``SCM_RIGHTS``, :func:`exchange_fds`) and each peer maps them back to back into
its own VA range.  The result: a contiguous tensor of any size that every peer sees as one
contiguous range too, so the zero-copy IPC kernels (csrc/runtime/ipc.hip) run on 4 GB / 8 GB
tensors with no staging — the reference's in-place 8 GB ``allreduceArray``
(/root/reference/README.md:313, ProcessCommSlave.java:1733-1763).

Only the control-plane ``allgather_obj`` is used for rendezvous (socket names, chunk counts,
errors): a failure on any rank is agreed and raised on every rank.
"""
from __future__ import annotations

import ctypes
import os
import socket
import threading
import uuid
from typing import Dict, List, Optional

import torch

from ..exceptions import Mp4jException
from ..ops import native
from ..ops.native import check, c_int, c_size_t, c_void_p

_U64P = ctypes.POINTER(ctypes.c_uint64)
_INTP = ctypes.POINTER(ctypes.c_int)

native.register_signatures({
    "mp4x_vmm_granularity": (c_int, [ctypes.POINTER(c_size_t)]),
    "mp4x_vmm_create": (c_int, [c_size_t, c_int, ctypes.POINTER(c_void_p), _U64P, _INTP]),
    "mp4x_vmm_import": (c_int, [_INTP, c_size_t, c_int, ctypes.POINTER(c_void_p), _U64P]),
    "mp4x_vmm_free": (c_int, [c_void_p, c_size_t, c_int, _U64P]),
    "mp4x_vmm_release_keep_va": (c_int, [c_void_p, c_size_t, c_int, _U64P]),
    "mp4x_vmm_va_hint": (ctypes.c_uint64, [c_int]),
    "mp4x_vmm_chunk_create": (c_int, [c_size_t, _U64P, _INTP]),
    "mp4x_vmm_chunk_import": (c_int, [c_int, _U64P]),
    "mp4x_vmm_chunk_release": (c_int, [ctypes.c_uint64]),
    "mp4x_vmm_map_chunks": (c_int, [_U64P, ctypes.POINTER(c_size_t), c_int, ctypes.POINTER(c_void_p)]),
    "mp4x_vmm_unmap_chunks": (c_int, [c_void_p, ctypes.POINTER(c_size_t), c_int]),
    "mp4x_release_all": (c_int, [c_void_p]),
})

DEFAULT_CHUNK = 512 << 20
_BIG_FRAG = 2 << 20
_FDS_PER_MSG = 200          # SCM_RIGHTS carries at most 253 fds per message (SCM_MAX_FD)


def chunk_plan(nbytes: int, gran: int, chunk: Optional[int] = None) -> (int, int):
    """(chunk bytes, chunk count) for a ``nbytes`` buffer: chunks are granularity multiples of
    at most ``chunk`` (``MP4X_VMM_CHUNK``) bytes; a small buffer is one chunk of its rounded
    size.  Pure function (unit-tested on CPU)."""
    if nbytes <= 0:
        raise Mp4jException("memAlloc needs a positive size")
    gran = max(1, int(gran))
    if nbytes >= _BIG_FRAG and _BIG_FRAG % gran == 0:
        gran = _BIG_FRAG          # 2 MiB multiples: large TLB fragments, 2 MiB aligned VA
    cap = int(chunk or os.environ.get("MP4X_VMM_CHUNK", DEFAULT_CHUNK))
    cap = max(gran, cap // gran * gran)
    need = -(-nbytes // gran) * gran
    if need <= cap:
        return need, 1
    return cap, -(-need // cap)


def chunk_sizes(nbytes: int, gran: int, cap: Optional[int] = None) -> List[int]:
    """Chunk sizes of a chunk-pool allocation of ``nbytes`` (largest first): ``cap``-byte chunks
    (``MP4X_VMM_CHUNK`` rounded down to a power-of-two number of units), then the binary
    decomposition of the rest in power-of-two multiples of the unit (2 MiB when the granularity
    divides it).  Few distinct sizes, so a freed chunk serves later allocations of OTHER sizes
    (:class:`ChunkPool`).  Pure function (unit-tested on CPU)."""
    if nbytes <= 0:
        raise Mp4jException("memAlloc needs a positive size")
    gran = max(1, int(gran))
    unit = _BIG_FRAG if _BIG_FRAG % gran == 0 else gran
    top = max(unit, int(cap or os.environ.get("MP4X_VMM_CHUNK", DEFAULT_CHUNK)) // unit * unit)
    top = unit << ((top // unit).bit_length() - 1)          # a power-of-two number of units
    need = -(-int(nbytes) // unit) * unit
    out = [top] * (need // top)
    rem = need % top
    s = top // 2
    while rem:
        if rem >= s:
            out.append(s)
            rem -= s
        s //= 2
    return out


class Chunk:
    """One physical chunk this rank owns: pool id (the same on every rank's books: alloc / free
    are collective), size, generic allocation handle, dmabuf fd while it is new (not yet sent)."""
    __slots__ = ("id", "size", "handle", "fd")

    def __init__(self, cid: int, size: int, handle: int, fd: int):
        self.id, self.size, self.handle, self.fd = cid, size, handle, fd


class ChunkPool:
    """This rank's physical memAlloc chunks: free ones per size, reused by later allocations of
    any size (csrc/runtime/vmm.hip "chunk pool" says why nothing is released before close), plus
    every peer chunk this rank imported, kept by (peer rank, chunk id) so a reused chunk is
    mapped again with no fd exchange."""

    def __init__(self, lib):
        self.lib = lib
        self.free: Dict[int, List[Chunk]] = {}
        self.owned: List[Chunk] = []
        self.peer: Dict[tuple, int] = {}
        self._next = 0

    def take(self, sizes: List[int]) -> List[Chunk]:
        out = []
        try:
            for sz in sizes:
                lst = self.free.get(sz)
                if lst:
                    out.append(lst.pop())
                    continue
                h = ctypes.c_uint64()
                fd = ctypes.c_int(-1)
                check(self.lib.mp4x_vmm_chunk_create(sz, ctypes.byref(h), ctypes.byref(fd)), "vmm_chunk_create")
                c = Chunk(self._next, sz, h.value, fd.value)
                self._next += 1
                self.owned.append(c)
                out.append(c)
        except Exception:
            self.give(out)
            raise
        return out

    def give(self, chunks: List[Chunk]) -> None:
        for c in chunks:
            self.free.setdefault(c.size, []).append(c)

    def discard(self, chunks: List[Chunk]) -> None:
        """Drop chunks for good (a failed allocation sent them and some peer may not hold
        them): released, never handed out again."""
        gone = set(map(id, chunks))
        self.owned = [c for c in self.owned if id(c) not in gone]
        for lst in self.free.values():
            lst[:] = [c for c in lst if id(c) not in gone]
        for c in chunks:
            native.soft_check(self.lib.mp4x_vmm_chunk_release(c.handle), "vmm_chunk_release")

    def import_fd(self, rank: int, cid: int, fd: int) -> int:
        h = ctypes.c_uint64()
        check(self.lib.mp4x_vmm_chunk_import(fd, ctypes.byref(h)), "vmm_chunk_import")
        self.peer[(rank, cid)] = h.value
        return h.value

    @property
    def pooled_bytes(self) -> int:
        return sum(c.size for c in self.owned)

    def release_all(self) -> None:
        """At close: every imported and owned chunk (best effort; nothing may map them any more)."""
        for h in self.peer.values():
            native.soft_check(self.lib.mp4x_vmm_chunk_release(h), "vmm_chunk_release")
        self.peer = {}
        for c in self.owned:
            if c.fd is not None and c.fd >= 0:
                try:
                    os.close(c.fd)
                except OSError:
                    pass
            native.soft_check(self.lib.mp4x_vmm_chunk_release(c.handle), "vmm_chunk_release")
        self.owned, self.free = [], {}


class MappedRange:
    """Chunks mapped back to back at a fresh VA range of this process (own or a peer's).
    :meth:`free` only unmaps: the range stays reserved (recorded in the VA quarantine), the chunks
    stay with their pool."""

    def __init__(self, lib, handles: List[int], sizes: List[int]):
        self.lib = lib
        self.sizes = list(sizes)
        self._sizes = (c_size_t * len(sizes))(*sizes)
        n = len(handles)
        va = c_void_p()
        rc = lib.mp4x_vmm_map_chunks((ctypes.c_uint64 * n)(*handles), self._sizes, n, ctypes.byref(va))
        if va.value:
            _QUARANTINE.append((va.value, sum(sizes)))
        check(rc, "vmm_map_chunks")
        self.va = va.value
        self.fds: List[int] = []

    @property
    def nbytes(self) -> int:
        return sum(self.sizes)

    def close_fds(self) -> None:
        pass

    def free(self, keep_va=None) -> None:
        """Unmap (best effort: a failed unmap only leaves address space mapped, logged)."""
        if self.va:
            native.soft_check(self.lib.mp4x_vmm_unmap_chunks(c_void_p(self.va), self._sizes, len(self.sizes)),
                              "vmm_unmap_chunks")
            self.va = 0


class VmmRegion:
    """``n`` chunks of ``chunk`` bytes mapped back to back at ``va`` in THIS process — either
    this rank's own allocation (``fds`` exported) or an imported peer allocation."""

    def __init__(self, lib, va: int, chunk: int, handles, fds: Optional[List[int]] = None):
        self.lib = lib
        self.va = va
        self.chunk = chunk
        self.n = len(handles)
        self._handles = (ctypes.c_uint64 * self.n)(*handles)
        self.fds = list(fds or [])

    @property
    def nbytes(self) -> int:
        return self.chunk * self.n

    @classmethod
    def create(cls, lib, chunk: int, n: int, export: bool = True) -> "VmmRegion":
        va = c_void_p()
        handles = (ctypes.c_uint64 * n)()
        fds = (ctypes.c_int * n)(*([-1] * n))
        check(lib.mp4x_vmm_create(chunk, n, ctypes.byref(va), handles, fds if export else None), "vmm_create")
        return cls(lib, va.value, chunk, list(handles), list(fds) if export else None)

    @classmethod
    def import_fds(cls, lib, fds: List[int], chunk: int) -> "VmmRegion":
        n = len(fds)
        va = c_void_p()
        handles = (ctypes.c_uint64 * n)()
        check(lib.mp4x_vmm_import((ctypes.c_int * n)(*fds), chunk, n, ctypes.byref(va), handles), "vmm_import")
        return cls(lib, va.value, chunk, list(handles))

    def close_fds(self) -> None:
        for fd in self.fds:
            if fd >= 0:
                try:
                    os.close(fd)
                except OSError:
                    pass
        self.fds = []

    def free(self, keep_va: Optional[List] = None) -> None:
        """Unmap + release the chunks and free the VA range — or, with ``keep_va`` (a list),
        keep the range reserved and append ``(va, bytes)`` to it: the physical memory goes back
        to the device but no later reservation of this process lands on these addresses.  Kept
        ranges stay reserved for the life of the PROCESS (:data:`_QUARANTINE`, also across
        communicators): a VA free breaks later exports on this runtime (csrc/runtime/vmm.hip)."""
        self.close_fds()
        if self.va:
            if keep_va is not None:
                check(self.lib.mp4x_vmm_release_keep_va(c_void_p(self.va), self.chunk, self.n, self._handles),
                      "vmm_release_keep_va")
                keep_va.append((self.va, self.nbytes))
            else:
                check(self.lib.mp4x_vmm_free(c_void_p(self.va), self.chunk, self.n, self._handles), "vmm_free")
            self.va = 0


class _VaQuarantine(list):
    """Process-wide record of the VA ranges this process keeps reserved instead of freeing
    (hipMemAddressFree breaks later exports on this runtime, see csrc/runtime/vmm.hip): they
    hold no physical memory, only address space.  Nothing releases them before the process
    exits.  Growth: one memAlloc / memFree cycle of B bytes at p ranks keeps about
    p * (B + B * (p - 1) / p) bytes of VA per process (the own range, p - 1 imported views, and
    the push scratch's ranges); against the 2^48-byte GPU VA space that is ~16,000 cycles of 1 GB
    tensors at p = 8 — fine for long-lived arenas (DDP buckets, ZeRO shards), not for a memAlloc
    per step.  ``quarantined_bytes()`` reports it (tests/test_vmm_chunks_cpu.py)."""


_QUARANTINE = _VaQuarantine()


def va_quarantine() -> _VaQuarantine:
    return _QUARANTINE


def quarantined_bytes() -> int:
    return sum(b for _, b in _QUARANTINE)


class _CudaArray:
    """``__cuda_array_interface__`` over a raw device range (bytes); ``torch.as_tensor`` keeps
    this object alive for the tensor's lifetime."""

    def __init__(self, ptr: int, nbytes: int, owner=None):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}
        self.owner = owner


def tensor_at(ptr: int, nbytes: int, dtype: torch.dtype, device: torch.device, owner=None) -> torch.Tensor:
    """A 1-D ``dtype`` tensor viewing ``nbytes`` of device memory at ``ptr`` (no copy)."""
    es = torch.empty((), dtype=dtype).element_size()
    if nbytes % es:
        raise Mp4jException(f"{nbytes} bytes is not a whole number of {dtype} elements")
    with torch.cuda.device(device):
        raw = torch.as_tensor(_CudaArray(ptr, nbytes, owner), device=device)
    return raw.view(dtype)


def exchange_fds(server, rank: int, p: int, mine: List[int], timeout: float = 120.0) -> Dict[int, List[int]]:
    """Collective: every rank gets every peer's fd list (``SCM_RIGHTS`` duplicates, owned by the
    caller) over abstract unix sockets; only the socket names go through the control plane.

    Every rank serves its fds to each connecting peer from a thread while it connects to every
    peer itself, so no ordering between ranks can deadlock.  Same node only (abstract socket
    namespace of one network namespace)."""
    name = f"\0mp4x-fd-{uuid.uuid4().hex}"
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    err = None
    try:
        srv.bind(name)
        srv.listen(max(1, p))
        srv.settimeout(timeout)
    except OSError as e:
        err = f"{type(e).__name__}: {e}"
    names = server.call("allgather_obj", rank, (name, len(mine), err))
    bad = [(i, e) for i, (_, _, e) in enumerate(names) if e]
    if bad:
        srv.close()
        raise Mp4jException(f"fd exchange socket setup failed on ranks {bad}")
    serve_err: List[str] = []

    def serve():
        try:
            for _ in range(p - 1):
                conn, _ = srv.accept()
                with conn:
                    conn.settimeout(timeout)
                    conn.recv(4)                      # the peer's hello
                    for i in range(0, max(1, len(mine)), _FDS_PER_MSG):
                        part = mine[i:i + _FDS_PER_MSG]
                        socket.send_fds(conn, [len(part).to_bytes(4, "little")], part)
                    conn.recv(1)                      # the peer holds the fds: done
        except Exception as e:   # noqa: BLE001
            serve_err.append(f"{type(e).__name__}: {e}")

    th = threading.Thread(target=serve, daemon=True, name="mp4x-fd-serve")
    th.start()
    got: Dict[int, List[int]] = {}
    local_err = None
    try:
        for j in range(p):
            if j == rank:
                continue
            c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            c.settimeout(timeout)
            with c:
                c.connect(names[j][0])
                c.sendall(rank.to_bytes(4, "little"))
                fds: List[int] = []
                want = names[j][1]
                for _ in range(max(1, -(-want // _FDS_PER_MSG))):   # the messages serve() sends
                    msg, part, _, _ = socket.recv_fds(c, 4, _FDS_PER_MSG)
                    if not msg:
                        raise Mp4jException(f"fd exchange: rank {j} closed early")
                    fds += part
                if len(fds) != want:
                    raise Mp4jException(f"fd exchange: {len(fds)} fds from rank {j}, expected {want}")
                c.sendall(b"k")
                got[j] = fds
    except Exception as e:   # noqa: BLE001
        local_err = f"{type(e).__name__}: {e}"
    th.join(timeout)
    srv.close()
    if serve_err and local_err is None:
        local_err = serve_err[0]
    errs = server.call("allgather_obj", rank, local_err)
    failed = [(i, e) for i, e in enumerate(errs) if e]
    if failed:
        for fl in got.values():
            for fd in fl:
                os.close(fd)
        raise Mp4jException(f"fd exchange failed on ranks {failed}")
    return got
