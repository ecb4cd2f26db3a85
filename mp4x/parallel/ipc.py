"""Host side of the custom xGMI allreduce (csrc/runtime/ipc.hip).

Each rank allocates one fine-grained uncached data buffer (``MP4X_IPC_BYTES``, default
64 MiB) plus a signal block, exports both with ``hipIpcGetMemHandle``, exchanges the handles
through the master (``allgather_obj``) and maps every peer's pair with
``hipIpcOpenMemHandle``.  A call copies the input into the own data buffer (stream ordered)
and launches ONE kernel that synchronises with the peers' kernels through epoch flags and
reduces straight out of peer HBM.  Messages larger than the buffer are processed in
half-buffer pieces whose input copies (side stream) overlap the previous piece's kernel.

Only needs the mp4x control plane (no RCCL communicator), so it also runs with several
processes sharing one GPU — which is how it is tested on a single-GPU box.
"""
from __future__ import annotations

import contextlib
import ctypes
import logging
import os
from typing import List, Optional

import torch

from ..exceptions import Mp4jException
from ..operators import DType, OpCode, dtype_of_torch
from ..ops import native
from ..ops.native import check, capturing_now, ptr_array, stream_ptr, c_int, c_int64, c_void_p, c_size_t, PP
from . import occupancy

native.register_signatures({
    "mp4x_ipc_signal_bytes": (c_size_t, []),
    "mp4x_ipc_alloc": (c_int, [c_size_t, ctypes.POINTER(c_void_p)]),
    "mp4x_ipc_alloc_data": (c_int, [c_size_t, c_int, ctypes.POINTER(c_void_p)]),
    "mp4x_ipc_free": (c_int, [c_void_p]),
    "mp4x_host_word_alloc": (c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p)]),
    "mp4x_host_word_free": (c_int, [c_void_p]),
    "mp4x_ipc_set_host_error": (c_int, [c_void_p, c_void_p]),
    "mp4x_ipc_set_spin": (c_int, [c_void_p, ctypes.c_double, c_void_p]),
    "mp4x_ipc_op_supported": (c_int, [c_int, c_int]),
    "mp4x_ipc_occupancy_ar": (c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)]),
    "mp4x_ipc_occupancy_push": (c_int, [c_int, c_int, c_int, ctypes.POINTER(c_int)]),
    "mp4x_ipc_occupancy_rs": (c_int, [c_int, c_int, c_int, ctypes.POINTER(c_int)]),
    "mp4x_ipc_occupancy_misc": (c_int, [c_int, c_int, c_int, ctypes.POINTER(c_int)]),
    "mp4x_mem_range": (c_int, [c_void_p, ctypes.POINTER(c_void_p), ctypes.POINTER(c_size_t)]),
    "mp4x_dev_alloc": (c_int, [c_size_t, ctypes.POINTER(c_void_p)]),
    "mp4x_ipc_allreduce_push": (c_int, [c_int, c_int, PP, PP, PP, c_int, c_int, c_int64, ctypes.c_uint32, c_int,
                                        c_void_p, ctypes.c_float, c_void_p]),
    "mp4x_ipc_handle_size": (c_int, []),
    "mp4x_ipc_get_handle": (c_int, [c_void_p, c_void_p]),
    "mp4x_ipc_open_handle": (c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    "mp4x_ipc_close_handle": (c_int, [c_void_p]),
    "mp4x_ipc_read_error": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_uint32)]),
    "mp4x_ipc_error_word": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_uint32), c_int, c_void_p]),
    "mp4x_ipc_fp8_allreduce": (c_int, [c_int, PP, PP, c_int, c_int, c_int64, c_int64, c_void_p, c_int64,
                                       ctypes.c_uint32, c_int, c_void_p, ctypes.c_float, c_void_p]),
    "mp4x_memset_async": (c_int, [c_void_p, c_int, c_size_t, c_void_p]),
    "mp4x_memcpy_async": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "mp4x_ipc_allreduce": (c_int, [c_int, c_int, c_int, PP, PP, c_int, c_int, c_int64, c_void_p, ctypes.c_uint32,
                                   c_int, c_void_p, c_void_p]),
    "mp4x_ipc_allreduce_ex": (c_int, [c_int, c_int, c_int, PP, PP, c_int, c_int, c_int64, c_void_p, c_void_p,
                                      ctypes.c_uint32, c_int, c_void_p, ctypes.c_float, c_void_p]),
    "mp4x_ipc_allreduce_ex2": (c_int, [c_int, c_int, c_int, PP, PP, c_int, c_int, c_int64, c_void_p, c_void_p,
                                       ctypes.c_uint32, c_int, c_void_p, ctypes.c_float, c_void_p, c_int64, c_int64]),
    "mp4x_ipc_reduce_scatter_from": (c_int, [c_int, c_int, PP, PP, c_int, c_int, ctypes.POINTER(c_int64),
                                             ctypes.POINTER(c_int64), c_void_p, c_void_p, ctypes.c_uint32, c_int,
                                             c_void_p, c_void_p]),
    "mp4x_ipc_bump_epoch": (c_int, [c_void_p, c_void_p]),
    "mp4x_ipc_copy_plan_check": (c_int, [c_int, c_int, ctypes.POINTER(c_int64), c_int, ctypes.POINTER(c_int64), c_int,
                                         c_void_p, c_void_p, c_int64]),
    "mp4x_ipc_copy_plan": (c_int, [PP, PP, c_int, c_int, ctypes.POINTER(c_int64), c_int, ctypes.POINTER(c_int64), c_int,
                                   c_void_p, c_void_p, c_int64, c_int64, ctypes.c_uint32, c_int, c_void_p, c_void_p]),
    "mp4x_device_pci_id": (c_int, [ctypes.c_char_p, c_int]),
    "mp4x_ipc_reduce_scatter": (c_int, [c_int, c_int, PP, PP, c_int, c_int, c_int64, c_int64, c_void_p,
                                        ctypes.c_uint32, c_int, c_void_p, c_void_p]),
    "mp4x_ipc_allgather": (c_int, [PP, PP, c_int, c_int, ctypes.POINTER(c_int64), ctypes.POINTER(c_int64),
                                   c_void_p, ctypes.c_uint32, c_int, c_void_p, c_void_p]),
})

LOG = logging.getLogger("mp4x.ipc")

ONESHOT, TWOSHOT = 0, 1
from .ipc_forms import PUSH_TAG, ZC_TAG, IpcForms  # noqa: E402,F401 (re-exported)
PUSH_ON = os.environ.get("MP4X_IPC_PUSH", "1") == "1"
# staging buffers: fine-grained uncached (default) or coarse-grained (MP4X_IPC_DATA_MEM=coarse, A/B)
DATA_COARSE = os.environ.get("MP4X_IPC_DATA_MEM", "uncached").lower() == "coarse"
# hipIpcOpenMemHandle of an allocation of 2^31 bytes or more never returns on this ROCm
# (measured: 2.0 GB opens in 0.1 ms, 2 GiB hangs — profiles/r2/ipc_open_probe.jsonl), so
# registration refuses such allocations (every rank alike): the staged kernels run instead.
IPC_OPEN_MAX = int(os.environ.get("MP4X_IPC_OPEN_MAX", (1 << 31) - 1))
# Memory lifetime (diagnosed with tools/repro/ipc_lifetime_repro.hip):
# CLOSE_PEERS — a deregistration closes this rank's mappings of the peers' allocations (refcounted
#   per allocation) and frees its push scratch, instead of caching every mapping and pooling every
#   scratch until close();
# VMM_POLICY — how memAlloc / memFree manage memory (tests/test_vmm_policy_gpu.py measures every
#   one for exactness and device-memory growth; tools/repro/ipc_lifetime_repro.hip shows, in plain
#   HIP, why only the first and "fresh_va" / "pool" are exact on this runtime):
#   "chunks":         (default) physical chunks of power-of-two sizes from a per-rank pool
#                     (vmm.ChunkPool) mapped at a fresh VA range per allocation; memFree unmaps
#                     and returns the chunks to the pool (reused by allocations of any size, no
#                     fd exchange for a reused chunk); nothing released or VA-freed before close;
#   "fresh_va":       release the physical chunks collectively (every importer's mapping first, the
#                     owners' memory after a barrier) but keep every VA range reserved, so no later
#                     mapping of this process lands on recycled addresses (vmm.va_quarantine);
#   "ordered":        the same release, VA ranges freed too;
#   "hint":           "ordered", and every new reservation asks for an address above every range
#                     reserved before (csrc/runtime/vmm.hip reserve());
#   "keep_owner_va" / "keep_import_va": only the owner's / only the importers' ranges kept;
#   "pool":           park the allocation in a per-size pool that the next memAlloc of that size
#                     reuses (round 3's behaviour; MP4X_VMM_RELEASE=0 still selects it).
CLOSE_PEERS = os.environ.get("MP4X_IPC_CLOSE_PEERS", "1") == "1"
# Release ORDER of everything a peer maps (registered tensors at deregistration, self-test buffers,
# the staging buffers of an instance closed mid-job): every importer closes its mappings (and
# flushes, _flush_translations), a control-plane barrier, and only then does each owner free its
# memory — the order mem_free always used.  (Round 4's corruption turned out to need a RELEASE of a
# peer-mapped push scratch, whatever the order: push scratches are pooled now, see _alloc_scratch
# and profiles/r5/rootcause/.)  MP4X_TEST_UNORDERED_RELEASE=1 restores round 4's order (owner frees
# first, no barrier) for the release-order tests; never for a job.
UNORDERED_RELEASE = os.environ.get("MP4X_TEST_UNORDERED_RELEASE", "0") == "1"
# MP4X_TEST_FREE_SCRATCH=1: round 4's push-scratch handling (freed at deregistration, the peers'
# mappings of it closed) instead of the pool — the trigger of round 4's corruption; diagnosis only
# (tools/gpu/r4repro.sh, profiles/r5/rootcause/).
FREE_SCRATCH = os.environ.get("MP4X_TEST_FREE_SCRATCH", "0") == "1"
VMM_POLICIES = ("chunks", "fresh_va", "ordered", "hint", "keep_owner_va", "keep_import_va", "pool")
VMM_POLICY = os.environ.get("MP4X_VMM_POLICY") or (
    "pool" if os.environ.get("MP4X_VMM_RELEASE") == "0" else "chunks")
if VMM_POLICY not in VMM_POLICIES:
    raise ValueError(f"MP4X_VMM_POLICY={VMM_POLICY!r}: expected one of {VMM_POLICIES}")
VMM_RELEASE = VMM_POLICY != "pool"
SUPPORTED_DTYPES = {torch.float32, torch.float64, torch.bfloat16, torch.float16, torch.int32, torch.int64,
                    torch.int16, torch.int8, torch.uint8}
_FLOAT_DTYPES = (torch.float32, torch.float64, torch.bfloat16, torch.float16)

_FP8_NARROW = os.environ.get("MP4X_FP8_NARROW") == "1"    # the r1 4-byte-lane fp8 kernel (A/B)


def ipc_mode_report(err: Optional[str] = None) -> dict:
    """Which IPC mode the HIP runtime of this process most likely uses, and — for a failed handle
    export or open (``err``) — the reason and the fix.  The dmabuf mode needs
    ``HSA_ENABLE_IPC_MODE_LEGACY=0`` in the environment when the HSA runtime starts; ``import mp4x``
    sets it (unless set), which is too late when HIP was initialised before (mp4x/__init__.py)."""
    import mp4x
    at = dict(getattr(mp4x, "IPC_MODE_AT_IMPORT", {}) or {})
    env = at.get("env_before_import")
    legacy = env not in (None, "0") or (env is None and at.get("hip_initialized_before_import"))
    rep = {"legacy_env_before_import": env, "hip_initialized_before_import": at.get("hip_initialized_before_import"),
           "dmabuf_expected": not legacy}
    if err is not None:
        handle = any(k in err for k in ("ipc_get_handle", "ipc_open_handle", "hipIpc", "invalid argument"))
        if legacy:
            cause = (f"HSA_ENABLE_IPC_MODE_LEGACY={env}" if env not in (None, "0") else
                     "HIP was initialised before `import mp4x` with HSA_ENABLE_IPC_MODE_LEGACY unset")
            rep["reason"] = (f"IPC handle export/import failed in the legacy IPC mode ({cause}); this platform "
                             f"needs dmabuf IPC: start the process with HSA_ENABLE_IPC_MODE_LEGACY=0 (or import mp4x "
                             f"before anything touches the GPU)")
        elif handle:
            rep["reason"] = "IPC handle export/import failed although the dmabuf mode was requested: " + err[:200]
        else:
            rep["reason"] = err[:200]
    return rep


def staging_needs_vmm(alloc_bytes: int) -> bool:
    """Is a staging allocation of ``alloc_bytes`` (buffer + slots) above the IPC open limit, so it
    must be built from VMM chunks exported as dmabuf fds instead of one hipIpc allocation?"""
    return int(alloc_bytes) > IPC_OPEN_MAX


def next_epoch(e: int) -> int:
    """The host epoch after ``e`` (low 30 bits, never 0, wrapping to 2 so consecutive epochs always
    alternate parity): csrc/runtime/ipc_common.hpp ``next_epoch`` — the one-shot's double-buffered
    slots are chosen by the parity."""
    return ((e + 1) & 0x3FFFFFFF) or 2


# Two double-buffered slots (csrc/runtime/ipc_ar.hip k_ipc_oneshot / k_ipc_twoshot), appended to
# every instance's staging buffer: a staged, fused, one-piece one-shot then has ONE cross-rank
# barrier per call and a two-shot two (no end barrier).  MP4X_IPC_SLOTS=0 turns them off (A/B);
# MP4X_IPC_SLOT_BYTES sizes them (4 MiB: the staged two-shot's range below the zero-copy sizes,
# where a barrier round trip is a visible share of the call; at least the one-shot tier).
SLOTS_ON = os.environ.get("MP4X_IPC_SLOTS", "1") == "1"
SLOT_BYTES = int(os.environ.get("MP4X_IPC_SLOT_BYTES", 4 << 20))


def ipc_op_ok(dtype, op) -> bool:
    """Does the IPC tier reduce ``op`` over ``dtype``?  Every operator of the reference's table
    (Operators.java:29-353) for every primitive dtype, plus 16-bit floats and uint8: SUM / MAX /
    MIN / PROD everywhere, BITS_AND / OR / XOR on integers, FLOAT_*_LOC on the packed f64 words,
    INT_*_LOC on the packed i64 words (csrc/runtime/ipc_common.hpp rt_op_ok).  Custom operators
    (possibly non-commutative host callables) never run here."""
    if getattr(op, "is_custom", False) or dtype not in SUPPORTED_DTYPES:
        return False
    c = op.code
    if c in (OpCode.SUM, OpCode.MAX, OpCode.MIN, OpCode.PROD):
        return True
    if c in (OpCode.BAND, OpCode.BOR, OpCode.BXOR):
        return dtype not in _FLOAT_DTYPES
    if c in (OpCode.FMAXLOC, OpCode.FMINLOC):
        return dtype == torch.float64
    if c in (OpCode.IMAXLOC, OpCode.IMINLOC):
        return dtype == torch.int64
    return False


def spin_default() -> float:
    """Barrier spin bound (seconds) of the IPC kernels in normal operation: ``MP4X_IPC_SPIN_S``,
    else the collective watchdog's fail-stop budget ``MP4X_WATCHDOG_TIMEOUT`` (600 s, the
    reference's heartbeat gap, Server.java:82-83).  A collective waits for a straggling peer as
    long as the job's failure detector would, like the reference's ring step that blocks on
    ``recvResultQueue.take()`` (ProcessCommSlave.java:1355); only the mesh self-test and the
    autotune probes use a short bound (:meth:`IpcAllreduce.spin_bound`)."""
    v = os.environ.get("MP4X_IPC_SPIN_S")
    if v:
        return float(v)
    return float(os.environ.get("MP4X_WATCHDOG_TIMEOUT", 600.0))


def probe_spin() -> float:
    """Spin bound of the autotune probes (``MP4X_IPC_PROBE_SPIN_S``, 10 s): a candidate whose
    barrier cannot complete on this topology is ruled out in seconds, not after the watchdog."""
    return float(os.environ.get("MP4X_IPC_PROBE_SPIN_S", 10.0))


def _agree(comm, rank, obj, is_bad):
    """``allgather_obj`` of ``obj`` over the mesh's ranks and whether ``is_bad`` holds for ANY rank
    of the JOB.  A sub-mesh (parallel/hier.py) answers for the whole job, so a failure on one node
    makes every node raise at the same agreement point and their control-plane calls stay paired
    (a node raising alone would pair its next global call with the others' setup)."""
    both = getattr(comm.server, "allgather_both", None)
    if both is not None:
        mine, every = both(rank, obj)
        return mine, any(is_bad(x) for x in every)
    allv = comm.server.call("allgather_obj", rank, obj)
    return allv, any(is_bad(x) for x in allv)


class FastAr(ctypes.Structure):
    """ctypes layout of the latency fast paths' per-instance state (csrc/runtime/ipc_ar.hip
    ``FastAr``)."""
    _fields_ = [("herr", c_void_p * 8), ("epoch", c_void_p), ("data_ptrs", c_void_p),
                ("signal_ptrs", c_void_p), ("rank", ctypes.c_int32), ("p", ctypes.c_int32),
                ("slot_base", ctypes.c_int64), ("slot_vecs", ctypes.c_int64), ("order", c_void_p),
                ("own_err", c_void_p)]


class _Reg:
    """One registered tensor on this rank: every rank's pointer to it (``peers``, own included),
    every rank's push scratch (or None), and what this rank must release at deregistration."""
    __slots__ = ("peers", "scratch", "keep", "scratch_alloc", "vmm", "nown", "peer_keys", "chunks", "scr_keys")

    def __init__(self, keep=None):
        self.peers: List[int] = []
        self.scratch = None
        self.keep = keep                 # the registered tensor: its memory stays allocated
        self.scratch_alloc = None        # own push scratch: (allocation, IPC handle bytes)
        self.vmm: list = []              # memAlloc: own regions first (nown of them), then imported
        self.nown = 0
        self.peer_keys: list = []        # (rank, handle bytes) of every peer mapping this one uses
        self.chunks = None               # memAlloc under the chunk pool: this rank's chunks
        self.scr_keys: list = []         # the peer_keys that are push scratches


class IpcAllreduce(IpcForms):
    def __init__(self, comm, nbytes: Optional[int] = None, tag: str = "default", slots: bool = True):
        self.comm = comm
        self.rank = comm.rank
        self.p = comm.slaveNum
        if not (2 <= self.p <= 8):
            raise Mp4jException("IPC allreduce supports 2..8 ranks")
        self.lib = None
        self.spin_s = None
        self.cus = None                  # CUs of this GPU (grid caps), read lazily
        self._data = c_void_p()
        self._sig = c_void_p()
        self._herr = c_void_p()          # pinned host error word (CPU address)
        self._herr_word = None           # its ctypes view, made once (read on every call)
        self._opened: List[c_void_p] = []
        # Every local step that can fail runs before the first collective inside a try, and its
        # error travels in that collective: a rank that fails alone must not leave its peers
        # waiting in an allgather it never joins (every rank raises together instead).
        local_err = None
        try:
            self.lib = native.hip()
            if VMM_POLICY == "hint":
                self.lib.mp4x_vmm_va_hint(1)
            self.device = torch.cuda.current_device()
            hs = self.lib.mp4x_ipc_handle_size()
        except Exception as e:   # noqa: BLE001
            local_err = f"{type(e).__name__}: {e}"
        # IPC handles only open on the same node: a job spanning hosts keeps RCCL (decided from
        # the exchanged host names, identically on every rank, before anything is allocated)
        from .hier import node_id
        nid = comm.node_id() if hasattr(comm, "node_id") else node_id(self.rank)
        infos, bad = _agree(comm, self.rank, (nid, local_err), lambda x: bool(x[1]))
        errs = [(i, e) for i, (_, e) in enumerate(infos) if e]
        if bad:
            raise Mp4jException(f"IPC setup failed on ranks {errs or 'of another node'}")
        hosts = [h for h, _ in infos]
        if len(set(hosts)) != 1:
            raise Mp4jException(f"IPC allreduce needs all ranks on one node (hosts: {sorted(set(hosts))})")
        self.nbytes = int(nbytes or int(os.environ.get("MP4X_IPC_BYTES", 64 << 20)))
        self.nbytes = (self.nbytes + 4095) // 4096 * 4096
        # the two slots live above self.nbytes (nothing else stages there); only the instance that
        # serves the latency tier has them (``slots``: the large-message, fp8 and hier instances
        # never run a slotted call)
        slot = max(SLOT_BYTES, int(os.environ.get("MP4X_IPC_ONESHOT_MAX", 256 << 10))) if SLOTS_ON and slots else 0
        self._slot_bytes = (slot + 4095) // 4096 * 4096
        self._slot_base = self.nbytes // 16          # in 16-byte vectors
        self._slot_vecs = self._slot_bytes // 16
        alloc_bytes = self.nbytes + 2 * self._slot_bytes
        # a staging buffer above the IPC open limit is built like a memAlloc tensor (VMM chunks,
        # dmabuf fds to the peers): rank-independent (the size is the same on every rank).  The
        # limit applies to the whole ALLOCATION, slots included (nbytes just below
        # 2 GiB plus the slots would reach the size hipIpcOpenMemHandle never returns from)
        self._vmm_data = staging_needs_vmm(alloc_bytes)
        self._data_regions: list = []     # VMM data buffer: own region + imported peer regions
        # a local failure here (out of memory, no IPC support) must still reach the allgather
        # below: raising before it would leave the peers waiting there for this rank
        local_err = None
        try:
            if self._vmm_data:
                from . import vmm
                g = ctypes.c_size_t()
                check(self.lib.mp4x_vmm_granularity(ctypes.byref(g)), "vmm_granularity")
                chunk, nch = vmm.chunk_plan(alloc_bytes, g.value)
                own = vmm.VmmRegion.create(self.lib, chunk, nch)
                self._data_regions.append(own)
                self._data = c_void_p(own.va)
                check(self.lib.mp4x_memset_async(own.va, 0, alloc_bytes, None), "vmm data zero")
                torch.cuda.synchronize()
            else:
                check(self.lib.mp4x_ipc_alloc_data(alloc_bytes, int(DATA_COARSE), ctypes.byref(self._data)),
                      "ipc_alloc(data)")
            check(self.lib.mp4x_ipc_alloc(self.lib.mp4x_ipc_signal_bytes(), ctypes.byref(self._sig)),
                  "ipc_alloc(sig)")
            herr_dev = c_void_p()
            check(self.lib.mp4x_host_word_alloc(ctypes.byref(self._herr), ctypes.byref(herr_dev)), "host_word_alloc")
            check(self.lib.mp4x_ipc_set_host_error(self._sig, herr_dev), "ipc_set_host_error")
            self.set_spin(spin_default(), on_current_stream=False)     # nothing queued yet
            hd = ctypes.create_string_buffer(hs)
            hsg = ctypes.create_string_buffer(hs)
            if not self._vmm_data:
                check(self.lib.mp4x_ipc_get_handle(self._data, hd), "ipc_get_handle(data)")
            check(self.lib.mp4x_ipc_get_handle(self._sig, hsg), "ipc_get_handle(sig)")
            pci = ctypes.create_string_buffer(64)
            check(self.lib.mp4x_device_pci_id(pci, 64), "device_pci_id")
            blob = hd.raw + hsg.raw + pci.value
        except Exception as e:
            local_err = str(e)
            blob = b"ERR:" + local_err.encode()
        allh, bad = _agree(comm, self.rank, blob, lambda b: bytes(b).startswith(b"ERR:"))
        failed = [(i, bytes(b)[4:].decode(errors="replace")) for i, b in enumerate(allh)
                  if bytes(b).startswith(b"ERR:")]
        if bad:
            self.close(sync=False)
            raise Mp4jException(f"IPC buffer setup failed on ranks {failed or 'of another node'}")
        ids = [bytes(b[2 * hs:]) for b in allh]
        share = max(max(ids.count(i) for i in ids), int(getattr(comm, "gpu_share", 1)))
        # ranks on one device (rehearsal): every launch's grid is capped so all ranks' blocks fit
        # at once, per kernel instantiation from its occupancy (grid_cap, parallel/occupancy.py)
        self.share = share
        self.shared_gpu = share > 1
        self.grid_caps = {}
        self._cap_fast = {}          # (family, torch dtype, operator) -> cap: the per-call lookup
        self.data_ptrs: List[int] = []
        self.sig_ptrs: List[int] = []
        err = None
        got = {}
        if self._vmm_data:
            from . import vmm
            try:
                got = vmm.exchange_fds(comm.server, self.rank, self.p, self._data_regions[0].fds)   # collective
            except Exception:
                self.close(sync=False)
                raise
            self._data_regions[0].close_fds()
        try:
            for r, blob in enumerate(allh):
                if r == self.rank:
                    self.data_ptrs.append(self._data.value)
                    self.sig_ptrs.append(self._sig.value)
                    continue
                for i, lst in ((0, self.data_ptrs), (1, self.sig_ptrs)):
                    if i == 0 and self._vmm_data:
                        own = self._data_regions[0]
                        pr = vmm.VmmRegion.import_fds(self.lib, got[r], own.chunk)
                        self._data_regions.append(pr)
                        lst.append(pr.va)
                        continue
                    h = ctypes.create_string_buffer(bytes(blob[i * hs:(i + 1) * hs]), hs)   # pci id follows
                    ptr = c_void_p()
                    check(self.lib.mp4x_ipc_open_handle(h, ctypes.byref(ptr)), f"ipc_open_handle(rank {r})")
                    self._opened.append(ptr)
                    lst.append(ptr.value)
        except Exception as e:   # decide collectively: every rank enables IPC or none does
            err = str(e)
        finally:
            for fl in got.values():             # every received fd, also after a failure midway
                for fd in fl:
                    os.close(fd)
        oks, anybad = _agree(comm, self.rank, b"" if err is None else err.encode(), bool)
        if anybad:
            # agreed on every rank (job-wide for a sub-mesh): some peers may have mapped this
            # rank's buffers already, so the teardown is ordered like any other
            self.close(sync=False, collective=True)
            bad = [(i, bytes(o).decode()) for i, o in enumerate(oks) if o]
            raise Mp4jException(f"IPC peer mapping failed on ranks {bad or 'of another node'}")
        self._pp_data = ptr_array(self.data_ptrs)
        self._pp_sig = ptr_array(self.sig_ptrs)
        # integer addresses of the two pointer arrays, for the ctypes-free launcher
        self._pp_data_addr = ctypes.addressof(self._pp_data[1])
        self._pp_sig_addr = ctypes.addressof(self._pp_sig[1])
        self._epoch_box = (ctypes.c_uint32 * 1)()     # host epoch (also bumped by the native fast path)
        self._fast_state = None    # native latency fast path state (fast_state())
        self.on_change = None      # callback of the owning engine: registrations / epoch mode changed
        self._pp_hi = None         # peer pointers of the upper half-buffers (pipelined large path)
        self._copy_stream = None
        self._epoch_dev = None     # device epoch counter for graph-captured calls (lazy)
        self._sig_stream = None    # private stream for error-word reads (lazy)
        self._overlap_default = os.environ.get("MP4X_IPC_OVERLAP", "0") == "1"
        self._fuse_copy = os.environ.get("MP4X_IPC_FUSED_COPY", "1") == "1"
        # registered caller tensors (zero-copy two-shot): (data_ptr, nbytes) -> (peer pointers,
        # every rank's push scratch or None)
        self._regs = {}
        self._peer_bases = {}       # (rank, handle bytes) -> mapped address
        self._peer_refs = {}        # (rank, handle bytes) -> registrations using the mapping
        self._scratch_pool = {}     # push-scratch bytes -> [(allocation, handle)] free for reuse
        self._scratch_size = {}     # push-scratch address -> bytes
        self._vmm_pool = {}         # memAlloc size -> [freed registrations] (see mem_free)
        self._chunk_pool = None     # memAlloc chunk pool (VMM_POLICY "chunks", vmm.ChunkPool)
        # all ranks mapped before anyone launches
        comm.server.call("barrier", self.rank)

    # ---------------------------------------------------------------- host epoch
    @property
    def epoch(self) -> int:
        """The host-side epoch of the staged / zero-copy protocols (low 30 bits; graph mode uses
        the device counter instead).  Kept in a native word (``_epoch_box``) that the latency fast
        path (``mp4x_ipc_fast_allreduce``) bumps too, so both paths draw from ONE sequence."""
        box = self.__dict__.get("_epoch_box")
        return int(box[0]) if box is not None else 0

    @epoch.setter
    def epoch(self, v: int) -> None:
        box = self.__dict__.get("_epoch_box")
        if box is None:
            box = self.__dict__["_epoch_box"] = (ctypes.c_uint32 * 1)()
        box[0] = int(v)

    def _changed(self) -> None:
        cb = self.__dict__.get("on_change")
        if cb is not None:
            cb()

    def fast_state(self, herr_words) -> Optional[int]:
        """Address of the native latency fast path's state for this instance (csrc/runtime/ipc_ar.hip
        ``FastAr``): ``herr_words`` = the pinned host error words of every IPC instance of the
        engine (the fail-stop check of every call).  Rebuilt when the list changes."""
        if self._epoch_dev is not None or not self._herr:
            return None
        words = tuple(int(w) for w in herr_words if w)[:8]
        st = self._fast_state
        if st is None or st[1] != words:
            s = FastAr()
            for i, w in enumerate(words):
                s.herr[i] = w
            s.epoch = ctypes.addressof(self._epoch_box)
            s.data_ptrs = self._pp_data_addr
            s.signal_ptrs = self._pp_sig_addr
            s.rank, s.p = self.rank, self.p
            s.slot_base, s.slot_vecs = self._slot_base, self._slot_vecs
            s.order = self.order().addr
            s.own_err = self._herr.value
            st = self._fast_state = (s, words)
        return ctypes.addressof(st[0])

    def latency_blocks(self, total: int, algo: int, dtype, op) -> int:
        """Grid of a staged one-/two-shot of ``total`` bytes (0 = the kernel's own default): on a
        GPU shared by the ranks, the co-residency cap of that kernel (:meth:`grid_cap`)."""
        if not self.shared_gpu:
            return 0
        vec_per_block = 512          # kIpcThreads 16-byte vectors per block and grid step
        cap = self.grid_cap("oneshot" if algo == ONESHOT else "twoshot", dtype, op)
        return max(1, min(cap, -(-min(total, self.nbytes) // 16 // vec_per_block)))

    # ---------------------------------------------------------------- fail-stop
    def host_error(self) -> int:
        """The host-visible barrier-timeout word (0 = fine; 1/2/3 = a start/mid/end barrier of an
        earlier kernel timed out), read from pinned memory: no device synchronisation."""
        w = self._herr_word
        if w is None:
            if not self._herr:
                return 0
            w = self._herr_word = ctypes.c_uint32.from_address(self._herr.value)
        return w.value

    def raise_if_failed(self) -> None:
        """Fail the call instead of corrupting it: if an earlier IPC kernel of this instance gave
        up waiting for a peer (a rank skipped or died in a collective), its result was left
        incomplete — raise ``Mp4jException`` once (the word is cleared) before launching more.
        Called at the start of every IPC collective (reference fail-stop contract,
        ProcessCommSlave.java:360-373)."""
        if self.__dict__.get("_closed"):
            raise Mp4jException(f"rank {self.rank}: IPC instance used after close()")
        code = self.host_error()
        if code:
            ctypes.c_uint32.from_address(self._herr.value).value = 0
            if code == 5:
                raise Mp4jException(f"rank {self.rank}: an earlier IPC collective failed to launch after its epoch "
                                    f"moved (a HIP launch error); its peers' kernels of that call time out, and "
                                    f"the result of that call is invalid")
            if code == 4:
                raise Mp4jException(f"rank {self.rank}: IPC protocol mismatch — a peer ran the staged form of a "
                                    f"collective while this rank ran the zero-copy form (or the reverse): buffer "
                                    f"registrations differ across ranks (e.g. a rank-local deregister); the result "
                                    f"of that call is invalid")
            where = {1: "start", 2: "mid", 3: "end"}.get(code, str(code))
            raise Mp4jException(f"rank {self.rank}: an earlier IPC collective timed out at its {where} barrier "
                                f"(a peer skipped, failed or died in that call); its result is invalid")

    def set_spin(self, seconds: float, on_current_stream: bool = True) -> None:
        """Barrier spin bound of this instance's kernels (stream-ordered on the current stream:
        kernels queued before keep the previous bound)."""
        st = stream_ptr() if on_current_stream else None
        check(self.lib.mp4x_ipc_set_spin(self._sig, float(seconds), st), "ipc_set_spin")
        self.spin_s = float(seconds)

    @contextlib.contextmanager
    def spin_bound(self, seconds: float):
        """A short spin bound while the block runs (self-test, autotune probes), then the previous one."""
        old = self.spin_s if self.spin_s is not None else spin_default()
        self.set_spin(seconds)
        try:
            yield self
        finally:
            self.set_spin(old)

    # ---------------------------------------------------------------- co-residency grid caps
    _OCC_FAMILY = {"gather": 0, "plan": 1, "fp8": 2, "fp8n": 3}

    def grid_cap(self, family: str, dtype=None, op=None) -> int:
        """Largest grid a launch of ``family`` ((dtype, op) kernel; see parallel/occupancy.py)
        may use: 256 with a GPU of its own; on a GPU shared by ``share`` ranks, the budget derived
        from the kernel instantiation's occupancy (API and compiler resources, the smaller) so
        every rank's blocks are resident at once.  Rank-independent (every rank of a shared GPU
        computes the same value), memoised and logged once per kernel."""
        if not self.shared_gpu:
            return occupancy.MAX_BLOCKS
        fast = self._cap_fast.get((family, dtype, op))
        if fast is not None:                       # the per-call path: one dict probe
            return fast
        code = int(op.code) if op is not None else 0
        key = (family, dtype, code)
        cap = self.grid_caps.get(key)
        if cap is not None:
            self._cap_fast[(family, dtype, op)] = cap
            return cap
        dt = int(dtype_of_torch(dtype)) if dtype is not None else int(DType.F32)
        n = ctypes.c_int(0)
        try:
            if family in ("oneshot", "twoshot"):
                rc = self.lib.mp4x_ipc_occupancy_ar(0 if family == "oneshot" else 1, dt, code, self.p, ctypes.byref(n))
            elif family == "push":
                rc = self.lib.mp4x_ipc_occupancy_push(dt, code, self.p, ctypes.byref(n))
            elif family == "rs":
                rc = self.lib.mp4x_ipc_occupancy_rs(dt, code, self.p, ctypes.byref(n))
            else:
                rc = self.lib.mp4x_ipc_occupancy_misc(self._OCC_FAMILY[family], dt, self.p, ctypes.byref(n))
            api = n.value if rc == 0 else 0
        except Exception:   # noqa: BLE001 — the compiler table still bounds it
            api = 0
        if self.cus is None:
            self.cus = int(torch.cuda.get_device_properties(self.device).multi_processor_count)
        tbl = occupancy.table_bpc(family, dt, DType(dt).name, code, self.p)
        known = [x for x in (api, tbl) if x]
        bpc = min(known) if known else 1
        cap = occupancy.shared_grid_cap(self.cus, bpc, self.share)
        self.grid_caps[key] = cap
        self._cap_fast[(family, dtype, op)] = cap
        LOG.info("rank %d: grid cap %s %s op=%d p=%d share=%d: %d blocks (blocks/CU: api %s, compiler %s)",
                 self.rank, family, DType(dt).name, code, self.p, self.share, cap, api, tbl)
        return cap

    def grid_caps_summary(self) -> dict:
        """The caps computed so far, JSON-able (rehearsal / bench records)."""
        return {f"{f}:{str(d).replace('torch.', '') if d is not None else '-'}:{c}": v
                for (f, d, c), v in sorted(self.grid_caps.items(), key=str)}

    def supports(self, t: torch.Tensor, op) -> bool:
        return ipc_op_ok(t.dtype, op)

    def allreduce(self, view: torch.Tensor, op, algo: int = ONESHOT, out: Optional[torch.Tensor] = None,
                  blocks: int = 0, overlap: Optional[bool] = None, scale: float = 1.0,
                  capturing: Optional[bool] = None) -> torch.Tensor:
        """In place (or into ``out``) allreduce of a contiguous device tensor.

        ``overlap`` (messages larger than the buffer): pipeline half-buffer pieces with the
        input copies on a side stream; default from ``MP4X_IPC_OVERLAP`` (0).  It pays when the
        kernel is xGMI-bound; on a GPU shared by all ranks (single-GPU rehearsal) the copies
        compete for the same HBM and it measured 2x slower (profiles/r1/ipc_large_shared_gpu.jsonl)."""
        self.raise_if_failed()
        if out is None:
            out = view
        if not view.is_contiguous() or not out.is_contiguous():
            raise Mp4jException("IPC allreduce needs contiguous tensors")
        es = view.element_size()
        total = view.numel() * es
        if total % 16:
            raise Mp4jException("IPC allreduce needs 16-byte multiples")
        if out.data_ptr() % 16:
            # an oddly offset output on THIS rank must not change the protocol the peers run:
            # reduce into an aligned temporary (allocator-aligned) and copy out
            tmp = torch.empty(view.numel(), dtype=view.dtype, device=view.device)
            self.allreduce(view, op, algo, out=tmp, blocks=blocks, overlap=overlap, scale=scale)
            out.copy_(tmp)
            return out
        dt = int(dtype_of_torch(view.dtype))
        if not blocks and self.shared_gpu:
            blocks = self.latency_blocks(total, algo, view.dtype, op)
        if overlap is None:
            overlap = self._overlap_default
        if capturing is None:                      # the engine's latency path already knows
            capturing = capturing_now()
        if total > self.nbytes and overlap and not capturing:
            return self._allreduce_pipelined(view.view(torch.uint8), out.view(torch.uint8), total, dt, op, algo,
                                             blocks, out, scale)
        piece = self.nbytes - self.nbytes % 16
        off = 0
        st = self._launch_stream()
        # once prepare_graph() ran, EVERY call (eager or captured) takes its epoch from the device
        # counter, so eager calls and graph replays can interleave without reusing an epoch
        if capturing and self._epoch_dev is None:
            raise Mp4jException("call IpcAllreduce.prepare_graph() (collectively) before capturing")
        edev = self._epoch_dev.data_ptr() if self._epoch_dev is not None else None
        sp, dp = view.data_ptr(), out.data_ptr()
        # one piece that fits a slot -> the double-buffered slots (no end barrier).  The decision
        # must be the same on every rank, so it never depends on this rank's input alignment: a
        # slotted call needs the fused copy-in, and an unaligned input is first copied to an
        # aligned temporary (rank-local, the protocol is unchanged)
        slotted = self._fuse_copy and total <= piece and total <= self._slot_bytes
        if slotted and sp % 16:
            view = view.clone()
            sp = view.data_ptr()
        fused = sp % 16 == 0 and self._fuse_copy   # copy-in inside the kernel: one launch
        lx = native.launch_ext()
        code = int(op.code)
        while off < total:
            m = min(piece, total - off)
            if not fused:
                check(self.lib.mp4x_memcpy_async(self._data.value, sp + off, m, st), "ipc input copy")
            self._next_epoch(st, capturing)
            sb, sv = (self._slot_base, self._slot_vecs) if slotted else (0, 0)
            if lx is not None:
                rc = lx.allreduce_ex(algo, dt, code, self._pp_data_addr, self._pp_sig_addr, self.rank, self.p, m,
                                     sp + off if fused else None, dp + off, self.epoch, blocks, edev, scale, st, sb, sv)
            else:
                rc = self.lib.mp4x_ipc_allreduce_ex2(algo, dt, code, self._pp_data[0], self._pp_sig[0], self.rank,
                                                     self.p, m, sp + off if fused else None, dp + off, self.epoch,
                                                     blocks, edev, scale, st, sb, sv)
            check(rc, "mp4x_ipc_allreduce")
            off += m
        return out

    def _allreduce_pipelined(self, src, dst, total, dt, op, algo, blocks, out, scale=1.0):
        """Messages larger than the buffer: two half-buffers, the input copy of piece i+1 (side
        stream, HBM-bound) overlaps the xGMI-bound kernel of piece i.

        A half is refilled only after the kernel that last used it completed on THIS rank; that
        kernel's end barrier already guarantees every peer finished reading it.
        """
        half = (self.nbytes // 2) // 4096 * 4096
        if self._pp_hi is None:
            self._pp_hi = ptr_array([d + half for d in self.data_ptrs])
            self._copy_stream = torch.cuda.Stream()
        main = torch.cuda.current_stream()
        cs = self._copy_stream
        edev = self._epoch_dev.data_ptr() if self._epoch_dev is not None else None
        self.order().enter(stream_ptr(main))    # (before the side stream joins main)
        cs.wait_stream(main)            # the input was produced on the caller's stream
        kdone = [None, None]
        ms = stream_ptr(main)
        css = stream_ptr(cs)
        off = 0
        i = 0
        while off < total:
            m = min(half, total - off)
            slot = i & 1
            if kdone[slot] is not None:
                cs.wait_event(kdone[slot])
            check(self.lib.mp4x_memcpy_async(self.data_ptrs[self.rank] + slot * half, src.data_ptr() + off, m, css),
                  "ipc input copy")
            ev = torch.cuda.Event()
            ev.record(cs)
            main.wait_event(ev)
            self._next_epoch(ms, False)
            pp = self._pp_hi[0] if slot else self._pp_data[0]
            check(self.lib.mp4x_ipc_allreduce_ex(algo, dt, int(op.code), pp, self._pp_sig[0], self.rank, self.p, m,
                                                 None, dst.data_ptr() + off, self.epoch, blocks, edev, scale, ms),
                  "mp4x_ipc_allreduce")
            kd = torch.cuda.Event()
            kd.record(main)
            kdone[slot] = kd
            off += m
            i += 1
        return out


    # ---------------------------------------------------------------- registered buffers (zero-copy)
    # A caller tensor registered on every rank (collectively, like ncclCommRegister) is mapped
    # into every peer: the two-shot then reads and writes the peers' tensors directly — no
    # staging copy, no piece loop, for any size.  Rank r's kernel writes only chunk r of its own
    # tensor in the reduce-scatter half and only the foreign chunks in the all-gather half; the
    # start / mid / end barriers order those against the peers' reads (csrc/runtime/ipc.hip).
    # Contract: every rank registers the same-shaped tensor at the same point, keeps it alive
    # (and its caching-allocator segment) until ``deregister``, and runs allreduces on it (or on
    # the same [from, to) views of it) on every rank; a rank that runs the staged protocol
    # against a zero-copy peer fails that call at once (epoch tag) instead of mixing buffers.
    def register(self, t: torch.Tensor) -> bool:
        """Collective.  Map ``t`` (contiguous, 16-byte aligned, 16-byte multiple) into every peer.
        Returns True when every rank registered it (False on every rank otherwise).

        The registration holds a reference to ``t`` until :meth:`deregister`: its memory can
        never go back to the caching allocator (and be handed to another tensor at the same
        address) while peers still hold mappings of it."""
        key = (t.data_ptr(), t.numel() * t.element_size())
        if key in self._regs:
            ok_local = 1
        else:
            ok_local = 0
        hs = self.lib.mp4x_ipc_handle_size()
        blob = None
        err = None
        scr_alloc = None
        try:
            if not t.is_cuda or not t.is_contiguous() or t.data_ptr() % 16 or key[1] % 16 or key[1] == 0:
                raise Mp4jException("register needs a contiguous, 16-byte aligned device tensor of 16-byte multiple size")
            base, size = c_void_p(), c_size_t()
            check(self.lib.mp4x_mem_range(c_void_p(t.data_ptr()), ctypes.byref(base), ctypes.byref(size)), "mem_range")
            if size.value > IPC_OPEN_MAX:
                raise Mp4jException(f"allocation of {size.value} bytes is above the IPC open limit ({IPC_OPEN_MAX}); "
                                    f"allocate it with memAlloc")
            h = ctypes.create_string_buffer(hs)
            check(self.lib.mp4x_ipc_get_handle(base, h), "ipc_get_handle(registered)")
            scr_h = None
            if PUSH_ON and not ok_local:
                scr_alloc = self._alloc_scratch(key[1], hs)
                scr_h = scr_alloc[1]
            blob = (h.raw, t.data_ptr() - base.value, key[1], ok_local, scr_h)
        except Exception as e:   # noqa: BLE001 — travels in the allgather: every rank decides together
            err = str(e)
        allb = self.comm.server.call("allgather_obj", self.rank, (blob, err))
        errs = [(i, e) for i, (_, e) in enumerate(allb) if e]
        if errs or len({b[2] for b, _ in allb}) != 1:
            if self.rank == 0:            # agreed: every rank returns False; say why once
                LOG.warning("registerBuffer(%d bytes) refused: %s", key[1],
                            errs or f"sizes differ across ranks {[b[2] for b, _ in allb]}")
            self._free_scratch(scr_alloc)
            return False
        if all(b[3] for b, _ in allb):
            return True                               # already registered everywhere
        reg = _Reg(keep=t)
        err = None
        push = all(b[4] is not None for b, _ in allb)      # every rank has a receive scratch
        if not push:
            self._free_scratch(scr_alloc)
            scr_alloc = None
        scr = []
        try:
            for r, (b, _) in enumerate(allb):
                if r == self.rank:
                    reg.peers.append(t.data_ptr())
                    if push:
                        scr.append(scr_alloc[0].value)
                    continue
                hk = (r, bytes(b[0]))
                reg.peers.append(self._open_peer_base(hk, hs) + int(b[1]))
                reg.peer_keys.append(hk)
                if push:
                    sk = (r, bytes(b[4]))
                    scr.append(self._open_peer_base(sk, hs))
                    reg.peer_keys.append(sk)
                    reg.scr_keys.append(sk)
        except Exception as e:   # noqa: BLE001
            err = str(e)
        reg.scratch = scr if push else None
        reg.scratch_alloc = scr_alloc
        oks = self.comm.server.call("allgather_obj", self.rank, err)
        if any(oks):
            if self.rank == 0:
                LOG.warning("registerBuffer(%d bytes): peer mapping failed on ranks %s", key[1],
                            [(i, o) for i, o in enumerate(oks) if o])
            self._release_ordered(reg)                # agreed: every rank is here
            return False
        old = self._regs.get(key)
        if old is not None:
            # registered on this rank already but not on every rank: the new entry replaces it
            self._release(old)
        self._regs[key] = reg
        self._changed()
        return True

    def _open_peer_base(self, hk, hs: int) -> int:
        """Mapped address of peer allocation ``hk`` = (rank, handle bytes), opened once and
        reference-counted per registration using it (several registered tensors can share one
        caching-allocator segment); :meth:`_close_peer` closes it when the last one is released."""
        ent = self._peer_bases.get(hk)
        if ent is None:
            hb = ctypes.create_string_buffer(hk[1], hs)
            ptr = c_void_p()
            check(self.lib.mp4x_ipc_open_handle(hb, ctypes.byref(ptr)), f"ipc_open_handle(rank {hk[0]})")
            ent = self._peer_bases[hk] = ptr
        self._peer_refs[hk] = self._peer_refs.get(hk, 0) + 1
        return ent.value

    def _close_peer(self, hk, keep: bool = False) -> None:
        """Drop one registration's use of peer mapping ``hk``; the last one closes it
        (``CLOSE_PEERS``; otherwise it stays cached until close()).  ``keep``: a peer's pooled
        push scratch — its mapping stays open for the next registration the owner hands the
        same scratch to (same handle bytes)."""
        n = self._peer_refs.get(hk, 0) - 1
        if n > 0:
            self._peer_refs[hk] = n
            return
        self._peer_refs.pop(hk, None)
        if CLOSE_PEERS and not keep:
            ptr = self._peer_bases.pop(hk, None)
            if ptr is not None:
                native.soft_check(self.lib.mp4x_ipc_close_handle(ptr), "ipc_close_handle", LOG)

    @staticmethod
    def _scratch_class(size: int) -> int:
        """Pool size class of a push scratch of ``size`` bytes: the next power of two (>= 64 KiB),
        or the exact size where that power of two is above the IPC open limit."""
        c = 1 << 16
        while c < size:
            c <<= 1
        return c if c <= IPC_OPEN_MAX else size

    def _alloc_scratch(self, nbytes: int, hs: int):
        """Receive scratch of the push two-shot for a registered tensor of ``nbytes``: p-1 chunk
        slots, uncached (peers write it over xGMI, this rank reads it once per call).  Returns
        (allocation, IPC handle), or (None, None): the registration then has no push form.

        Scratches are POOLED per power-of-two size class and never freed before close(); the
        peers keep their mappings of them (``_close_peer(keep=True)``).  Round 4's corruption
        (profiles/r5/rootcause/) needed a scratch to be RELEASED mid-job — the owner's free AND
        every peer's close (keeping either one alive removed it; the order of the two did not
        matter): the first kernels of the IPC instance created right afterwards stored their
        barrier flags into the owner's newly allocated memory."""
        chunk = -(-(nbytes // 16) // self.p)
        size = max(16, (self.p - 1) * chunk * 16)
        if not FREE_SCRATCH:                   # (the diagnosis knob keeps round 4's exact sizes)
            size = self._scratch_class(size)
        pooled = self._scratch_pool.get(size)
        if pooled:
            return pooled.pop()
        ptr = c_void_p()
        try:
            if size > IPC_OPEN_MAX:
                return None, None
            check(self.lib.mp4x_ipc_alloc(size, ctypes.byref(ptr)), "ipc_alloc(scratch)")
            h = ctypes.create_string_buffer(hs)
            check(self.lib.mp4x_ipc_get_handle(ptr, h), "ipc_get_handle(scratch)")
        except Exception:   # noqa: BLE001
            if ptr:
                native.soft_check(self.lib.mp4x_ipc_free(ptr), "ipc_free", LOG)
            return None, None
        self._scratch_size[ptr.value] = size
        return ptr, h.raw

    def _free_scratch(self, scr) -> None:
        """Return a push scratch to the per-size-class pool (freed at close(), see
        :meth:`_alloc_scratch`)."""
        if scr and scr[0]:
            if FREE_SCRATCH:                  # diagnosis knob: round 4's release
                self._scratch_size.pop(scr[0].value, None)
                native.soft_check(self.lib.mp4x_ipc_free(scr[0]), "ipc_free", LOG)
                return
            self._scratch_pool.setdefault(self._scratch_size[scr[0].value], []).append(scr)

    def _release_imports(self, reg: "_Reg") -> None:
        """The importer half of a release: this rank's uses of the peers' mappings
        (:meth:`_close_peer`) and its imported memAlloc views."""
        scr_keys = set(reg.scr_keys)
        for hk in reg.peer_keys:
            self._close_peer(hk, keep=hk in scr_keys and not FREE_SCRATCH)   # pooled scratches stay mapped
        reg.peer_keys = []
        for i in reversed(range(reg.nown, len(reg.vmm))):
            reg.vmm[i].free(self._keep_va(own=False))
        del reg.vmm[reg.nown:]

    def _flush_translations(self) -> None:
        """After this rank closed IPC mappings of peer memory: map and unmap one small buffer in
        this process's GPU address space, then drain the device.  Round 5 found (profiles/r5/
        rootcause/) that right after an importer closes a mapping and the owner releases the
        memory, the importer's GPU can still reach the old pages through the closed mapping's
        address for a short while; an IPC mapping opened at that address in that window sent the
        first kernels' stores into pages the owner had already reused.  One map / unmap (or
        ~100 ms) closed the window in every run; it costs ~0.1 ms per release.
        ``MP4X_IPC_FLUSH_ON_CLOSE=0`` skips it (diagnosis)."""
        if os.environ.get("MP4X_IPC_FLUSH_ON_CLOSE", "1") != "1" or self.lib is None:
            return
        ptr = c_void_p()
        if self.lib.mp4x_ipc_alloc(2 << 20, ctypes.byref(ptr)) == 0:
            native.soft_check(self.lib.mp4x_ipc_free(ptr), "ipc_free", LOG)
        else:
            native.clear_hip_error()
        torch.cuda.synchronize(self.device)

    def _release_own(self, reg: "_Reg") -> None:
        """The owner half: this rank's push scratch, own memAlloc regions / chunks, tensor reference."""
        self._free_scratch(reg.scratch_alloc)
        reg.scratch_alloc = None
        for i in reversed(range(len(reg.vmm))):
            reg.vmm[i].free(self._keep_va(own=True))
        reg.vmm = []
        reg.nown = 0
        reg.keep = None
        if reg.chunks is not None and self._chunk_pool is not None:
            self._chunk_pool.give(reg.chunks)
            reg.chunks = []

    def _release(self, reg: "_Reg") -> None:
        """Rank-local release of ``reg``: the importer half, then the owner half.  The collective,
        ordered form (no owner frees before every importer closed) is :meth:`_release_ordered`;
        this one serves close() and the memAlloc paths that order themselves."""
        if UNORDERED_RELEASE:           # test knob: round 4's order (own scratch freed first)
            self._free_scratch(reg.scratch_alloc)
            reg.scratch_alloc = None
        self._release_imports(reg)
        self._release_own(reg)

    @staticmethod
    def _keep_va(own: bool = True):
        """The VA quarantine a released memAlloc range (this rank's own, or an imported peer
        view) goes to under :data:`VMM_POLICY` (None: free the range)."""
        from . import vmm
        keep = VMM_POLICY in ("chunks", "pool", "fresh_va") or \
            VMM_POLICY == ("keep_owner_va" if own else "keep_import_va")
        return vmm.va_quarantine() if keep else None

    def _release_ordered(self, reg: Optional["_Reg"]) -> None:
        """Collective release of a registration (``reg`` may be None on a rank that has none: it
        still joins the barrier).  Every rank drains its stream, closes ITS mappings of the
        peers' tensors and push scratches, a control-plane barrier, then each owner frees its
        own push scratch — no memory is freed while a peer still maps it (the order of
        :meth:`mem_free`; ``_release`` alone is the rank-local teardown used at close)."""
        torch.cuda.synchronize(self.device)
        if UNORDERED_RELEASE:           # test knob: round 4's order (owner first, nothing agreed)
            if reg is not None:
                self._release(reg)
            return
        if reg is not None:
            self._release_imports(reg)
            self._flush_translations()
        self.comm.server.call("barrier", self.rank)         # every importer closed its mappings
        if reg is not None:
            self._release_own(reg)

    def deregister(self, t: torch.Tensor) -> None:
        """Collective: forget ``t`` on every rank (the registration contract: every rank
        deregisters its tensor at the same point).  Ordered like :meth:`mem_free` — every rank
        drains its stream and closes its mappings of the peers' tensors and scratches, a
        barrier, and only then does each owner free its push scratch (:meth:`_release_ordered`).
        A memAlloc tensor stays registered until memFree (a collective fact: no barrier then)."""
        key = (t.data_ptr(), t.numel() * t.element_size())
        reg = self._regs.get(key)
        if reg is not None and reg.vmm:
            return
        if reg is not None:
            del self._regs[key]
            self._changed()
        self._release_ordered(reg)

    def _find(self, view: torch.Tensor):
        """(registration, byte offset of ``view`` in it) or (None, 0)."""
        if not self._regs:
            return None, 0
        a = view.data_ptr()
        n = view.numel() * view.element_size()
        hit = self._regs.get((a, n))            # the whole registered tensor: O(1)
        if hit is not None:
            return hit, 0
        for (ptr, nb), reg in self._regs.items():
            if ptr <= a and a + n <= ptr + nb:
                return reg, a - ptr
        return None, 0

    def registered(self, view: torch.Tensor):
        """Peer pointers of ``view`` when it lies inside a registered tensor and is a whole number
        of 16-byte vectors at a 16-byte aligned address (what the zero-copy kernels move), else
        None — a [from, to) view off that grid takes the staged kernels.  The alignment of a
        view is rank-independent: every rank's registered allocation is 16-byte aligned and
        the range is the same on every rank."""
        if view.data_ptr() % 16 or (view.numel() * view.element_size()) % 16:
            return None
        reg, d = self._find(view)
        if reg is None:
            return None
        return reg.peers if d == 0 else [q + d for q in reg.peers]

    def scratch_of(self, view: torch.Tensor):
        """Every rank's push scratch for ``view``'s registered tensor, or None (no push form)."""
        reg, _ = self._find(view)
        return None if reg is None else reg.scratch

    # ---------------------------------------------------------------- memAlloc (any size)
    def mem_alloc(self, nbytes: int, dtype: torch.dtype) -> torch.Tensor:
        """Collective (``ProcessCommSlave.memAlloc``): a ``nbytes`` device tensor that is mapped
        into every peer from the start — registered for the zero-copy kernels at ANY size, as
        one contiguous range per peer (parallel/vmm.py, csrc/runtime/vmm.hip).  Also allocates
        the push scratch the same way.  Raises on every rank when any rank failed."""
        from . import vmm
        nb16 = -(-int(nbytes) // 16) * 16
        es = torch.empty((), dtype=dtype).element_size()
        if VMM_POLICY == "chunks":
            return self._mem_alloc_chunks(nbytes, nb16, es, dtype)
        pooled = self._vmm_pool.get(nb16) if not VMM_RELEASE else None
        if pooled:
            # a freed allocation of this size (the same one on every rank: pool states agree)
            reg = pooled.pop()
            own_va = reg.vmm[0].va
            self._regs[(own_va, nb16)] = reg
            self._changed()
            t = vmm.tensor_at(own_va, nb16, torch.uint8, torch.device("cuda", self.device))
            return t[:nbytes // es * es].view(dtype)
        own = scr = None
        err = None
        plan = None
        try:
            g = ctypes.c_size_t()
            check(self.lib.mp4x_vmm_granularity(ctypes.byref(g)), "vmm_granularity")
            chunk, n = vmm.chunk_plan(nb16, g.value)
            own = vmm.VmmRegion.create(self.lib, chunk, n)
            sbytes = (self.p - 1) * (-(-(nb16 // 16) // self.p)) * 16
            schunk, sn = vmm.chunk_plan(max(16, sbytes), g.value)
            scr = vmm.VmmRegion.create(self.lib, schunk, sn) if PUSH_ON else None
            plan = (chunk, n, schunk if scr else 0, sn if scr else 0)
        except Exception as e:   # noqa: BLE001 — agreed below
            err = f"{type(e).__name__}: {e}"
        plans = self.comm.server.call("allgather_obj", self.rank, (plan, err))
        bad = [(i, e) for i, (_, e) in enumerate(plans) if e]
        if bad:
            for region in (own, scr):
                if region is not None:
                    region.free()
            raise Mp4jException(f"memAlloc({nbytes}) failed on ranks {bad}")
        push = all(pl[2] for pl, _ in plans)
        mine = own.fds + (scr.fds if (push and scr) else [])
        try:
            got = vmm.exchange_fds(self.comm.server, self.rank, self.p, mine)
        except Exception:
            for region in (own, scr):
                if region is not None:
                    region.free()
            raise
        own.close_fds()
        if scr is not None:
            scr.close_fds()
        reg = _Reg(keep=None)
        reg.vmm = [own] + ([scr] if scr is not None else [])
        reg.nown = len(reg.vmm)
        scratch = []
        err = None
        try:
            for r in range(self.p):
                if r == self.rank:
                    reg.peers.append(own.va)
                    scratch.append(scr.va if push else 0)
                    continue
                chunk, n, schunk, sn = plans[r][0]
                fds = got[r]
                pr = vmm.VmmRegion.import_fds(self.lib, fds[:n], chunk)
                reg.vmm.append(pr)
                reg.peers.append(pr.va)
                if push:
                    ps = vmm.VmmRegion.import_fds(self.lib, fds[n:n + sn], schunk)
                    reg.vmm.append(ps)
                    scratch.append(ps.va)
        except Exception as e:   # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        finally:
            for fl in got.values():             # every received fd, also after a failure midway
                for fd in fl:
                    os.close(fd)
        oks = self.comm.server.call("allgather_obj", self.rank, err)
        if any(oks):
            self._release_ordered(reg)          # agreed: every rank is here
            raise Mp4jException(f"memAlloc({nbytes}) peer mapping failed on ranks "
                                f"{[(i, o) for i, o in enumerate(oks) if o]}")
        reg.scratch = scratch if push else None
        t = vmm.tensor_at(own.va, nb16, torch.uint8, torch.device("cuda", self.device))
        self._regs[(own.va, nb16)] = reg
        self._changed()
        return t[:nbytes // es * es].view(dtype)

    def _mem_alloc_chunks(self, nbytes: int, nb16: int, es: int, dtype: torch.dtype) -> torch.Tensor:
        """memAlloc under the chunk pool (``VMM_POLICY == "chunks"``): this rank takes chunks from
        its pool (new ones only when none of a size is free), maps them at a fresh VA range, and
        tells every peer which chunk ids the tensor (and its push scratch) is made of; only NEW
        chunks' fds travel, a reused chunk is mapped again from the handle each peer kept."""
        from . import vmm
        pool = self._chunk_pool
        if pool is None:
            pool = self._chunk_pool = vmm.ChunkPool(self.lib)
        own_c, scr_c, maps = [], [], []
        err = plan = None
        try:
            g = ctypes.c_size_t()
            check(self.lib.mp4x_vmm_granularity(ctypes.byref(g)), "vmm_granularity")
            own_c = pool.take(vmm.chunk_sizes(nb16, g.value))
            maps.append(vmm.MappedRange(self.lib, [c.handle for c in own_c], [c.size for c in own_c]))
            if PUSH_ON:
                sbytes = (self.p - 1) * (-(-(nb16 // 16) // self.p)) * 16
                scr_c = pool.take(vmm.chunk_sizes(max(16, sbytes), g.value))
                maps.append(vmm.MappedRange(self.lib, [c.handle for c in scr_c], [c.size for c in scr_c]))
            plan = ([(c.id, c.size, c.fd >= 0) for c in own_c], [(c.id, c.size, c.fd >= 0) for c in scr_c])
        except Exception as e:   # noqa: BLE001 — agreed below
            err = f"{type(e).__name__}: {e}"
        plans = self.comm.server.call("allgather_obj", self.rank, (plan, err))
        bad = [(i, e) for i, (_, e) in enumerate(plans) if e]
        if bad:
            for m in maps:
                m.free()
            pool.give(own_c + scr_c)
            raise Mp4jException(f"memAlloc({nbytes}) failed on ranks {bad}")
        push = all(pl[1] for pl, _ in plans)
        new_own = [c for c in own_c + (scr_c if push else []) if c.fd >= 0]
        got = {}
        if any(new for pl, _ in plans for part in pl for (_, _, new) in part):
            try:
                got = vmm.exchange_fds(self.comm.server, self.rank, self.p, [c.fd for c in new_own])
            except Exception:   # agreed inside exchange_fds: every rank is here
                for m in maps:
                    m.free()
                pool.give(own_c + scr_c)          # unsent: their fds stay open for a later send
                raise
        for c in new_own:                       # sent: every peer holds these chunks now
            os.close(c.fd)
            c.fd = -1                           # (an unsent chunk keeps its fd for a later send)
        reg = _Reg(keep=None)
        reg.vmm = list(maps) if push else maps[:1]
        reg.nown = len(reg.vmm)
        reg.chunks = own_c + scr_c
        if not push and len(maps) > 1:
            maps[1].free()
        scratch = []
        err = None
        try:
            for r in range(self.p):
                if r == self.rank:
                    reg.peers.append(maps[0].va)
                    scratch.append(maps[1].va if push else 0)
                    continue
                fds = list(got.get(r, []))
                parts = plans[r][0][0] + (plans[r][0][1] if push else [])
                for cid, _, new in parts:
                    if new:
                        pool.import_fd(r, cid, fds.pop(0))
                for part, dst in ((plans[r][0][0], reg.peers), (plans[r][0][1] if push else None, scratch)):
                    if part is None:
                        continue
                    view = vmm.MappedRange(self.lib, [pool.peer[(r, cid)] for cid, _, _ in part],
                                           [sz for _, sz, _ in part])
                    reg.vmm.append(view)
                    dst.append(view.va)
        except Exception as e:   # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        finally:
            for fl in got.values():             # every received fd, also after a failure midway
                for fd in fl:
                    os.close(fd)
        oks = self.comm.server.call("allgather_obj", self.rank, err)
        if any(oks):
            # a chunk sent in THIS call may be missing on some peer: never hand it out again
            sent = set(map(id, new_own))
            reg.chunks = [c for c in reg.chunks if id(c) not in sent]
            self._release_ordered(reg)          # agreed: every rank is here
            pool.discard(new_own)
            raise Mp4jException(f"memAlloc({nbytes}) peer mapping failed on ranks "
                                f"{[(i, o) for i, o in enumerate(oks) if o]}")
        reg.scratch = scratch if push else None
        t = vmm.tensor_at(maps[0].va, nb16, torch.uint8, torch.device("cuda", self.device))
        self._regs[(maps[0].va, nb16)] = reg
        self._changed()
        return t[:nbytes // es * es].view(dtype)

    def mem_free(self, t: torch.Tensor) -> None:
        """Collective: release a :meth:`mem_alloc` tensor on every rank (its peers' mappings
        first, after every rank's stream drained)."""
        key = None
        for k, reg in self._regs.items():
            if reg.vmm and k[0] == t.data_ptr():
                key = k
                break
        if key is None:
            raise Mp4jException("memFree: not a memAlloc tensor of this communicator")
        torch.cuda.synchronize(self.device)
        self.comm.server.call("barrier", self.rank)     # no peer kernel still reads or writes it
        reg = self._regs.pop(key)
        self._changed()
        if reg.chunks is not None:
            # chunk pool: unmap every view (own + peers', VA ranges stay reserved) and return this
            # rank's chunks to its pool; nothing is released (csrc/runtime/vmm.hip says why)
            self._release(reg)
            return
        if not VMM_RELEASE:
            # park the allocation in a per-size pool, handed out again by the next memAlloc of the
            # same size (every rank's pool state is identical: alloc / free are collective)
            self._vmm_pool.setdefault(key[1], []).append(reg)
            return
        # Ordered, collective release.  Round 3 released every rank's imported views and its own
        # chunks in one local pass, so an owner could release its chunks while a peer still had
        # them imported and mapped; the next allocation's peer views then read zeros.  Here every
        # importer unmaps and releases first, and the owners release only after all have.
        for region in reg.vmm[reg.nown:]:
            region.free(self._keep_va(own=False))
        torch.cuda.synchronize(self.device)
        self.comm.server.call("barrier", self.rank)     # every peer released its imports
        for region in reg.vmm[:reg.nown]:
            region.free(self._keep_va(own=True))
        reg.vmm = []
        reg.keep = None

    def allreduce_push(self, view: torch.Tensor, op, peers, scratch, scale: float = 1.0) -> torch.Tensor:
        """In place, on registered tensors, with every xGMI transfer a posted WRITE (see
        ``k_ipc_twoshot_push``): one kernel, any size."""
        self.raise_if_failed()
        total = view.numel() * view.element_size()
        if total % 16 or view.data_ptr() % 16:
            raise Mp4jException("zero-copy IPC allreduce needs 16-byte aligned, 16-byte multiple views")
        if torch.cuda.is_current_stream_capturing() and self._epoch_dev is None:
            raise Mp4jException("call IpcAllreduce.prepare_graph() (collectively) before capturing")
        self._push_ptrs(total, op, peers, scratch, view.dtype, scale)
        return view

    def _push_ptrs(self, total: int, op, peers, scratch, dtype, scale: float = 1.0) -> None:
        st = self._launch_stream()
        edev = self._next_epoch(st)
        chunk = -(-(total // 16) // self.p)
        blocks = max(1, min(self.grid_cap("push", dtype, op), -(-chunk // 512))) if self.shared_gpu else 0
        pp = ptr_array(peers)
        sp = ptr_array(scratch)
        check(self.lib.mp4x_ipc_allreduce_push(int(dtype_of_torch(dtype)), int(op.code), pp[0], sp[0],
                                               self._pp_sig[0], self.rank, self.p, total,
                                               self.epoch | ZC_TAG | PUSH_TAG, blocks, edev, scale, st),
              "mp4x_ipc_allreduce_push")

    def allreduce_registered(self, view: torch.Tensor, op, peers, scale: float = 1.0, grid: int = 0) -> torch.Tensor:
        """In-place two-shot straight on the registered tensors (see :meth:`register`): ONE
        kernel, no staging and no pieces, whatever the size."""
        total = view.numel() * view.element_size()
        if total % 16 or view.data_ptr() % 16:
            raise Mp4jException("zero-copy IPC allreduce needs 16-byte aligned, 16-byte multiple views")
        if torch.cuda.is_current_stream_capturing() and self._epoch_dev is None:
            raise Mp4jException("call IpcAllreduce.prepare_graph() (collectively) before capturing")
        self.allreduce_registered_ptrs(view.data_ptr(), total, op, peers, view.dtype, scale, grid)
        return view

    def allreduce_registered_ptrs(self, dst: int, total: int, op, peers, dtype, scale: float = 1.0,
                                  grid: int = 0) -> None:
        """The zero-copy two-shot on raw pointers (``dst`` = this rank's buffer, ``peers`` = every
        rank's mapped buffer).  ``grid``: block count (0 = the default, up to one per CU; the
        autotuner's ``ipc2z_b<N>`` candidates try fewer — fewer, longer-lived readers per link)."""
        self.raise_if_failed()
        st = self._launch_stream()
        edev = self._next_epoch(st)
        blocks = self._grid(total // 16, "twoshot", dtype, op)   # >= 8: every XCD passes the barriers
        if grid > 0:
            blocks = min(grid, self.grid_cap("twoshot", dtype, op))
        pp = self._peer_pp(peers)
        lx = native.launch_ext()
        if lx is not None:
            rc = lx.allreduce_ex(TWOSHOT, int(dtype_of_torch(dtype)), int(op.code), ctypes.addressof(pp[1]),
                                 self._pp_sig_addr, self.rank, self.p, total, None, dst, self.epoch | ZC_TAG, blocks,
                                 edev, scale, st)
        else:
            rc = self.lib.mp4x_ipc_allreduce_ex(TWOSHOT, int(dtype_of_torch(dtype)), int(op.code), pp[0],
                                                self._pp_sig[0], self.rank, self.p, total, None, dst,
                                                self.epoch | ZC_TAG, blocks, edev, scale, st)
        check(rc, "mp4x_ipc_allreduce(zero-copy)")

    def _peer_pp(self, peers):
        """The native pointer array of a registration's peer list, built once per list object
        (the per-call path of the zero-copy forms; a registration keeps its list)."""
        cache = self.__dict__.setdefault("_pp_cache", {})
        ent = cache.get(id(peers))
        if ent is None or ent[0] is not peers:
            if len(cache) >= 256:
                cache.clear()
            ent = cache[id(peers)] = (peers, ptr_array(peers))
        return ent[1]

    # ---------------------------------------------------------------- fused fp8 two-shot
    QBLOCK = 256
    FP8_DTYPES = (torch.float32, torch.bfloat16, torch.float16)

    def fp8_ok(self, view: torch.Tensor) -> bool:
        """Rank-independent qualification (dtype, shape); an oddly offset tensor on one rank is
        handled inside :meth:`allreduce_fp8` so every rank runs the same kernels."""
        return view.dtype in self.FP8_DTYPES and view.is_contiguous() \
            and view.numel() % 4 == 0 and view.numel() > 0

    def _fp8_piece_blocks(self) -> int:
        """Quant blocks per rank chunk per piece: p * cb blocks of 256 fp8 bytes + 4-byte scales
        must fit the buffer (scales 16-byte aligned after the q bytes)."""
        per_block = self.QBLOCK + 4
        cb = (self.nbytes - 16) // (self.p * per_block)
        if cb < 1:
            raise Mp4jException("IPC buffer too small for the fp8 two-shot")
        return int(cb)

    def allreduce_fp8(self, view: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        """In-place SUM allreduce with the block-scaled e4m3 codec on the xGMI links, one fused
        kernel per piece (csrc/runtime/ipc.hip ``k_ipc_fp8_twoshot``): quantise this rank's
        piece into its own buffer (K6), then pull + dequantise + f32-sum + requantise the own
        chunk from every peer at once, then pull + dequantise every peer's chunk.  Same numerics
        as the RCCL fp8 schedule (two quantisations, f32 accumulation in rank order).  Needs
        :meth:`fp8_ok`."""
        if not self.fp8_ok(view):
            raise Mp4jException("fp8 IPC allreduce needs a contiguous f32/bf16/f16 tensor, n % 4 == 0")
        self.raise_if_failed()
        if view.data_ptr() % 16:
            self._aligned(view, lambda t: self.allreduce_fp8(t, scale))
            return view
        Q = self.QBLOCK
        n = view.numel()
        es = view.element_size()
        dt = int(dtype_of_torch(view.dtype))
        cbmax = self._fp8_piece_blocks()
        st = self._launch_stream()
        base = view.data_ptr()
        off = 0
        while off < n:
            m = min(n - off, self.p * cbmax * Q)
            cb = -(-m // (self.p * Q))                   # quant blocks per rank chunk
            nq = self.p * cb * Q                         # q bytes of this piece
            soff = (nq + 15) // 16 * 16
            own = self._data.value
            used = -(-m // Q)                            # blocks the quantiser writes
            if used < self.p * cb:                       # zero the blocks past the input
                check(self.lib.mp4x_memset_async(own + used * Q, 0, (self.p * cb - used) * Q, st), "fp8 q tail")
                check(self.lib.mp4x_memset_async(own + soff + used * 4, 0, (self.p * cb - used) * 4, st),
                      "fp8 scale tail")
            check(self.lib.mp4x_quant_fp8(dt, base + off * es, m, own, own + soff, st), "fp8 quant")
            edev = self._next_epoch(st)
            check(self.lib.mp4x_ipc_fp8_allreduce(dt, self._pp_data[0], self._pp_sig[0], self.rank, self.p, cb, soff,
                                                  base + off * es, m, self.epoch,
                                                  self._blocks_for_waves(cb if _FP8_NARROW else -(-cb // 4), view.dtype),
                                                  edev, scale, st), "mp4x_ipc_fp8_allreduce")
            off += m
        return view

    def _blocks_for_waves(self, waves: int, dtype) -> int:
        """Grid of the fused fp8 two-shot (8 waves per block).  On a GPU shared by the ranks
        (rehearsals) the cap of this kernel's occupancy applies (:meth:`grid_cap`; its 40 KB LDS
        tile and register load fit fewer blocks per CU than the generic kernels)."""
        if not self.shared_gpu:
            return 0
        return max(1, min(self.grid_cap("fp8n" if _FP8_NARROW else "fp8", dtype), -(-waves // 8)))

    def prepare_graph(self):
        """Move the epoch counter to device memory so hipGraph replays get fresh epochs.

        Collective (every rank calls it at the same point in its call sequence)."""
        if self._epoch_dev is None:
            torch.cuda.synchronize()
            self._epoch_dev = torch.full((1,), self.epoch, dtype=torch.int32, device="cuda")
            self._fast_state = None
            self._changed()
        return self

    def error_word(self, clear: bool = False) -> int:
        """This rank's barrier-timeout word (0 = fine, 1/2/3 = start/mid/end barrier timed out).

        Read on a private stream (never serialises with the caller's streams; safe from the
        watchdog thread); ``clear`` resets it so the next check starts clean."""
        if self._sig_stream is None:
            self._sig_stream = torch.cuda.Stream(device=self.device)
        v = ctypes.c_uint32(0)
        check(self.lib.mp4x_ipc_error_word(self._sig, ctypes.byref(v), int(bool(clear)),
                                           stream_ptr(self._sig_stream)), "ipc_error_word")
        if clear and self._herr:
            # the pinned host copy too: a probe timeout that was read and handled here (autotune)
            # must not fail the next call at its entry check
            ctypes.c_uint32.from_address(self._herr.value).value = 0
        return int(v.value)

    def close(self, sync: bool = True, collective: bool = False):
        """Tear the instance down: every mapping of the peers' memory first, then this rank's own
        memory.  ``collective`` (every rank closes this instance at the same point, e.g. a mid-job
        re-grow or an instance dropped after a failed first-use probe): a control-plane barrier
        between the two halves, so no owner frees what a peer still maps — the process goes on
        allocating and exporting afterwards.  Without it (process teardown, failure paths that
        cannot agree) the halves run back to back."""
        if self.lib is None or self.__dict__.get("_closed"):
            return                    # idempotent: a second (collective) close must not barrier again
        self._closed = True
        self._fast_state = None
        self._changed()
        if sync:
            torch.cuda.synchronize()
        if self._sig and self._herr:
            self.lib.mp4x_ipc_set_host_error(self._sig, None)
        # ---- importer half: the peers' staging / signal buffers, registered tensors, scratches
        for ptr in self._opened:
            native.soft_check(self.lib.mp4x_ipc_close_handle(ptr), "ipc_close_handle", LOG)
        self._opened = []
        regions = getattr(self, "_data_regions", [])
        for region in reversed(regions[1:]):               # imported views of the peers' data
            try:
                region.free(self._keep_va(own=False))
            except Exception:   # noqa: BLE001 — best effort at teardown
                pass
        del regions[1:]
        pooled = [r for lst in getattr(self, "_vmm_pool", {}).values() for r in lst]
        regs = list(getattr(self, "_regs", {}).values()) + pooled
        for reg in regs:
            try:
                self._release_imports(reg)
            except Exception:   # noqa: BLE001 — best effort at teardown
                pass
        for ptr in getattr(self, "_peer_bases", {}).values():
            native.soft_check(self.lib.mp4x_ipc_close_handle(ptr), "ipc_close_handle", LOG)
        self._peer_bases = {}
        self._peer_refs = {}
        if collective and not UNORDERED_RELEASE:
            self._flush_translations()
            self.comm.server.call("barrier", self.rank)     # every importer unmapped before the owners free
        # ---- owner half
        if self._data and not getattr(self, "_vmm_data", False):
            native.soft_check(self.lib.mp4x_ipc_free(self._data), "ipc_free", LOG)
        self._data = c_void_p()
        for region in regions:
            try:
                region.free(self._keep_va())
            except Exception:   # noqa: BLE001 — best effort at teardown
                pass
        self._data_regions = []
        if self._sig:
            native.soft_check(self.lib.mp4x_ipc_free(self._sig), "ipc_free", LOG)
            self._sig = c_void_p()
        if self._herr:
            self._herr_word = None
            self.lib.mp4x_host_word_free(self._herr)
            self._herr = c_void_p()
        for reg in regs:
            try:
                self._release_own(reg)
            except Exception:   # noqa: BLE001 — best effort at teardown
                pass
        self._regs = {}
        self._vmm_pool = {}
        if getattr(self, "_chunk_pool", None) is not None:
            self._chunk_pool.release_all()
            self._chunk_pool = None
        for lst in getattr(self, "_scratch_pool", {}).values():
            for ptr, _ in lst:
                native.soft_check(self.lib.mp4x_ipc_free(ptr), "ipc_free", LOG)
        self._scratch_pool = {}
