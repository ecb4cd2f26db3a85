"""Device data plane — GPU tensors over RCCL (xGMI) + the hand-written CDNA4 kernels.

One process per GPU.  The communicator is a ``torch.distributed`` process group with the
``nccl`` backend (= RCCL on ROCm), bootstrapped through the mp4x master (rank 0 hosts a
TCPStore whose address travels through the master's key/value service) or reused when
the launcher (torchrun) already initialised one.

Algorithm families (selected per call, see :meth:`DeviceEngine.select`):

``rccl``   RCCL's own collective (ncclAllReduce / ReduceScatter / AllGather / Broadcast /
           Reduce).  RCCL runs multi-channel rings/trees over the 7 xGMI links.  Used for
           (dtype, op) pairs RCCL supports.
``a2a``    two-shot "direct" schedule built from RCCL data movement and mp4x kernels:
           all-to-all (every rank pulls its 1/p block from all p peers over all links at
           once) → K1 multi-input reduce kernel in RANK order (deterministic, any op incl.
           bitwise / *_LOC / int16) → all-gather.  Reduce-scatter alone is the first half.
``fp8``    the same two-shot schedule with the K6 block-scaled e4m3 codec on the wire:
           quantise → all-to-all(q, scales) → fused dequant+reduce(f32)+requant →
           all-gather(q, scales) → dequant.  4x fewer bytes than f32 on every link.
``p2p``    grouped ncclSend/ncclRecv (batch_isend_irecv) for gather / scatter /
           ragged allgather: the root talks to all peers concurrently.
``ipc*``   mp4x's own xGMI kernels over IPC-mapped peer memory (parallel/ipc.py,
           csrc/runtime/ipc.hip): one-shot / two-shot allreduce through staging buffers, and
           on registered / memAlloc tensors one zero-copy kernel per call for every collective
           (two-shot pull or push, direct RS / AG, copy plans for the rooted ones).
``rhd``    recursive halving / doubling over grouped send/recv, K1 per round.
``hier``   jobs spanning nodes: IPC RS inside each node, RCCL on 1/L of the bytes across
           nodes, IPC AG (parallel/hier.py).

Autotuning (RCCL vs the IPC forms vs a2a / rhd / hier, exact-probed, agreed, pinned per size
class) lives in parallel/autotune.py.

Semantics mirror ProcessCommSlave (in place on ``[from, to)`` views, last rank takes the
remainder in allreduce/reduce splits, rank-order reductions) — see process_comm.py.
"""
from __future__ import annotations

import bisect
import contextlib
import ctypes
import datetime
import logging
import os
import time
from typing import Dict, List, NamedTuple, Optional, Sequence

import torch
import torch.distributed as dist

from ..exceptions import Mp4jException
from ..operators import DType, OpCode, Operator, dtype_of_torch, for_dtype
from ..ops.native import capturing_now
from ..utils.commutils import CommUtils
from .autotune import ZC_GRIDS, AutotuneMixin, _TunedTable, _tune_key, zc_grid  # noqa: F401 (re-exported)
from .engine_rooted import RootedMixin
from .engine_schedules import ScheduleMixin
from .hier import NodeLayout

LOG = logging.getLogger("mp4x.device")

_RCCL_OPS = {OpCode.SUM: dist.ReduceOp.SUM, OpCode.MAX: dist.ReduceOp.MAX,
             OpCode.MIN: dist.ReduceOp.MIN, OpCode.PROD: dist.ReduceOp.PRODUCT}
# dtypes RCCL reduces natively (no int16 in RCCL)
_RCCL_DTYPES = {torch.float64, torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32,
                torch.int8, torch.uint8}


_IPC_DTYPES = None
_IPC_OP_OK = None


def _ipc_dtypes():
    """``ipc.SUPPORTED_DTYPES`` without an import statement per call (the latency tier)."""
    global _IPC_DTYPES
    if _IPC_DTYPES is None:
        from .ipc import SUPPORTED_DTYPES
        _IPC_DTYPES = SUPPORTED_DTYPES
    return _IPC_DTYPES


def _ipc_op_ok(dtype, op) -> bool:
    """``ipc.ipc_op_ok`` without an import statement per call."""
    global _IPC_OP_OK
    if _IPC_OP_OK is None:
        from .ipc import ipc_op_ok
        _IPC_OP_OK = ipc_op_ok
    return _IPC_OP_OK(dtype, op)


def _env_algo() -> str:
    return os.environ.get("MP4X_DEVICE_ALGO", "auto").lower()


def _flat(t: torch.Tensor) -> torch.Tensor:
    if not t.is_contiguous():
        raise Mp4jException("device collectives need contiguous tensors")
    return t.view(-1)


def reduce_into(out: torch.Tensor, ins: Sequence[torch.Tensor], op) -> None:
    """Rank-ordered multi-input reduce ``out = op(ins[0], ins[1], ...)``: the native K1 HIP kernel on
    the GPU (never a silent torch fallback there)."""
    if getattr(op, "is_custom", False):
        acc = ins[0].clone() if ins[0].data_ptr() != out.data_ptr() else out
        for x in ins[1:]:
            acc = op.fn(acc, x)
        if acc.data_ptr() != out.data_ptr():
            out.copy_(acc)
        return
    if out.is_cuda:
        from ..ops.device_ops import reduce_
        reduce_(out, list(ins), int(op.code))
    else:   # CPU tensors: only the gloo / loopback test configurations reach this
        half = ins[0].dtype in (torch.bfloat16, torch.float16)   # K1 accumulates these in f32
        acc = (ins[0].float() if half else ins[0]).numpy().copy()
        for x in ins[1:]:
            op.reduce_into(acc, (x.float() if half else x).numpy())
        out.copy_(torch.from_numpy(acc))


def local_reduce(out: torch.Tensor, inputs: Sequence[torch.Tensor], f: int, t: int, operator):
    """out[f:t] = op(out[f:t], in_1[f:t], ...) in one K1 launch (ThreadComm thread phase, K1b)."""
    if t <= f or not inputs:
        return out
    o = _flat(out)[f:t]
    ins = [o] + [_flat(x)[f:t] for x in inputs]
    op = operator if getattr(operator, "is_custom", False) else for_dtype(operator, dtype_of_torch(o.dtype))
    reduce_into(o, ins, op)
    return out



class _ArEntry(NamedTuple):
    """A memoised staged allreduce (also a reduce's): the field order is what
    ``_mp4x_launch.fast_allreduce`` reads (csrc/pyext/launch_ext.cpp)."""
    state: int          # FastAr address (IpcAllreduce.fast_state)
    algo: int
    dtype: int
    op: int
    offset: int         # byte offset of the [from, to) range in the tensor
    nbytes: int
    blocks: int
    scale: float
    stat: str           # the engine's call count it bumps ("allreduce.ipc1", ...)
    inst: object        # keeps the instance alive with the entry
    api: str            # the API call count it bumps ("allreduceArray", ...)


class _PlanEntry(NamedTuple):
    """A memoised copy plan (``_mp4x_launch.fast_plan``)."""
    state: int
    stage: int          # address of the stage quadruples (sa)
    nstage: int
    pull: int           # address of the pull quadruples (pa)
    npull: int
    src_off: int        # byte offsets from the tensor's address, -1 = none
    out_off: int
    grid_len: int
    buf_vecs: int
    blocks: int
    stat: str
    api: str
    inst: object
    sa: object          # the ctypes arrays behind stage / pull, kept alive
    pa: object


class _RsEntry(NamedTuple):
    """A memoised fused reduce-scatter (``_mp4x_launch.fast_rs``)."""
    state: int
    dtype: int
    op: int
    seg_lo: int         # addresses of the p segment bounds (16-byte vectors)
    seg_hi: int
    src_off: int
    out_off: int
    blocks: int
    stat: str
    api: str
    inst: object
    lo_arr: object
    hi_arr: object


class _FastMemo(dict):
    """The latency fast paths' memo (call shape -> native launch entry).  Keys carry the tensor's
    address only when the tensor overlaps a registered tensor of the default IPC instance (a
    call on it, or on a [from, to) range of it, may take the zero-copy kernels), 0 otherwise:
    the staged launch of a shape does not depend on where an unregistered tensor lives.
    ``reg_starts`` / ``reg_ends``: the registered ranges, sorted and disjoint (refreshed at every
    invalidation — registration changes invalidate)."""
    __slots__ = ("reg_starts", "reg_ends")

    def __init__(self):
        super().__init__()
        self.reg_starts: list = []
        self.reg_ends: list = []

    @property
    def by_ptr(self) -> bool:
        """Is any tensor registered (then registered addresses key their own entries)?"""
        return bool(self.reg_starts)

    def addr_key(self, base: int, nbytes: int) -> int:
        """The address part of a key: ``base`` when [base, base + nbytes) overlaps a registered
        range, else 0 (the last range starting inside or before the tensor decides: the ranges
        are disjoint)."""
        s = self.reg_starts
        if not s:
            return 0
        i = bisect.bisect_right(s, base + nbytes - 1) - 1
        return base if i >= 0 and self.reg_ends[i] > base else 0


class DeviceEngine(AutotuneMixin, ScheduleMixin, RootedMixin):
    # (class defaults: engines assembled without __init__ in unit tests see one node, no hier)
    layout = NodeLayout([])
    _dm_large = "auto"
    _hier = None
    _hier_failed = False
    _hier_auto = False                    # MP4X_HIER=1: pick / autotune the node-aware schedule by itself
    hier_min_bytes = 1 << 20
    _probe_depth = 0
    _probe_s: Optional[float] = None      # explicit bound of the innermost probing(seconds) scope
    _zc_vmm = True                        # memAlloc builds VMM tensors (False: registered plain ones)
    _ipc_obj = _ipc_large = _ipc_fp8_big = None
    _fast_ar = None                       # (engines assembled without __init__: no fast path)
    _oneshot_ar_max = 0                   # the staged allreduce's one-shot limit when it differs

    def __init__(self, comm, device_index: Optional[int] = None, backend: Optional[str] = None, coll=None,
                 device=None):
        self.comm = comm
        self.rank = comm.rank
        self.p = comm.slaveNum
        self.stats: Dict[str, int] = {}
        use_cuda = torch.cuda.is_available()
        self._owns_pg = False
        self.pg = None
        if coll is not None:
            # injected back-end (LoopbackColl: p virtual ranks in one process)
            self.coll = coll
            self.backend = coll.backend
            self.device = torch.device(device) if device is not None else \
                (torch.device("cuda", torch.cuda.current_device()) if use_cuda else torch.device("cpu"))
            if self.device.type == "cuda":
                from ..ops import native
                native.hip()
        else:
            self.backend = backend or os.environ.get("MP4X_DEVICE_BACKEND") or ("nccl" if use_cuda else "gloo")
            if use_cuda:
                if device_index is None:
                    lr = os.environ.get("MP4X_DEVICE_INDEX", os.environ.get("LOCAL_RANK"))
                    device_index = int(lr) if lr is not None else self.rank % torch.cuda.device_count()
                torch.cuda.set_device(device_index)
                self.device = torch.device("cuda", device_index)
                from ..ops import native
                native.hip()   # fail loudly here if the kernels are missing on a GPU box
            else:
                self.device = torch.device("cpu")
            if dist.is_initialized():
                if dist.get_world_size() != self.p or dist.get_rank() != self.rank:
                    raise Mp4jException(f"torch.distributed already initialised with world={dist.get_world_size()} "
                                        f"rank={dist.get_rank()} but mp4x has p={self.p} rank={self.rank}")
                self.pg = dist.group.WORLD
            else:
                self._init_pg()
            from .coll import TorchColl
            self.coll = TorchColl(self.pg, self.backend)
        # the communicator's stream order (parallel/order.py): every IPC launch, fast path and
        # RCCL call of this engine runs after the previous one, whatever stream issued it
        self.order = None
        if self.device.type == "cuda" and coll is None:
            from .order import CommOrder
            self.order = CommOrder()
            self.coll.order = self.order
        self.algo = _env_algo()
        self.a2a_bytes = int(os.environ.get("MP4X_A2A_MIN_BYTES", 0))
        # custom xGMI IPC allreduce (csrc/runtime/ipc.hip) below these sizes
        self.ipc_enabled = os.environ.get("MP4X_IPC", "1") == "1" and self.device.type == "cuda" and 2 <= self.p <= 8 \
            and coll is None
        self.ipc_oneshot_max = int(os.environ.get("MP4X_IPC_ONESHOT_MAX", 256 << 10))
        self.ipc_twoshot_max = int(os.environ.get("MP4X_IPC_TWOSHOT_MAX", 16 << 20))
        # two ranks: the one-shot moves the same bytes over the one link as the two-shot with one
        # barrier fewer, so the staged allreduce takes it for every size a slot holds (measured on
        # one GPU: 1.7-2.2x faster than the two-shot at 256 KiB - 4 MiB, profiles/r5/tiers/)
        # the staged allreduce's one-shot / two-shot crossover follows the per-link byte model at
        # this rank count (parallel/tiers.py): the slot size (4 MiB) at two ranks, 512 KiB at
        # three, 256 KiB from four on; autotune re-pins the size classes it measures
        from .ipc import SLOTS_ON, SLOT_BYTES
        from .tiers import oneshot_max
        self._oneshot_ar_max = oneshot_max(self.p, SLOT_BYTES) if self.p >= 2 and SLOTS_ON and \
            "MP4X_IPC_ONESHOT_MAX" not in os.environ else 0
        self._ipc_obj = None
        self._ipc_large = None
        self._ipc_large_failed = False   # set on every rank together (setup failure is collective)
        self._ipc_fp8_big = None         # whole-tensor fp8 staging (see _ipc_fp8_whole)
        self._ipc_fp8_big_failed = False
        self.probe_failures: List[dict] = []   # first-use probe failures of lazily made instances
        self._rccl_variants: Dict[int, object] = {}   # min CTAs -> TorchColl on a dedicated communicator
        # (dtype, op code, log2 size class) -> algorithm measured fastest by autotune_allreduce
        self._fast_ar = _FastMemo()                   # latency fast path: call shape -> native launch
        self._tuned: Dict[tuple, str] = _TunedTable()
        self._tuned.on_change = self._invalidate_fast
        self._sel_memo: Dict[tuple, tuple] = {}       # select() decisions of repeated call shapes
        self._dm_large = os.environ.get("MP4X_DM_LARGE", "auto")
        self._zc = os.environ.get("MP4X_IPC_ZC", "1") == "1"   # zero-copy two-shot on registered tensors
        self._select_tuned = False
        # which ranks share a node (parallel/hier.py): a job spanning nodes has no global IPC mesh;
        # its allreduce can run node-aware (xGMI inside a node, RCCL across nodes)
        from .hier import node_id
        self.layout = NodeLayout(self.all_gather_object(node_id(self.rank)) if self.p > 1 and coll is None
                                 else ["local"] * self.p)
        if self.layout.multi_node:
            self.ipc_enabled = False
        self._load_shared_tuning(shared=coll is None)      # (keys on the layout's node count)
        self.hier_min_bytes = int(os.environ.get("MP4X_HIER_MIN_BYTES", 1 << 20))
        # the node-aware schedule is opt-in (VERDICT r5 Next #7): one MI355X node is the whole
        # target machine; a multi-node job asks for it with MP4X_HIER=1 (or forces it by name)
        self._hier_auto = os.environ.get("MP4X_HIER", "0") == "1"
        self._hier = None
        self._hier_failed = False
        # fail-stop detector for hung / failed collectives (parallel/watchdog.py)
        from . import watchdog
        self.watchdog = watchdog.CollectiveWatchdog(self) if coll is None and watchdog.enabled() else None

    def _load_shared_tuning(self, shared: bool = True) -> None:
        """``MP4X_TUNE_FILE``, else (``MP4X_TUNE_AUTO=1``) the topology-keyed table of this job's
        topology in ``MP4X_TUNE_DIR`` (parallel/tiers.py): rank 0 reads the table and every rank
        pins RANK 0's copy (shared through the control plane), checked against rank 0's topology
        record (agreed here, used by every later ``_topology`` call).  A file present on one host
        only, or unreadable on one rank, can then never make ranks pin different schedules for the
        same call (which would pair mismatched collectives and hang).  Collective when more than
        one rank."""
        from . import tiers
        table, err = None, None
        path = os.environ.get("MP4X_TUNE_FILE")
        topo = None
        if (self.rank == 0 or not shared) and (path or tiers.auto_enabled()):
            topo = self._topology()            # (the xGMI probe runs only when a table is in play)
            if not path:
                path = tiers.tune_path(topo)
            if path and os.path.exists(path):
                try:
                    import json
                    with open(path) as f:
                        table = json.load(f)
                except Exception as e:   # noqa: BLE001 — a broken table is ignored, not fatal
                    err = str(e)
        if self.p > 1 and shared:      # (injected loopback ranks share one process and file)
            try:
                table, topo = self.all_gather_object((table, topo))[0]
            except Exception as e:   # noqa: BLE001
                LOG.warning("tuning table not shared (%s): none pinned", e)
                return
        if topo is not None:
            self._topo_agreed = topo
        if err:
            LOG.warning("ignoring tuning table %s: %s", path, err)
        if table is None:
            return
        try:
            n = self.load_tuning(table)
            self.tune_loaded = n
            LOG.info("rank %d: %d pinned schedules from rank 0's %s", self.rank, n, path)
        except Exception as e:   # noqa: BLE001 — a foreign table is refused identically on every rank
            self._tuned.clear()
            LOG.warning("ignoring tuning table %s: %s", path, e)

    # ------------------------------------------------------------------ bootstrap
    def _init_pg(self):
        srv = self.comm.server
        key = f"mp4x/tcpstore/{self.backend}"
        timeout = datetime.timedelta(seconds=float(os.environ.get("MP4X_PG_TIMEOUT", 1800)))
        if self.rank == 0:
            host = self.comm.transport.advertise_host
            store = dist.TCPStore(host, 0, self.p, True, timeout=timeout, wait_for_workers=False)
            srv.call("kv_set", key, f"{host}:{store.port}".encode())
        else:
            addr = srv.call("kv_get", key, 600.0).decode()
            host, port = addr.rsplit(":", 1)
            store = dist.TCPStore(host, int(port), self.p, False, timeout=timeout)
        kw = {}
        if self.device.type == "cuda" and self.backend == "nccl":
            kw["device_id"] = self.device       # eager RCCL communicator bound to this GPU
        dist.init_process_group(self.backend, store=store, rank=self.rank, world_size=self.p, timeout=timeout, **kw)
        self._store = store
        self.pg = dist.group.WORLD
        self._owns_pg = True
        LOG.info("rank %d: device communicator up (%s, %s)", self.rank, self.backend, self.device)

    def abort(self):
        """Fail-stop teardown (``ncclCommAbort``): a rank blocked in a collective with a dead
        peer returns instead of hanging.  Called by ``ProcessCommSlave.close(code != 0)``."""
        self._stop_watchdog()
        self._invalidate_fast()
        for name in ("_ipc_obj", "_ipc_large", "_ipc_fp8_big", "_hier"):
            setattr(self, name, None)          # peers may be gone: no synchronising close
        if self._owns_pg and dist.is_initialized():
            try:
                from torch.distributed.distributed_c10d import _abort_process_group
                for c in self._rccl_variants.values():
                    _abort_process_group(c.pg)
                self._rccl_variants = {}
                _abort_process_group(self.pg)
            except Exception:
                try:
                    self.pg.abort()
                except Exception:
                    pass
            self._owns_pg = False

    def _stop_watchdog(self):
        wd = getattr(self, "watchdog", None)
        if wd is not None:
            wd.stop()

    def shutdown(self):
        self._stop_watchdog()
        self._invalidate_fast()
        for name in ("_ipc_obj", "_ipc_large", "_ipc_fp8_big", "_hier"):
            obj = getattr(self, name)
            if obj is not None:
                try:
                    obj.close()
                except Exception:
                    pass
                setattr(self, name, None)
        if self._owns_pg and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass
            self._owns_pg = False

    # ------------------------------------------------------------------ helpers
    def _count(self, name):
        self.stats[name] = self.stats.get(name, 0) + 1

    @staticmethod
    def _flat(t: torch.Tensor) -> torch.Tensor:
        if not t.is_contiguous():
            raise Mp4jException("device collectives need contiguous tensors")
        return t.view(-1)

    def _op(self, operator, t: torch.Tensor) -> Operator:
        if getattr(operator, "is_custom", False):
            return operator
        return for_dtype(operator, dtype_of_torch(t.dtype))

    def rccl_ok(self, op, dtype) -> bool:
        if getattr(op, "is_custom", False):
            return False
        if self.backend in ("gloo", "loopback"):
            return op.code in _RCCL_OPS and dtype not in (torch.bfloat16, torch.float16, torch.int16)
        return op.code in _RCCL_OPS and dtype in _RCCL_DTYPES

    def ipc(self):
        """Lazily set up the IPC peer mappings (collective: every rank reaches this together).

        A new mesh runs :meth:`_ipc_self_test` before any IPC tier is used: on first contact with
        a topology whose peer mappings misbehave, every rank disables IPC together (logged) and
        the job runs on RCCL instead of returning wrong sums."""
        if self._ipc_obj is None and self.ipc_enabled:
            try:
                from .ipc import IpcAllreduce
                inst = IpcAllreduce(self.comm)
                self._adopt(inst)
            except Exception as e:
                # never a silent fall-back: the verdict says why (e.g. the legacy IPC mode) and how
                # to fix it, once, on every rank (setup failures are agreed inside IpcAllreduce)
                from .ipc import ipc_mode_report
                rep = ipc_mode_report(str(e))
                LOG.warning("IPC allreduce disabled: %s%s", e, f" — {rep['reason']}" if rep.get("reason") else "")
                self.ipc_enabled = False
                self.ipc_selftest = {"ok": False, "failures": [f"setup: {str(e)[:300]}"], "ipc_mode": rep}
                return None
            bad = self._ipc_self_test(inst)
            if bad and all(": zero_copy_memalloc" in b for b in bad):
                # only the memAlloc (VMM-imported) region failed: registered caching-allocator
                # tensors keep the zero-copy forms; memAlloc hands out registered plain tensors
                # (up to the IPC open limit) instead of VMM ones (the verdict is agreed)
                LOG.warning("rank %d: IPC memAlloc zero-copy self-test failed (%s): memAlloc falls back to "
                            "registered plain tensors on every rank", self.rank, bad)
                self._zc_vmm = False
                self.ipc_selftest = dict(self.ipc_selftest or {}, zero_copy_memalloc=False)
                bad = None
            elif bad and all(": zero_copy_" in b for b in bad):
                # only the zero-copy forms failed (identically known on every rank: the verdict is
                # agreed): keep the staged kernels, run registered / memAlloc tensors staged
                LOG.warning("rank %d: IPC zero-copy self-test failed (%s): zero-copy forms disabled on every rank, "
                            "staged IPC kernels kept", self.rank, bad)
                self._zc = False
                self.ipc_selftest = dict(self.ipc_selftest or {}, zero_copy=False)
                bad = None
            if bad:
                LOG.warning("rank %d: IPC self-test failed (%s): IPC tiers disabled on every rank, RCCL used",
                            self.rank, bad)
                self._drop_instance(inst)                # agreed: every rank is here
                self.ipc_enabled = False
                self.ipc_selftest = {"ok": False, "failures": bad}
                return None
            self._ipc_obj = inst
            inst.on_change = self._invalidate_fast
            self._invalidate_fast()
            self._probe_spin(inst)
        return self._ipc_obj

    ipc_selftest: Optional[dict] = None
    tune_loaded = 0                       # schedules pinned from a saved table at creation
    order = None                          # (engines assembled without __init__: no stream order)

    def _adopt(self, inst) -> None:
        """A new IPC instance of this communicator joins its stream order before its first launch
        (the self-test and first-use probe included)."""
        if self.order is not None:
            inst.use_order(self.order)

    # ------------------------------------------------------------------ fail-stop at the call boundary
    def _ipc_all(self):
        """Every IPC instance of this engine (None entries skipped)."""
        h = self._hier
        return [i for i in (self._ipc_obj, self._ipc_large, self._ipc_fp8_big,
                            h.ipc if h is not None else None) if i is not None]

    def check_failed(self) -> None:
        """Raise :class:`Mp4jException` if an IPC collective of this rank gave up waiting for a
        peer (its spin bound expired: a peer died, diverged or was later than the fail-stop
        budget).  Reads pinned host words only — no device synchronisation — so it runs at the
        entry of EVERY device collective, in ``barrier()`` and in ``close()``: a result that
        followed a timeout is never consumed silently, whether or not the watchdog runs."""
        for inst in (self._ipc_obj, self._ipc_large, self._ipc_fp8_big):
            if inst is not None:
                inst.raise_if_failed()
        h = self._hier
        if h is not None and h.ipc is not None:
            h.ipc.raise_if_failed()

    def _oneshot_limit(self) -> int:
        """Largest staged allreduce that runs the one-shot (the two-shot above): the latency tier's
        ``ipc_oneshot_max``, or at two ranks the slot size (see __init__)."""
        return max(self.ipc_oneshot_max, self._oneshot_ar_max)

    # ------------------------------------------------------------------ latency fast path
    def _invalidate_fast(self) -> None:
        """Forget every memoised latency-tier launch (any input of the decision changed: the pinned
        table, a tier attribute, a registration, an instance, the epoch mode).  While any tensor is
        registered the memo keys on the buffer address too (an address inside a registered range
        takes the zero-copy kernels instead); with none, one entry serves every buffer of a shape."""
        fa = self.__dict__.get("_fast_ar")
        if fa is None:
            return
        fa.clear()
        if isinstance(fa, _FastMemo):
            inst = self.__dict__.get("_ipc_obj")
            rng = sorted((int(a), int(a) + int(n)) for a, n in (getattr(inst, "_regs", None) or {}))
            fa.reg_starts = [a for a, _ in rng]
            fa.reg_ends = [b for _, b in rng]

    _FAST_MAX = 256

    def _fast_remember(self, arr, frm, to, operator, operand, scale, view, op, algo: str,
                       kind: str = "allreduce") -> None:
        """Memoise the native launch of a call that just took the staged latency tier (one-/two-
        shot on the default instance, one piece, fused copy-in, in place, host epochs), keyed by
        everything that decided it, so the next call of that shape runs ``mp4x_ipc_fast_allreduce``
        from the public API's first lines (ProcessCommSlave.allreduceArray)."""
        fa = self.__dict__.get("_fast_ar")
        inst = self._ipc_obj
        if fa is None or inst is None or inst._epoch_dev is not None or not inst._fuse_copy or \
                self._probe_depth or os.environ.get("MP4X_FAST_PATH", "1") != "1":
            return
        from ..ops import native
        lx = native.launch_ext()
        if lx is None or not hasattr(lx, "fast_allreduce"):
            return
        total = view.numel() * view.element_size()
        ptr = view.data_ptr()
        if total % 16 or ptr % 16 or total > inst.nbytes or total > self.ipc_twoshot_max or \
                not view.is_contiguous() or capturing_now():
            return
        from .ipc import ONESHOT, TWOSHOT
        state = inst.fast_state(self._fast_words())
        if state is None:
            return
        a = ONESHOT if algo == "ipc1" else TWOSHOT
        from ..operators import dtype_of_torch
        base = arr.data_ptr()
        key = (fa.addr_key(base, arr.numel() * arr.element_size()) if isinstance(fa, _FastMemo) else base,
               arr.get_device(), arr.numel(), frm, to, arr.dtype,
               operator, getattr(operand, "codec", None), getattr(operand, "compress", False), scale)
        if kind != "allreduce":
            key = (kind,) + key
        if len(fa) >= self._FAST_MAX:
            fa.clear()
        # the buffer as an offset from the tensor's address: the call passes its tensor's address
        # (an unaligned one is refused natively before anything is launched: the full path runs)
        fa[key] = _ArEntry(state, a, int(dtype_of_torch(view.dtype)), int(op.code), ptr - base, total,
                           inst.latency_blocks(total, a, view.dtype, op), self._fused_scale(scale, view),
                           kind + "." + algo, inst, kind + "Array")

    def _fast_words(self) -> list:
        """The pinned host error words of every IPC instance (the fast paths' fail-stop check)."""
        h = self._hier
        return [i._herr.value for i in (self._ipc_obj, self._ipc_large, self._ipc_fp8_big,
                                        h.ipc if h is not None else None) if i is not None and i._herr]

    def _plan_memo(self, memo: bool, kind: str, arr, key_tail: tuple, fn) -> bool:
        """Run ``fn``, a staged copy-plan form of the default instance (the latency tier of
        broadcast / gather / scatter / all-gather) or its fused reduce-scatter.  With ``memo``
        (the public API's full path), a call that ran exactly ONE host-epoch launch reading /
        writing only ``arr`` is memoised for the API's fast path (``mp4x_ipc_fast_plan`` /
        ``mp4x_ipc_fast_rs``), keyed like the allreduce memo (shape, device; the tensor's address
        only when it overlaps a registered tensor) plus ``key_tail`` (ranges, root).  Anything else (a temporary for an unaligned tensor, several
        launches, device epochs) is not memoised."""
        inst = self._ipc_obj
        fa = self.__dict__.get("_fast_ar")
        if not memo or not isinstance(fa, _FastMemo) or inst is None or self._probe_depth or \
                os.environ.get("MP4X_FAST_PATH", "1") != "1":
            return fn()
        sink = []
        inst._plan_sink = sink
        try:
            ok = fn()
        finally:
            inst._plan_sink = None
        if not ok or len(sink) != 1 or sink[0][-1] is not None or capturing_now():
            return ok
        rec = sink[0]
        src, out = (rec[5], rec[6])
        base = arr.data_ptr()
        end = base + arr.numel() * arr.element_size()
        if any(x is not None and not base <= x < end for x in (src, out)):
            return ok
        from ..ops import native
        lx = native.launch_ext()
        if lx is None or not hasattr(lx, "fast_plan" if rec[0] == "plan" else "fast_rs"):
            return ok
        state = inst.fast_state(self._fast_words())
        if state is None:
            return ok
        key = (kind, fa.addr_key(base, end - base), arr.get_device(), arr.numel(), arr.dtype) + key_tail
        if len(fa) >= self._FAST_MAX:
            fa.clear()
        so, oo = (src - base if src is not None else -1), (out - base if out is not None else -1)
        if rec[0] == "plan":
            _, sa, ns, pa, npl, _, _, grid_len, buf_vecs, blocks, _ = rec
            fa[key] = _PlanEntry(state, ctypes.addressof(sa), ns, ctypes.addressof(pa), npl, so, oo, grid_len,
                                 buf_vecs, blocks, kind + ".ipc", kind + "Array", inst, sa, pa)
        else:                                       # "rs": the fused reduce-scatter
            _, dt, code, lo_a, hi_a, _, _, blocks, _ = rec
            fa[key] = _RsEntry(state, dt, code, ctypes.addressof(lo_a), ctypes.addressof(hi_a), so, oo, blocks,
                               kind + ".ipc", "reduceScatterArray", inst, lo_a, hi_a)
        return ok

    def _probe_spin(self, inst) -> None:
        if self._probe_depth and inst is not None:
            from .ipc import probe_spin
            inst.set_spin(self._probe_s or probe_spin())

    @contextlib.contextmanager
    def probing(self, seconds: Optional[float] = None):
        """Autotune / probe scope: every IPC instance (also ones created inside) uses the short
        probe spin bound (``MP4X_IPC_PROBE_SPIN_S``, or ``seconds``), so a candidate that cannot
        complete on this topology is ruled out in seconds instead of after the fail-stop budget;
        that budget is restored afterwards.  Collective in effect (every rank enters it around
        the same calls)."""
        from .ipc import probe_spin, spin_default
        self._probe_depth += 1
        prev = self._probe_s
        if seconds is not None:
            self._probe_s = float(seconds)
        try:
            if self._probe_depth == 1 or seconds is not None:
                for inst in self._ipc_all():
                    inst.set_spin(self._probe_s or probe_spin())
            yield
        finally:
            self._probe_depth -= 1
            self._probe_s = prev
            restore = spin_default() if self._probe_depth == 0 else (self._probe_s or probe_spin())
            if self._probe_depth == 0 or seconds is not None:
                for inst in self._ipc_all():
                    try:
                        inst.set_spin(restore)
                    except Exception as e:   # noqa: BLE001 — a dead mesh is reported by the next call
                        LOG.warning("rank %d: could not restore the IPC spin bound: %s", self.rank, e)

    def _ipc_self_test(self, inst) -> Optional[list]:
        """Collective exact-pattern test of every IPC kernel family on the fresh mesh (f32 SUM):
        one-shot 64 KiB, two-shot 64 KiB and 4 MiB, direct reduce-scatter / all-gather 4 MiB, a
        copy-plan broadcast, and the zero-copy two-shot on a registered 4 MiB tensor.  Short
        barrier spin bound (``MP4X_IPC_SELFTEST_SPIN_S``, 2 s) while it runs.  The verdict is the
        union of every rank's failures (agreed through the control plane, not through the
        transport under test).  Returns None when everything was exact on every rank."""
        if os.environ.get("MP4X_IPC_SELFTEST", "1") == "0":
            return None
        from . import ipc as ipcm
        from ..operators import Operators
        t0 = time.perf_counter()
        fails = []
        try:
            inst.set_spin(float(os.environ.get("MP4X_IPC_SELFTEST_SPIN_S", "2")))
        except Exception as e:   # noqa: BLE001
            fails.append(f"set_spin: {e}")
        dev = self.device
        p, r = self.p, self.rank
        op = for_dtype(Operators.Float.SUM, DType.F32)
        cap = inst.nbytes // 4

        def pattern(n):
            t = torch.empty(n, dtype=torch.float32, device=dev)
            exp = self._fill_probe(t, op)
            return t, exp

        def step(name, fn):
            try:
                bad = fn()
                torch.cuda.synchronize(dev)
                code = inst.host_error()
                inst.raise_if_failed()
                nbad = 0 if code else bad()
                if code:
                    fails.append(f"{name}: barrier timeout {code}")
                elif nbad:
                    fails.append(f"{name}: {nbad} wrong elements")
            except Exception as e:   # noqa: BLE001
                fails.append(f"{name}: {type(e).__name__}: {e}")
                try:
                    torch.cuda.synchronize(dev)
                    inst.raise_if_failed()
                except Exception:   # noqa: BLE001
                    pass

        def allreduce_case(n, algo):
            def fn():
                t, exp = pattern(n)
                inst.allreduce(t, op, algo=algo)
                return lambda: int((t != exp).sum())
            return fn

        n64k, n4m = min(cap, 16 << 10), min(cap, 1 << 20)
        step("oneshot_64KiB", allreduce_case(n64k, ipcm.ONESHOT))
        step("twoshot_64KiB", allreduce_case(n64k, ipcm.TWOSHOT))
        step("twoshot_4MiB", allreduce_case(n4m, ipcm.TWOSHOT))

        froms, tos, _ = CommUtils.even_split(0, n4m, p)
        a16 = all((f * 4) % 16 == 0 for f in froms + tos)

        def rs():
            t, exp = pattern(n4m)
            if not inst.reduce_scatter(t, froms, tos, op):
                return lambda: 0
            return lambda: int((t[froms[r]:tos[r]] != exp[froms[r]:tos[r]]).sum())

        def ag():
            t = torch.full((n4m,), -1.0, device=dev)
            exp = torch.arange(n4m, device=dev, dtype=torch.float32).remainder_(251)
            t[froms[r]:tos[r]] = exp[froms[r]:tos[r]]
            if not inst.allgather(t, froms, tos):
                return lambda: 0
            return lambda: int((t != exp).sum())

        def bcast():
            n = min(cap, 1 << 18)
            exp = torch.arange(n, device=dev, dtype=torch.float32).remainder_(113)
            t = exp.clone() if r == p - 1 else torch.zeros(n, device=dev)
            if not inst.broadcast(t, 0, n, p - 1):
                return lambda: 0
            return lambda: int((t != exp).sum())

        if a16:
            step("reduce_scatter_4MiB", rs)
            step("allgather_4MiB", ag)
        step("broadcast_1MiB", bcast)
        if self._zc:
            # on a dedicated plain allocation (a tensor from the caching allocator may sit in a
            # segment too large to map, see ipc.IPC_OPEN_MAX).  The memAlloc (VMM-imported) region
            # is checked at the first memAlloc instead (_memalloc_self_test): a job that never
            # calls it never maps a VMM import across GPUs (first contact keeps to hipIpc).
            for name, fn in (("zero_copy_twoshot_and_plans_4MiB", lambda: inst.selftest_zero_copy(n4m)),):
                try:
                    nbad = fn()
                    if nbad:
                        fails.append(f"{name}: {'setup failed' if nbad < 0 else f'{nbad} wrong elements'}")
                    torch.cuda.synchronize(dev)
                    code = inst.host_error()
                    inst.raise_if_failed()
                    if code:
                        fails.append(f"{name}: barrier timeout {code}")
                except Exception as e:   # noqa: BLE001
                    fails.append(f"{name}: {type(e).__name__}: {e}")
        try:
            inst.set_spin(ipcm.spin_default())     # normal operation: the fail-stop budget
        except Exception as e:   # noqa: BLE001
            fails.append(f"set_spin: {e}")
        if os.environ.get("MP4X_IPC_SELFTEST_INJECT", "").strip() == str(r):   # failure-path tests
            fails.append("injected failure (MP4X_IPC_SELFTEST_INJECT)")
        allf = self.comm.server.call("allgather_obj", self.rank, fails)
        bad = [f"rank {i}: {x}" for i, fl in enumerate(allf) for x in (fl or [])]
        from .ipc import ipc_mode_report
        self.ipc_selftest = {"ok": not bad, "failures": bad, "seconds": round(time.perf_counter() - t0, 3),
                             "ipc_mode": ipc_mode_report()}
        if not bad:
            LOG.info("rank %d: IPC self-test passed in %.3f s", self.rank, self.ipc_selftest["seconds"])
        return bad or None

    RCCL_CTA_VARIANTS = (64, 112)

    def rccl_variant(self, ctas: int):
        """TorchColl over a second RCCL communicator created with ncclConfig minCTAs = maxCTAs =
        ``ctas`` (channels).  RCCL's default channel count is a heuristic; on a full xGMI mesh more
        channels can put more links and CUs on a large message, so autotune measures these
        communicators side by side with the default one.  Collective, lazily created."""
        c = self._rccl_variants.get(ctas)
        if c is None:
            from .coll import TorchColl
            opts = dist.ProcessGroupNCCL.Options()
            opts.config.min_ctas = ctas
            opts.config.max_ctas = ctas
            pg = dist.new_group(ranks=list(range(self.p)), backend="nccl", pg_options=opts)
            c = self._rccl_variants[ctas] = TorchColl(pg, self.backend)
            c.order = self.order           # the same communicator order as the default RCCL calls
        return c

    def ipc_large(self):
        """Second IPC instance with a large buffer (``MP4X_IPC_LARGE_BYTES``, default 256 MiB)
        for messages above the two-shot tier, when autotuning (or ``MP4X_DEVICE_ALGO=ipc2``)
        routes them to IPC.  Collective, lazily created."""
        if self._ipc_large is None and not self._ipc_large_failed and self.ipc() is not None:
            try:
                from .ipc import IpcAllreduce
                inst = IpcAllreduce(self.comm, nbytes=int(os.environ.get("MP4X_IPC_LARGE_BYTES", 256 << 20)),
                                    tag="large", slots=False)
                self._adopt(inst)
            except Exception as e:
                LOG.warning("large-message IPC allreduce disabled: %s", e)
                self._ipc_large_failed = True
                return self._ipc_obj
            # first use of a fresh mesh: every form this instance serves, exact, agreed
            bad = self._probe_instance(inst, large_forms=True) \
                if os.environ.get("MP4X_TEST_SKIP_FIRST_USE_PROBE", "0") != "1" else []
            if bad:
                LOG.warning("rank %d: large-message IPC instance failed its first-use probe (%s): dropped on "
                            "every rank, the default instance serves those calls", self.rank, bad)
                self._drop_instance(inst)
                self._ipc_large_failed = True
                self.probe_failures.append({"instance": "large", "failures": bad})
                return self._ipc_obj
            self._ipc_large = inst
            inst.on_change = self._invalidate_fast
            self._invalidate_fast()                # its error word joins the fast path's check
            self._probe_spin(inst)
            if self._ipc_obj is not None and self._ipc_obj._epoch_dev is not None:
                inst.prepare_graph()   # a capture is being prepared: same epoch mode
        return self._ipc_large or self._ipc_obj

    probe_failures: list = []      # (class default; the engine's own list is made in __init__)

    def _drop_instance(self, inst) -> None:
        """Collective: close an IPC instance every rank agreed to drop (ordered: every importer
        unmaps before any owner frees, ``IpcAllreduce.close(collective=True)``)."""
        try:
            inst.close(collective=True)
        except Exception as e:   # noqa: BLE001 — a teardown error must not hide the fallback
            LOG.warning("rank %d: closing a dropped IPC instance: %s", self.rank, e)

    def hier(self):
        """The node-aware allreduce (parallel/hier.py) of a job spanning >= 2 nodes of equal size,
        or None.  Collective, lazily created; a setup failure is agreed (every rank gets None)."""
        if self._hier is None and not self._hier_failed and self.layout.hier_ok():
            self._invalidate_fast()
            from .hier import HierAllreduce
            try:
                self._hier = HierAllreduce(self, self.layout)
            except Exception as e:   # noqa: BLE001
                LOG.warning("rank %d: hierarchical allreduce disabled: %s", self.rank, e)
                self._hier_failed = True
            ok = self.all_gather_object(self._hier is not None)
            if not all(ok):
                if self._hier is not None:
                    self._hier.close()
                self._hier, self._hier_failed = None, True
        return self._hier

    def _hier_ok(self, op, dtype, nbytes) -> bool:
        """Rank-independent: a multi-node layout and an (op, dtype, size) the schedule serves."""
        if not self.layout.hier_ok() or self._hier_failed or nbytes % 16 or getattr(op, "is_custom", False):
            return False
        if dtype not in _ipc_dtypes() or not self.rccl_ok(op, dtype):
            return False
        return op.code == OpCode.SUM or (op.code in (OpCode.MAX, OpCode.MIN) and dtype.is_floating_point)

    def _ipc_ok(self, op, dtype, nbytes) -> bool:
        """The IPC kernels reduce (op, dtype): every operator of the reference's table (see
        ``ipc.ipc_op_ok``), on 16-byte multiples, with IPC enabled."""
        if not self.ipc_enabled or nbytes % 16 or op is None:
            return False
        return _ipc_op_ok(dtype, op)

    _SEL_MEMO_MAX = 512

    def select(self, kind: str, nbytes: int, op, dtype, operand=None) -> str:
        """Per-call algorithm choice (size tiers, dtype/op support, MP4X_DEVICE_ALGO override).

        Memoised per call shape: the decision is a pure function of the key below (the forced
        algorithm, the pinned table's mutation count, the IPC / hierarchical state and the tier
        thresholds are part of it), so a repeated small collective skips the tier logic — on
        the latency tier every microsecond of host time is a microsecond of latency."""
        gen = getattr(self._tuned, "gen", None)
        memo = getattr(self, "_sel_memo", None)
        if gen is None or memo is None:
            return self._select(kind, nbytes, op, dtype, operand)
        # the tier state (every attribute _select reads: _TIER_ATTRS) enters as ONE version number
        # that any assignment to those attributes bumps — hashing them all per call cost ~1 us
        key = (kind, nbytes, op, dtype, getattr(operand, "codec", None), getattr(operand, "compress", False),
               gen, self._state_ver)
        try:
            hit = memo.get(key)
        except TypeError:       # an unhashable custom operator: no memo
            return self._select(kind, nbytes, op, dtype, operand)
        if hit is not None:
            self._select_tuned = hit[1]
            return hit[0]
        algo = self._select(kind, nbytes, op, dtype, operand)
        if len(memo) >= self._SEL_MEMO_MAX:
            memo.clear()
        memo[key] = (algo, self._select_tuned)
        return algo

    def _select(self, kind: str, nbytes: int, op, dtype, operand=None) -> str:
        forced = self.algo
        codec = getattr(operand, "codec", None) if operand is not None else None
        if codec in ("fp8", "bf16") and kind == "allreduce" and \
                dtype in ((torch.float32, torch.bfloat16, torch.float16) if codec == "fp8" else (torch.float32,)) \
                and op is not None and not getattr(op, "is_custom", False) and op.code == OpCode.SUM \
                and self.device.type == "cuda":
            return codec
        if kind == "allreduce" and op is not None and not getattr(op, "is_custom", False) and \
                (codec == "zs" or (codec is None and getattr(operand, "compress", False))):
            return "zs"       # lossless wire compression (the reference's compress=true contract)
        if zc_grid(forced)[0] in ("ipc1", "ipc2", "ipc2p", "ipc2z", "ipc2w") and kind == "allreduce" and \
                self._ipc_ok(op, dtype, nbytes):
            return forced
        if forced == "rhd" and kind == "allreduce" and not getattr(op, "is_custom", False):
            return forced     # (custom operators may be non-commutative: rank-ordered a2a only)
        if forced == "hier" and kind == "allreduce" and op is not None and self._hier_ok(op, dtype, nbytes):
            return forced
        self._select_tuned = False
        if kind == "allreduce" and op is not None and forced in ("", "auto") and self._tuned:
            tt = self._tuned
            t = tt.pinned(_tune_key(dtype, op, nbytes)) if hasattr(tt, "pinned") else tt.get(_tune_key(dtype, op, nbytes))
            if t is not None and self._algo_valid(t, op, dtype, nbytes):
                self._select_tuned = True
                return t
        if op is not None and not self.rccl_ok(op, dtype):
            # RCCL cannot reduce it (bitwise, *_LOC, int16, ...): the IPC kernels run every
            # operator of the table in one fused kernel per call; a2a only without a mesh
            if kind in ("allreduce", "reduce") and forced in ("", "auto") and self._ipc_ok(op, dtype, nbytes) \
                    and self.device.type == "cuda":
                return "ipc1" if kind == "allreduce" and nbytes <= self._oneshot_limit() else "ipc2"
            return "a2a"
        if forced in ("", "auto") and kind == "allreduce" and nbytes >= self.hier_min_bytes and self._hier_auto and \
                self._hier_ok(op, dtype, nbytes):
            return "hier"     # several nodes: xGMI inside each, RCCL on 1/L of the bytes across
        if forced in ("rccl", "a2a"):
            return forced
        if forced.startswith("rccl_c") and kind == "allreduce" and op is not None \
                and self._algo_valid(forced, op, dtype, nbytes):
            return forced
        if kind == "allreduce" and self._ipc_ok(op, dtype, nbytes):
            if nbytes <= self._oneshot_limit():
                return "ipc1"
            if nbytes <= self.ipc_twoshot_max or (self.backend != "nccl" and self.device.type == "cuda"
                                                  and self._dm_large != "rccl"):
                return "ipc2"     # (no RCCL underneath: the IPC two-shot takes every size)
        if self.a2a_bytes and nbytes >= self.a2a_bytes:
            return "a2a"
        return "rccl"

    # ------------------------------------------------------------------ hipGraph capture
    _CAPTURABLE = ("rccl", "ipc1", "ipc2", "ipc2z", "ipc2w", "a2a", "rhd", "fp8", "bf16")

    def capture(self, fn, warmup: int = 2):
        """Capture ``fn()`` — a fixed sequence of device collectives on fixed tensors, e.g. a DDP
        step's bucket allreduces — into one hipGraph and return the ``torch.cuda.CUDAGraph``;
        ``graph.replay()`` then re-issues every kernel and RCCL call with no host launch cost.

        Collective: every rank captures the same sequence.  The IPC instances switch to device
        epochs first (``IpcAllreduce.prepare_graph``) so replays never reuse a flag value, and
        while capturing ``select`` keeps to schedules without host synchronisation (no zs /
        pipelined pieces / sparse)."""
        if self.device.type != "cuda":
            raise Mp4jException("capture needs a GPU device engine")
        self._invalidate_fast()
        for inst in (self.ipc(), self._ipc_large, self._ipc_fp8_big):
            if inst is not None:
                inst.prepare_graph()
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream(self.device).wait_stream(side)
        self._sync()
        # the warm-up may have created the large-message instance: it needs device epochs too
        for inst in (self._ipc_obj, self._ipc_large, self._ipc_fp8_big):
            if inst is not None:
                inst.prepare_graph()
        self.barrier()
        g = torch.cuda.CUDAGraph()
        wd = self.watchdog
        if wd is not None:
            wd.quiet += 1        # no device polls from the watchdog thread during the capture
        try:
            with torch.cuda.graph(g, stream=side):
                fn()
        finally:
            if wd is not None:
                wd.quiet -= 1
        self._sync()
        return g

    def local_reduce(self, out: torch.Tensor, inputs: Sequence[torch.Tensor], f: int, t: int, operator):
        return local_reduce(out, inputs, f, t, operator)

    def _reduce_into(self, out: torch.Tensor, ins: Sequence[torch.Tensor], op) -> None:
        reduce_into(out, ins, op)

    # ================================================================== allreduce
    def allreduce(self, arr: torch.Tensor, frm: int, to: int, operator, operand=None, small: bool = False,
                  out: Optional[torch.Tensor] = None, scale: float = 1.0, memo: bool = False):
        """In-place allreduce of ``arr[frm:to]``; with ``out`` the result goes to ``out[frm:to]``
        and ``arr`` is left untouched (the staged IPC kernels write ``out`` directly; other
        schedules copy into ``out`` first and run in place there).

        ``scale`` (float dtypes): the result is multiplied by it — the 1/p average of a DP
        gradient sync fused into the collective's own final write (IPC kernels, fp8 requantise)
        or RCCL's ncclAvg, instead of a separate pass over the buffer.

        ``memo`` (the public API's full path): memoise this call shape's native launch when it took
        the staged latency tier, for ProcessCommSlave.allreduceArray's fast path."""
        if frm == 0 and arr.dim() == 1 and to == arr.shape[0] and arr.is_contiguous():
            view = arr                    # the whole 1-D tensor: no view objects on the latency tier
        else:
            view = self._flat(arr)[frm:to]
        if scale != 1.0 and not view.is_floating_point():
            raise Mp4jException("allreduce scale= needs a floating-point tensor")
        if out is not None:
            oview = self._flat(out)[frm:to]
            if view.numel() == 0:
                return out
        if view.numel() == 0:
            return arr
        op = self._op(operator, view)
        nbytes = view.numel() * view.element_size()
        algo = self.select("allreduce", nbytes, op, view.dtype, operand)
        capturing = view.is_cuda and capturing_now()
        if zc_grid(algo)[0] not in self._CAPTURABLE and capturing:
            # host-synchronising schedule inside a hipGraph capture: use a capturable twin
            algo = "ipc2" if algo == "ipc2p" else ("rccl" if self.rccl_ok(op, view.dtype) else "a2a")
        if out is not None:
            if algo in ("ipc1", "ipc2") and self.ipc() is not None and nbytes <= self.ipc_twoshot_max and \
                    (not capturing or self._ipc_obj._epoch_dev is not None):
                from .ipc import ONESHOT, TWOSHOT
                self._count("allreduce." + algo + ".out")
                self._ipc_obj.allreduce(view, op, algo=ONESHOT if algo == "ipc1" else TWOSHOT, out=oview,
                                        scale=self._fused_scale(scale, view))
                self._post_scale(oview, scale, fused=True)
                return out
            if view.is_cuda:   # the local copy runs through the K1 kernel (NIN = 1)
                from ..ops.device_ops import reduce_
                reduce_(oview, [view], int(OpCode.SUM))
            else:
                oview.copy_(view)
            view, arr = oview, out
        if (algo == "ipc2" or (algo == "ipc1" and nbytes > self.ipc_oneshot_max)) and not self._select_tuned \
                and self._zc and self._ipc_obj is not None and self._ipc_obj.registered(view) is not None:
            # registered on this rank (registration is collective): zero-copy above the latency
            # tier (also where two ranks would stage into the one-shot's slots)
            algo = "ipc2z"
        self._count("allreduce." + algo)
        fused = self._run_allreduce(algo, view, op, scale=self._fused_scale(scale, view), capturing=capturing)
        self._post_scale(view, scale, fused)
        if memo and (algo == "ipc1" or algo == "ipc2") and out is None and not capturing and \
                self._fast_ar is not None and view.is_cuda:
            self._fast_remember(arr, frm, to, operator, operand, scale, view, op, algo)
        return arr

    @staticmethod
    def _fused_scale(scale: float, view: torch.Tensor) -> float:
        return float(scale) if view.dtype in (torch.float32, torch.float64, torch.bfloat16, torch.float16) else 1.0

    def _post_scale(self, view: torch.Tensor, scale: float, fused: bool) -> None:
        """The scale a schedule could not fuse: one K1 scale pass (device) / in-place multiply."""
        if scale == 1.0 or (fused and self._fused_scale(scale, view) == scale):
            return
        if view.is_cuda and view.dtype in (torch.float32, torch.float64, torch.bfloat16, torch.float16):
            from ..ops.device_ops import scale_
            scale_(view, view, float(scale))
        else:
            view.mul_(scale)

    # ------------------------------------------------------------------ registered buffers
    def register_buffer(self, t: torch.Tensor) -> bool:
        """Collective: map ``t`` into every peer for the zero-copy two-shot allreduce (no staging
        copy, no pieces, any size).  Every rank registers its same-shaped tensor at the same
        point and keeps it (and its allocation) alive until :meth:`deregister_buffer`.  Returns
        True when the mesh accepted it on every rank; False (every rank) leaves the staged path."""
        if not self._zc or self.p < 2 or self.ipc() is None:
            return False
        return self._ipc_obj.register(self._flat(t))

    def deregister_buffer(self, t: torch.Tensor) -> None:
        if self._ipc_obj is not None:
            self._ipc_obj.deregister(self._flat(t))

    _memalloc_checked = False

    def _memalloc_self_test(self) -> None:
        """Collective, once, at the first memAlloc: the VMM-imported region through the zero-copy
        two-shot, pull and push, twice on the same memory, in two alloc / free cycles
        (``IpcAllreduce.selftest_memalloc``), exact, agreed.  On failure memAlloc hands out
        registered plain tensors on every rank (``_zc_vmm`` False); the zero-copy forms on
        registered tensors stay.  ``MP4X_IPC_SELFTEST_INJECT_MEMALLOC=<rank>`` rehearses it."""
        self._memalloc_checked = True
        inst = self._ipc_obj
        fails = []
        try:
            inst.set_spin(float(os.environ.get("MP4X_IPC_SELFTEST_SPIN_S", "2")))
            nbad = inst.selftest_memalloc(min(inst.nbytes // 4, 1 << 18))
            if nbad:
                fails.append(f"zero_copy_memalloc_1MiB: {'setup failed' if nbad < 0 else f'{nbad} wrong elements'}")
            torch.cuda.synchronize(self.device)
            code = inst.host_error()
            inst.raise_if_failed()
            if code:
                fails.append(f"zero_copy_memalloc_1MiB: barrier timeout {code}")
        except Exception as e:   # noqa: BLE001
            fails.append(f"zero_copy_memalloc_1MiB: {type(e).__name__}: {e}")
            try:                       # a timed-out kernel of the test must not fail the next call
                torch.cuda.synchronize(self.device)
                inst.raise_if_failed()
            except Exception:   # noqa: BLE001
                pass
        try:
            from .ipc import probe_spin, spin_default
            inst.set_spin(probe_spin() if self._probe_depth else spin_default())
        except Exception as e:   # noqa: BLE001
            fails.append(f"set_spin: {e}")
        if os.environ.get("MP4X_IPC_SELFTEST_INJECT_MEMALLOC", "").strip() == str(self.rank):
            fails.append("zero_copy_memalloc_1MiB: injected failure (MP4X_IPC_SELFTEST_INJECT_MEMALLOC)")
        allf = self.comm.server.call("allgather_obj", self.rank, fails)
        bad = [f"rank {i}: {x}" for i, fl in enumerate(allf) for x in (fl or [])]
        self.ipc_selftest = dict(self.ipc_selftest or {}, zero_copy_memalloc=not bad)
        if bad:
            LOG.warning("rank %d: IPC memAlloc zero-copy self-test failed (%s): memAlloc falls back to "
                        "registered plain tensors on every rank", self.rank, bad)
            self._zc_vmm = False
            self.ipc_selftest["memalloc_failures"] = bad

    def mem_alloc(self, n: int, dtype: torch.dtype) -> Optional[torch.Tensor]:
        """Collective: an ``n``-element tensor mapped into every peer at any size (see
        ``IpcAllreduce.mem_alloc``), or None on every rank when there is no IPC mesh (the
        caller then allocates a plain tensor: the staged kernels / RCCL serve it).  When only
        the memAlloc self-test failed on this topology, a plain tensor registered with the peers
        (hipIpc, up to the IPC open limit) stands in for the VMM one."""
        if self.p < 2 or self.device.type != "cuda" or self.ipc() is None or not self._zc:
            return None
        if not self._memalloc_checked and self._zc_vmm and os.environ.get("MP4X_IPC_SELFTEST", "1") != "0":
            self._memalloc_self_test()
        es = torch.empty((), dtype=dtype).element_size()
        if not self._zc_vmm:
            from .ipc import IPC_OPEN_MAX
            if n * es > IPC_OPEN_MAX:
                return None
            t = torch.empty(n, dtype=dtype, device=self.device)
            self._ipc_obj.register(self._flat(t))         # collective; False = staged, still correct
            return t
        return self._ipc_obj.mem_alloc(n * es, dtype)

    def mem_free(self, t: torch.Tensor) -> None:
        if self._ipc_obj is None:
            return
        reg = self._ipc_obj._find(t)[0]
        if reg is not None and reg.vmm:
            self._ipc_obj.mem_free(t)
        elif reg is not None and not self._zc_vmm:
            self._ipc_obj.deregister(self._flat(t))      # the registered stand-in of mem_alloc

    def _run_allreduce(self, algo: str, view: torch.Tensor, op, scale: float = 1.0,
                       capturing: Optional[bool] = None) -> bool:
        """Run schedule ``algo``; returns True when ``scale`` was applied inside it (fused).
        ``capturing``: whether a hipGraph capture is in progress, when the caller knows."""
        if algo == "ipc1" or algo == "ipc2":
            # the latency tier first: a staged one-/two-shot on the default instance, not capturing
            inst = self._ipc_obj
            if capturing is None:
                capturing = capturing_now()
            if inst is not None and not capturing and view.numel() * view.element_size() <= self.ipc_twoshot_max:
                inst.allreduce(view, op, algo=0 if algo == "ipc1" else 1, scale=scale, capturing=False)
                return True
        algo, grid = zc_grid(algo)
        if algo in ("ipc1", "ipc2", "ipc2p", "ipc2z", "ipc2w") and self.ipc() is None:
            algo = "rccl" if self.rccl_ok(op, view.dtype) else "a2a"
        if algo in ("ipc2z", "ipc2w"):
            peers = self._ipc_obj.registered(view) if self._zc else None
            if peers is not None and (not capturing_now() or self._ipc_obj._epoch_dev is not None):
                scr = self._ipc_obj.scratch_of(view) if algo == "ipc2w" else None
                if scr is not None:     # posted remote writes only (push form)
                    self._ipc_obj.allreduce_push(view, op, peers, scr, scale=scale)
                else:
                    self._ipc_obj.allreduce_registered(view, op, peers, scale=scale, grid=grid)
                return True
            algo = "ipc2"        # not registered (on this rank): the staged two-shot
        if algo in ("ipc1", "ipc2", "ipc2p") and capturing_now():
            nb = view.numel() * view.element_size()
            inst = self.ipc_large() if nb > self.ipc_twoshot_max else self._ipc_obj
            if inst is None or inst._epoch_dev is None:
                algo = "rccl" if self.rccl_ok(op, view.dtype) else "a2a"
        if algo == "hier":
            h = self.hier()
            if h is not None and h.supports(view, op):
                h.allreduce(view, op, scale=scale)
                return True
            algo = "rccl" if self.rccl_ok(op, view.dtype) else "a2a"
        if algo == "rccl":
            avg = scale != 1.0 and abs(scale * self.p - 1.0) < 1e-9 and op.code == OpCode.SUM \
                and self.backend == "nccl"
            self.coll.all_reduce(view, op.code, avg=avg)          # ncclAvg: RCCL's fused average
            return avg
        elif algo.startswith("rccl_c"):
            self.rccl_variant(int(algo[6:])).all_reduce(view, op.code)
        elif algo in ("ipc1", "ipc2", "ipc2p"):
            from .ipc import ONESHOT, TWOSHOT
            nbytes = view.numel() * view.element_size()
            inst = self.ipc_large() if nbytes > self.ipc_twoshot_max else self._ipc_obj
            inst.allreduce(view, op, algo=ONESHOT if algo == "ipc1" else TWOSHOT,
                           overlap=True if algo == "ipc2p" else None, scale=scale)
            return True
        elif algo == "rhd":
            self._allreduce_rhd(view, op)
        elif algo == "zs":
            self._allreduce_zs(view, op)
        elif algo == "fp8":
            inst = self._ipc_fp8(view)
            if inst is not None:
                self._count("allreduce.fp8.ipc")
                inst.allreduce_fp8(view, scale=scale)   # fused quant-on-the-links two-shot over xGMI
                return True
            self._allreduce_fp8(view)
        elif algo == "bf16":
            # 2x-compressed wire: bf16 all-to-all, f32 accumulation inside the K1 kernel
            # (bf16 inputs, one rounding), bf16 all-gather, widened back in place
            w = view.to(torch.bfloat16)
            self._allreduce_a2a(w, for_dtype(op, DType.BF16))
            view.copy_(w)
        else:
            self._allreduce_a2a(view, op)
        return False

    def _ipc_fp8(self, view: torch.Tensor):
        """The IPC instance that runs the fused fp8 two-shot for ``view``, or None (RCCL form).
        ``MP4X_FP8_TRANSPORT``: auto (IPC when available) | ipc | rccl."""
        mode = os.environ.get("MP4X_FP8_TRANSPORT", "auto").lower()
        if mode == "rccl" or not self.ipc_enabled or view.device.type != "cuda":
            return None
        if self.ipc() is None or not self._ipc_obj.fp8_ok(view):
            return None
        need = view.numel() * 260 // 256 + (64 << 10)          # e4m3 bytes + scales of the whole tensor
        capturing = torch.cuda.is_current_stream_capturing()
        if need <= self._ipc_obj.nbytes:
            inst = self._ipc_obj
        elif capturing or os.environ.get("MP4X_FP8_ONE_PIECE", "1") != "1":
            inst = self.ipc_large()
        else:
            inst = self._ipc_fp8_whole(need)
        if capturing and (inst is None or inst._epoch_dev is None):
            return None
        return inst

    def _ipc_fp8_whole(self, need: int):
        """An IPC instance whose staging buffer holds a whole fp8-quantised tensor, so the fused
        fp8 two-shot runs as ONE piece at any size (BASELINE config 5: 8 GB of f32 -> ~2 GB of
        e4m3 + scales, above the IPC open limit: a VMM-built buffer, ``IpcAllreduce._vmm_data``).
        Grown on demand (collective: every rank asks for the same size at the same call), kept."""
        inst = self._ipc_fp8_big
        if inst is not None and inst.nbytes >= need:
            return inst
        if self._ipc_fp8_big_failed:
            return self.ipc_large()
        try:
            if inst is not None:
                self._ipc_fp8_big = None
                inst.close(collective=True)       # re-grow mid-job: ordered, every rank here
            from .ipc import IpcAllreduce
            inst = IpcAllreduce(self.comm, nbytes=-(-need // (2 << 20)) * (2 << 20), tag="fp8", slots=False)
            self._adopt(inst)
            bad = self._probe_instance(inst, large_forms=False, fp8=True)
            if bad:
                self._drop_instance(inst)
                self.probe_failures.append({"instance": "fp8", "failures": bad})
                raise Mp4jException(f"first-use probe failed: {bad}")
            self._probe_spin(inst)
            if self._ipc_obj is not None and self._ipc_obj._epoch_dev is not None:
                inst.prepare_graph()
        except Exception as e:   # noqa: BLE001 — setup failures are agreed inside IpcAllreduce
            LOG.warning("whole-tensor fp8 IPC buffer disabled: %s", e)
            self._ipc_fp8_big_failed = True
            self._ipc_fp8_big = None
            return self.ipc_large()
        self._ipc_fp8_big = inst
        inst.on_change = self._invalidate_fast
        self._invalidate_fast()
        return inst

    def _probe_instance(self, inst, large_forms: bool = False, fp8: bool = False) -> list:
        """Collective first-use check of a NEW IPC instance (lazily created instances
        were never verified; a mesh built after a bad teardown read and wrote the wrong memory).
        Exact patterns, short spin bound, nothing else in flight:

        * the staged two-shot twice on the same tensor (the second call reduces the first call's
          result, so a stale line on either side of a link shows as a wrong element);
        * ``large_forms`` (the large-message instance): the piecewise broadcast / scatter /
          gather copy plans and reduce-scatter / all-gather, the forms the rooted and RS / AG
          schedules send to it;
        * ``fp8``: the fused fp8 two-shot within its codec bound (garbage, not rounding, fails).

        Returns every rank's failures, agreed through the control plane (empty = fine).
        ``MP4X_IPC_PROBE_INJECT=<rank>`` injects a failure on that rank (failure-path tests)."""
        from . import ipc as ipcm
        from ..operators import Operators
        fails = []
        p, r = self.p, self.rank
        try:
            inst.set_spin(float(os.environ.get("MP4X_IPC_SELFTEST_SPIN_S", "2")))
            op = for_dtype(Operators.Float.SUM, DType.F32)
            n = min(inst.nbytes // 4, 1 << 20)
            n -= n % (4 * p)                                # 16-byte segments for every rank
            t = torch.empty(n, dtype=torch.float32, device=self.device)

            def check(name, bad_fn):
                torch.cuda.synchronize(self.device)
                inst.raise_if_failed()
                nbad = int(bad_fn())
                if nbad:
                    fails.append(f"{name}: {nbad} wrong elements")

            exp = self._fill_probe(t, op)
            for rep in range(2):
                inst.allreduce(t, op, algo=ipcm.TWOSHOT)
                check(f"staged_twoshot_{rep}", lambda: (t != exp * (p ** rep)).sum())
            if large_forms:
                root = p - 1
                froms, tos, _ = CommUtils.even_split(0, n, p)
                segs = [(froms[j], tos[j], j) for j in range(p)]
                mine = slice(froms[r], tos[r])
                ex = self._copy_probe(t, [(0, n, root)])
                t.copy_(ex) if r == root else t.fill_(-1)
                inst.broadcast_large(t, 0, n, root)
                check("broadcast_large", lambda: (t != ex).sum())
                ex = self._copy_probe(t, segs)
                t.copy_(ex) if r == root else t.fill_(-1)
                inst.scatter_large(t, froms, tos, root)
                check("scatter_large", lambda: (t[mine] != ex[mine]).sum())
                t.fill_(-1)
                t[mine] = ex[mine]
                inst.gather_large(t, froms, tos, root)
                check("gather_large", lambda: (t != ex).sum() if r == root else 0)
                exp = self._fill_probe(t, op, salt=3)
                inst.reduce_scatter_large(t, froms, tos, op)
                check("reduce_scatter_large", lambda: (t[mine] != exp[mine]).sum())
                inst.allgather_large(t, froms, tos)
                check("allgather_large", lambda: (t != exp).sum())
            if fp8 and inst.fp8_ok(t):
                exp = self._fill_probe(t, op, salt=5)
                inst.allreduce_fp8(t)
                tol = 0.25 * float(exp.abs().max())
                check("fp8_twoshot", lambda: ((t - exp).abs() > tol).sum())
            del t
            inst.set_spin(ipcm.spin_default())
        except Exception as e:   # noqa: BLE001
            fails.append(f"{type(e).__name__}: {e}")
        if os.environ.get("MP4X_IPC_PROBE_INJECT", "").strip() == str(r):
            fails.append("injected failure (MP4X_IPC_PROBE_INJECT)")
        allf = self.comm.server.call("allgather_obj", self.rank, fails)
        return [f"rank {i}: {x}" for i, fl in enumerate(allf) for x in (fl or [])]

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    # ================================================================== reduce-scatter
    def reduce_scatter(self, arr: torch.Tensor, froms, tos, operator, operand=None, memo=None):
        """``memo``: the public API's key tail for this call shape (``(frm, counts, operator,
        codec, compress)``) — memoise the fused IPC reduce-scatter it runs for the API's fast path."""
        flat = self._flat(arr)
        r = self.rank
        base = froms[0]
        whole = flat[base:tos[-1]]
        if whole.numel() == 0:
            return arr
        op = self._op(operator, whole)
        counts = [t - f for f, t in zip(froms, tos)]
        algo = self.select("reduce_scatter", whole.numel() * whole.element_size(), op, whole.dtype, operand)
        if algo == "fp8":
            algo = "a2a"    # exact path for ragged RS; fp8 RS is used inside the compressed allreduce
        if algo in ("rccl", "a2a") and self._zc_ok(whole) and self._ipc_obj.reduce_scatter_registered(flat, froms,
                                                                                                        tos, op):
            self._count("reduce_scatter.ipc_zc")       # registered tensor: zero copy, any size
            return arr
        if algo in ("rccl", "a2a") and self._ipc_direct_ok(op, whole):
            if self._plan_memo(memo is not None, "reduce_scatter", arr, memo or (),
                               lambda: self._ipc_obj.reduce_scatter(flat, froms, tos, op)):
                self._count("reduce_scatter.ipc")
                return arr
        if algo in ("rccl", "a2a"):
            big = self._large_choice("reduce_scatter", whole, op)
            if big == "ipc":
                inst = self.ipc_large()
                if inst is not None and inst.reduce_scatter_large(flat, froms, tos, op):
                    self._count("reduce_scatter.ipc_large")
                    return arr
            elif big == "a2a":
                algo = "a2a"
        self._count("reduce_scatter." + algo)
        equal = len(set(counts)) == 1
        if algo == "rccl" and equal and self.coll.reduce_scatter_ok:
            self.coll.reduce_scatter_tensor(flat[froms[r]:tos[r]], whole, op.code)
        elif algo == "rccl" and self.coll.reduce_scatter_ok:
            cmax = max(counts)
            stage = torch.zeros(self.p * cmax, dtype=whole.dtype, device=whole.device)
            for j in range(self.p):
                if counts[j]:
                    stage[j * cmax:j * cmax + counts[j]].copy_(flat[froms[j]:tos[j]])
            out = torch.empty(cmax, dtype=whole.dtype, device=whole.device)
            self.coll.reduce_scatter_tensor(out, stage, op.code)
            if counts[r]:
                flat[froms[r]:tos[r]].copy_(out[:counts[r]])
        else:
            self._reduce_scatter_a2a(flat, froms, tos, op)
        return arr

    # ================================================================== allgather
    def allgather(self, arr: torch.Tensor, froms, tos, memo: bool = False):
        flat = self._flat(arr)
        whole = flat[froms[0]:tos[-1]]
        if whole.numel() and self._zc_ok(whole) and self._ipc_obj.allgather_registered(flat, froms, tos):
            self._count("allgather.ipc_zc")            # registered tensor: zero copy, any size
            return arr
        if whole.numel() and self._ipc_direct_ok(None, whole) and \
                self._plan_memo(memo, "allgather", arr, (tuple(froms), tuple(tos)),
                                lambda: self._ipc_obj.allgather(flat, froms, tos)):
            self._count("allgather.ipc")
            return arr
        big = self._large_choice("allgather", whole, None) if whole.numel() else None
        if big == "ipc":
            inst = self.ipc_large()
            if inst is not None and inst.allgather_large(flat, froms, tos):
                self._count("allgather.ipc_large")
                return arr
        elif big == "p2p":
            self._count("allgather.p2p")
            self._allgather_p2p(flat, froms, tos)
            return arr
        self._count("allgather")
        self._allgather_any(flat, froms, tos)
        return arr

    def _large_choice(self, kind: str, whole: torch.Tensor, op) -> Optional[str]:
        """Schedule for a reduce-scatter / all-gather above the direct-IPC tier: forced by
        ``MP4X_DEVICE_ALGO=ipc2`` (IPC pieces), or pinned by :meth:`autotune_reduce_scatter` /
        :meth:`autotune_allgather` for this (dtype, op, size class); None = RCCL."""
        if self.algo in ("ipc2", "ipc"):
            return "ipc" if self.ipc_enabled and (op is None or self._ipc_ok(op, whole.dtype, 16)) else None
        if self.algo not in ("", "auto"):
            return None
        t = self._tuned.pinned(self._rsag_key(kind, whole, op)) if self._tuned else None
        if t is None and self._dm_large_ok(whole) and (op is None or self._ipc_ok(op, whole.dtype, 16)):
            return "ipc"     # no RCCL underneath (see _dm_large_ok): the piecewise IPC kernels
        if t is None and op is not None and not self.rccl_ok(op, whole.dtype) and whole.is_cuda and \
                self._ipc_ok(op, whole.dtype, 16):
            return "ipc"     # an op RCCL cannot reduce: the piecewise IPC reduce-scatter, not a2a
        return t

    @staticmethod
    def _rsag_key(kind: str, whole: torch.Tensor, op) -> tuple:
        return (kind, whole.dtype, int(op.code) if op is not None else -1,
                max(0, whole.numel() * whole.element_size() - 1).bit_length())

    def _zc_ok(self, whole: torch.Tensor) -> bool:
        """Zero-copy RS / AG on a registered tensor (no schedule forced otherwise).  Whether the
        range is registered is decided per rank; registration is collective, and a rank running
        the other protocol fails the call at once (epoch tag), it cannot mix buffers."""
        return self._zc and whole.is_cuda and self._ipc_obj is not None and self.ipc_enabled and \
            self.algo in ("", "auto", "ipc2", "ipc2z", "ipc") and bool(self._ipc_obj._regs)

    def _ipc_direct_ok(self, op, whole: torch.Tensor) -> bool:
        """Direct IPC reduce-scatter / all-gather tier: up to the two-shot size, unless a schedule
        is forced.  (The range alignment is checked by IpcAllreduce, rank-independently.)"""
        nbytes = whole.numel() * whole.element_size()
        if self.algo not in ("", "auto") or nbytes > self.ipc_twoshot_max or not self.ipc_enabled:
            return False
        if op is not None and not self._ipc_ok(op, whole.dtype, 16):
            return False
        if whole.is_cuda and torch.cuda.is_current_stream_capturing() and \
                (self._ipc_obj is None or self._ipc_obj._epoch_dev is None):
            return False
        return self.ipc() is not None

    # ================================================================== sparse map
    def allreduce_map(self, mapData: Dict, operator):
        from .sparse import allreduce_map_device
        self._count("allreduce_map")
        return allreduce_map_device(self, mapData, operator)

    def all_to_all_v(self, send: torch.Tensor, send_counts: List[int], recv: Optional[torch.Tensor] = None):
        """Ragged all-to-all over rows of ``send`` (rows grouped by destination)."""
        self._count("all_to_all_v")
        if sum(send_counts) != send.shape[0]:
            raise Mp4jException(f"sendCounts sum {sum(send_counts)} != rows {send.shape[0]}")
        got = self._all_to_all_v_ipc(send, send_counts, recv)
        if got is not None:
            return got
        sc = torch.tensor(send_counts, dtype=torch.int64, device=self.device if self.backend == "nccl" else "cpu")
        rc = torch.empty_like(sc)
        self.coll.all_to_all_single(rc, sc)
        recv_counts = [int(x) for x in rc.tolist()]
        shape = (sum(recv_counts),) + tuple(send.shape[1:])
        if recv is None:
            recv = torch.empty(shape, dtype=send.dtype, device=send.device)
        elif tuple(recv.shape) != shape:
            raise Mp4jException(f"recvData shape {tuple(recv.shape)} != {shape}")
        self.coll.all_to_all_single(recv, send.contiguous(), recv_counts, list(send_counts))
        return recv, recv_counts

    def _all_to_all_v_ipc(self, send: torch.Tensor, send_counts: List[int], recv: Optional[torch.Tensor]):
        """The all-to-all-v as one IPC copy-plan kernel (sparse._ipc_rows_alltoallv) when the rows
        are whole 16-byte vectors and the largest rank's payload fits a staging buffer; the count
        matrix comes from one small all-gather.  Every condition is rank-independent (shape,
        dtype, environment, the gathered counts), so every rank takes the same path; None when
        the call does not qualify."""
        from . import sparse
        width = 1
        for d in send.shape[1:]:
            width *= int(d)
        rb = width * send.element_size()          # bytes per row
        if rb == 0 or rb % 16 or self.algo not in ("", "auto", "ipc") or not send.is_cuda or \
                not sparse._sparse_ipc_ok(self, send):
            return None
        mat = sparse._count_matrix(self, torch.tensor(list(send_counts), dtype=torch.int64, device=send.device))
        recv_counts = [mat[j][self.rank] for j in range(self.p)]
        shape = (sum(recv_counts),) + tuple(send.shape[1:])
        if recv is not None and tuple(recv.shape) != shape:
            raise Mp4jException(f"recvData shape {tuple(recv.shape)} != {shape}")
        out = sparse._ipc_rows_alltoallv(self, send.contiguous().view(torch.uint8).view(send.shape[0], rb), mat)
        if out is None:
            return None
        res = out.view(send.dtype).view(shape)
        if recv is not None:
            recv.copy_(res)
            res = recv
        return res, recv_counts

    def reduce_map(self, mapData: Dict, operator, root: int):
        from .sparse import reduce_map_device
        self._count("reduce_map")
        return reduce_map_device(self, mapData, operator, root)

    def gather_map(self, mapData: Dict, root: int):
        from .sparse import gather_map_device
        self._count("gather_map")
        return gather_map_device(self, mapData, root)

    def allgather_map(self, mapData: Dict):
        from .sparse import allgather_map_device
        self._count("allgather_map")
        return allgather_map_device(self, mapData)

    def reduce_scatter_map(self, mapDataList: List[Dict], operator):
        from .sparse import reduce_scatter_map_device
        self._count("reduce_scatter_map")
        return reduce_scatter_map_device(self, mapDataList, operator)

    def scatter_map(self, mapDataList, root: int):
        from .sparse import scatter_map_device
        self._count("scatter_map")
        return scatter_map_device(self, mapDataList, root)

    def broadcast_map(self, mapData: Dict, root: int):
        from .sparse import broadcast_map_device
        self._count("broadcast_map")
        return broadcast_map_device(self, mapData, root)

    def barrier(self):
        self.coll.barrier()

    def all_gather_object(self, obj) -> List:
        """Small host objects from every rank (rank order) — key dictionaries, handles."""
        if hasattr(self.coll, "_exchange"):
            return self.coll._exchange(obj)
        return self.comm.server.call("allgather_obj", self.rank, obj)


def _watched(name, fn):
    """Bracket a device collective: first the fail-stop check of the IPC error words (an earlier
    call that timed out fails this one, :meth:`DeviceEngine.check_failed`), then the watchdog
    (host time inside the call; a HIP event on the stream when the outermost collective returns)."""
    def wrapper(self, *args, **kwargs):
        if self._ipc_obj is not None or self._ipc_large is not None or self._ipc_fp8_big is not None or \
                self._hier is not None:
            self.check_failed()
        wd = self.watchdog
        if wd is None:
            return fn(self, *args, **kwargs)
        tok = wd.begin(name)
        try:
            return fn(self, *args, **kwargs)
        finally:
            wd.end(tok, self.device)
    wrapper.__name__ = fn.__name__
    wrapper.__doc__ = fn.__doc__
    wrapper.__wrapped__ = fn
    return wrapper


# Attributes the schedule choice reads (DeviceEngine._select): properties whose setter bumps
# ``_state_ver``, the select memo's view of them (class-level defaults kept).
_TIER_ATTRS = ("algo", "ipc_enabled", "ipc_oneshot_max", "_oneshot_ar_max", "ipc_twoshot_max", "_hier_failed",
               "_hier_auto", "backend",
               "a2a_bytes", "hier_min_bytes", "_dm_large", "layout", "device")


def _tier_attr(name, default):
    slot = "_tier_" + name

    def get(self):
        try:
            return self.__dict__[slot]
        except KeyError:
            if default is _NO_DEFAULT:
                raise AttributeError(name) from None
            return default

    def put(self, v):
        d = self.__dict__
        d[slot] = v
        d["_state_ver"] = d.get("_state_ver", 0) + 1
        fa = d.get("_fast_ar")
        if fa:
            fa.clear()

    return property(get, put, doc=f"tier input {name!r} (assignments invalidate the select memo)")


_NO_DEFAULT = object()
DeviceEngine._state_ver = 0
for _n in _TIER_ATTRS:
    setattr(DeviceEngine, _n, _tier_attr(_n, DeviceEngine.__dict__.get(_n, _NO_DEFAULT)))

_WATCHED = ["allreduce", "autotune_allreduce", "autotune_reduce_scatter", "autotune_allgather", "autotune_reduce",
            "autotune_broadcast", "autotune_gather", "autotune_scatter", "reduce_scatter", "allgather", "broadcast", "reduce", "gather",
            "scatter", "allreduce_map", "all_to_all_v", "reduce_map", "gather_map", "allgather_map",
            "reduce_scatter_map", "scatter_map", "broadcast_map", "barrier"]
for _n in _WATCHED:
    setattr(DeviceEngine, _n, _watched(_n, getattr(DeviceEngine, _n)))
