"""ProcessComm — one communicator per process (one process per GPU on MI355X).

Public API = the reference's ``ProcessCommSlave``
(/root/reference/src/main/java/com/fenbi/mp4j/comm/ProcessCommSlave.java), same
method names and argument order, plus snake_case aliases.  Shared semantics
(SURVEY §2.2):

* array collectives work IN PLACE on ``[from, to)`` ranges and return the same
  buffer; non-root results of gather/reduce are unspecified;
* ``slaveNum == 1`` returns the input unchanged;
* ranges are validated like ``CommUtils`` and raise :class:`Mp4jException`.

Data placement decides the engine:

* ``torch.Tensor`` on a GPU → :class:`~mp4x.parallel.device_engine.DeviceEngine`
  (RCCL over xGMI + the hand-written HIP kernels in ``csrc/``);
* numpy arrays / CPU tensors / Python lists (String / Object operands) /
  dicts → :class:`~mp4x.parallel.host_engine.HostEngine` over the TCP mesh.

Lifecycle (bootstrap, heartbeat, close/exception protocol, remote logs) follows
ProcessCommSlave.java:143-387.
"""
from __future__ import annotations

import logging
import os
import threading
import time
import traceback
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from ..control.client import MasterClient
from ..control.protocol import local_ip
from ..exceptions import Mp4jException, RangeError
from ..operands import Operand, Operands, DEFAULT_SERIALIZER
from ..operators import CustomOperator
from ..utils.commutils import CommUtils
from ..utils.hashing import owner_of
from .host_engine import HostEngine, choose_allreduce
from .transport import HostTransport

LOG = logging.getLogger("mp4x.comm")


# Return codes of the native fast paths that mean "nothing was launched, the epoch did not move"
# (csrc/include/mp4x/ops.h): the call goes on to the full path.  Any other nonzero code is a HIP
# error AFTER the epoch moved — raised at once (falling back would bump the epoch a
# second time and leave this rank a call ahead of its peers).
_NOT_LAUNCHED = frozenset((1001, 1002, 1003, 1004))


def _fast_ok(rc: int, where: str) -> bool:
    """True: the fast path launched.  False: refused before anything moved (take the full path).
    Raises for a launch error after the epoch moved."""
    if rc == 0:
        return True
    if rc in _NOT_LAUNCHED:
        return False
    from ..ops import native
    native.check(rc, where)
    return False


HEARTBEAT_DELAY = float(os.environ.get("MP4X_HEARTBEAT_DELAY", 5.0))
HEARTBEAT_PERIOD = float(os.environ.get("MP4X_HEARTBEAT_PERIOD", 15.0))
HEARTBEAT_MAX_FAIL = int(os.environ.get("MP4X_HEARTBEAT_MAX_FAIL", 4))
BCAST_TREE_BYTES = int(os.environ.get("MP4X_BCAST_TREE_BYTES", 1 << 16))
SHM_ON = os.environ.get("MP4X_SHM", "1") == "1"
# host allreduceMap of primitive values through the columnar path (parallel/hostmap.py)
HOST_MAP_COLUMNAR = os.environ.get("MP4X_HOST_MAP_COLUMNAR", "1") == "1"
# same-host ranks take /dev/shm at every size: 4 procs, 16 doubles 34 us vs 500 us over the TCP
# mesh; 800 KB 0.36 vs 1.8 ms; 8 procs 0.14 vs 1.3 ms (profiles/r1/host_shm_vs_tcp.jsonl)
SHM_MIN_BYTES = 0


def _is_device_tensor(x) -> bool:
    t = type(x)
    if t.__module__.startswith("torch") and t.__name__ in ("Tensor", "Parameter"):
        return bool(x.is_cuda)
    return False


def _is_torch(x) -> bool:
    t = type(x)
    return t.__module__.startswith("torch") and t.__name__ in ("Tensor", "Parameter")


def _host_view(arr, operand: Operand):
    """Returns (buffer usable by the host engine, restore fn)."""
    if isinstance(arr, np.ndarray):
        if arr.ndim != 1:
            raise Mp4jException("array collectives take 1-D arrays")
        return arr
    if _is_torch(arr):
        return arr.numpy()
    if isinstance(arr, list):
        return arr
    raise Mp4jException(f"unsupported array type {type(arr)}")


class _FaultInjector:
    """``MP4X_FAULT_INJECT="rank:op_index[:mode]"`` — kill rank at its op_index-th collective
    (mode ``exit`` = os._exit(9), ``raise`` = Mp4jException).  Used by the failure tests."""

    def __init__(self, rank: int):
        spec = os.environ.get("MP4X_FAULT_INJECT", "")
        self.active = False
        if spec:
            parts = spec.split(":")
            self.rank, self.at = int(parts[0]), int(parts[1])
            self.mode = parts[2] if len(parts) > 2 else "exit"
            self.active = self.rank == rank
        self.count = 0

    def tick(self, name: str):
        if not self.active:
            return
        self.count += 1
        if self.count == self.at:
            if self.mode == "raise":
                raise Mp4jException(f"fault injected in {name}")
            os._exit(9)


class ProcessCommSlave:
    """Process-level communicator (reference ``ProcessCommSlave``)."""

    def __init__(self, loginName: Optional[str] = None, masterHost: str = "127.0.0.1",
                 masterPort: int = 61235, *, rank: Optional[int] = None,
                 heartbeat: bool = True, device: Optional[int] = None):
        self.loginName = loginName or os.environ.get("USER", "mp4x")
        self.closed = False
        self._device_engine = None
        self._fast_ar = None       # the device engine's latency memo (allreduceArray fast path)
        self._fast_pl = None       # its copy-plan launcher (broadcast / gather / scatter / allgather)
        self._fast_rs = None       # its fused reduce-scatter launcher
        self._device_index = device
        self._shm = None
        self._shm_cfg = None       # (shm allowed for this job, MP4X_SHM_MIN_BYTES), read at first use
        LOG.info("master host:%s, master port:%s", masterHost, masterPort)
        self.server = MasterClient(masterHost, masterPort)
        loop = masterHost in ("127.0.0.1", "localhost", "::1")
        self.transport = HostTransport(advertise_host="127.0.0.1" if loop else local_ip())
        req = rank if rank is not None else int(os.environ.get("MP4X_RANK", -1))
        info = self.server.call("register", self.transport.address, int(req))
        if info is None:  # reference bug fixed: it tested `address == null` (ProcessCommSlave.java:159)
            raise Mp4jException("slaves connecting master failed, may be this slave restarted "
                                "or master port is occupied, task failed!")
        self.rank: int = int(info["rank"])
        self.addresses: List[str] = list(info["addresses"])
        self.slaveNum: int = len(self.addresses)
        self.rankMsgPrefix = f"[rank={self.rank}] "
        self.transport.set_peers(self.rank, self.addresses)
        self.engine = HostEngine(self.transport, self.rank, self.slaveNum)
        self._fault = _FaultInjector(self.rank)
        self.stats: Dict[str, Any] = {"calls": {}, "bytes": 0}
        from ..utils.trace import Tracer
        self.tracer = Tracer(self.rank)

        pid = os.getpid()
        host = self.transport.advertise_host
        if self.slaveNum > 1 and not loop:
            script = f'ssh {self.loginName}@{host} "kill -9 {pid}"'
        else:
            script = f"kill -9 {pid}"
        self.server.call("kill_me", self.rank, script)

        self._hb_stop = threading.Event()
        self._hb_fail = 0
        if heartbeat:
            self._hb_client = MasterClient(masterHost, masterPort)
            self._hb_thread = threading.Thread(target=self._heartbeat_loop, daemon=True, name="mp4x-heartbeat")
            self._hb_thread.start()
        else:
            self._hb_client = None
        self.info("this slave init finished!")

    # ================================================================ lifecycle
    def _heartbeat_loop(self):
        if self._hb_stop.wait(HEARTBEAT_DELAY):
            return
        while not self._hb_stop.is_set():
            try:
                if not self.closed:
                    self._hb_client.call("heartbeat", self.rank)
                self._hb_fail = 0
            except Exception as e:  # reference: >4 failures → System.exit(4) (ProcessCommSlave.java:212-227)
                self._hb_fail += 1
                LOG.error("rank:%d send heartbeat exception, exception time:%d: %s", self.rank, self._hb_fail, e)
                if self._hb_fail > HEARTBEAT_MAX_FAIL:
                    LOG.error("heart beat exception > %d master may be shutdowned! this slave will be shutdowned...",
                              HEARTBEAT_MAX_FAIL)
                    os._exit(4)
            if self._hb_stop.wait(HEARTBEAT_PERIOD):
                return

    def close(self, code: int = 0) -> None:
        """Reference ProcessCommSlave.close (:234-271).

        A clean close (code 0) first drains this rank's device work and checks the IPC error
        words: if a device collective gave up waiting for a peer, its result was invalid, so the
        close reports it (master error log), closes with code 1 (the job fails, as the reference's
        ``exception()`` -> ``close(1)``) and raises :class:`Mp4jException` afterwards."""
        if self.closed:
            return
        failure = None
        eng = self._device_engine
        if not code and eng is not None:
            try:
                if eng.device.type == "cuda":
                    import torch
                    torch.cuda.synchronize(eng.device)
                eng.check_failed()
            except Mp4jException as e:
                failure, code = e, 1
                try:
                    self.error(f"close: {e}")
                except Exception:   # noqa: BLE001 — the master may be gone; the code still says it
                    pass
        LOG.info("close code=%s", code)
        try:
            self.server.call("close", self.rank, int(code))
            master = getattr(self, "_embedded_master", None)
            if master is not None:
                # the master lives in this process (mp4x.launch): returning — and letting the
                # process exit — before every other rank's close message arrived would reset their
                # connections mid-close.  A failure close ends the wait at once.
                master.stop(timeout=float(os.environ.get("MP4X_MASTER_LINGER", 300.0)))
        finally:
            self.closed = True
            self._hb_stop.set()
            if self._device_engine is not None:
                try:
                    if code:
                        self._device_engine.abort()      # fail-stop: never block on a dead peer
                    else:
                        self._device_engine.shutdown()
                except Exception:
                    pass
            if self._shm is not None:
                self._shm.close()
            self.transport.close()
            self.server.close()
            if self._hb_client is not None:
                self._hb_client.close()
        if failure is not None:
            raise failure

    def exception(self, e: BaseException) -> None:
        """Report the stack to the master, wait, then ``close(1)`` (reference :360-373)."""
        tb = "".join(traceback.format_exception(type(e), e, e.__traceback__))
        try:
            self.error("slave exception:" + tb)
            time.sleep(float(os.environ.get("MP4X_EXCEPTION_SLEEP", 5.0)))
        finally:
            self.close(1)

    def writeFile(self, content: str, fileName: str) -> None:
        self.server.call("write_file", content, fileName)

    def info(self, s: str, onlyRank0: bool = True) -> None:
        if not onlyRank0:
            self.server.call("info", self.rank, self.rankMsgPrefix + str(s))
        elif self.rank == 0:
            self.server.call("info", self.rank, str(s))

    def debug(self, s: str, onlyRank0: bool = True) -> None:
        if not onlyRank0:
            self.server.call("debug", self.rank, self.rankMsgPrefix + str(s))
        elif self.rank == 0:
            self.server.call("debug", self.rank, str(s))

    def error(self, s: str) -> None:
        self.server.call("error", self.rank, self.rankMsgPrefix + str(s))

    def getSlaveNum(self) -> int:
        return self.slaveNum

    def getRank(self) -> int:
        return self.rank

    def barrier(self) -> None:
        """Master barrier (reference :432-438); device work queued before it is NOT waited for.
        Raises if an IPC collective of this rank already timed out (``DeviceEngine.check_failed``,
        pinned host words, no device sync) — after joining the barrier, so the peers are not
        left waiting in it."""
        self._tick("barrier")
        self.server.call("barrier", self.rank)
        if self._device_engine is not None:
            self._device_engine.check_failed()

    def peer_barrier(self) -> None:
        """O(log p) barrier over the data plane (no master round trip)."""
        self.engine.dissemination_barrier()

    # ================================================================ device engine
    @property
    def device(self):
        if self._device_engine is None:
            from .device_engine import DeviceEngine
            self._device_engine = DeviceEngine(self, self._device_index)
            self._enable_fast_path()
        return self._device_engine

    def _enable_fast_path(self) -> None:
        """Arm the allreduceArray latency fast path (VERDICT r4 Next #5): a call whose shape the
        device engine memoised (staged one-/two-shot on the default IPC instance) goes from the
        API's first lines to ONE native call, ``mp4x_ipc_fast_allreduce`` (error words, capture
        check, epoch, launch).  Off with fault injection (it counts every API call) or
        ``MP4X_FAST_PATH=0``."""
        eng = self._device_engine
        from ..ops import native
        if eng is None or self._fault.active or self.slaveNum < 2 or os.environ.get("MP4X_FAST_PATH", "1") != "1" \
                or getattr(eng.device, "type", None) != "cuda":
            return
        lx = native.launch_ext()
        if lx is None or not hasattr(lx, "fast_allreduce") or not hasattr(eng._fast_ar, "addr_key"):
            return
        import torch
        self._fast_lx = lx.fast_allreduce
        self._fast_pl = getattr(lx, "fast_plan", None)
        self._fast_rs = getattr(lx, "fast_rs", None)
        self._fast_stream = native.stream_ptr
        self._fast_tensor = torch.Tensor
        self._fast_calls = self.stats["calls"]
        self._fast_ar = eng._fast_ar

    def _fast_after(self, stat: str, api: str) -> None:
        """Book-keeping of a fast-path call: the API and engine call counts, and the watchdog's
        device-side coverage (an event when none is outstanding, as ``CollectiveWatchdog.end``)."""
        c = self._fast_calls
        c[api] = c.get(api, 0) + 1
        eng = self._device_engine
        st = eng.stats
        st[stat] = st.get(stat, 0) + 1
        wd = eng.watchdog
        if wd is not None and not wd._npending:
            wd.end(wd.begin(stat.partition(".")[0]), eng.device)

    def _fast_plan_call(self, kind: str, arrData, tail: tuple) -> bool:
        """The latency fast path of broadcast / gather / scatter / all-gather: a call shape the
        engine memoised (one staged copy plan, DeviceEngine._plan_memo) runs as ONE native call
        (``mp4x_ipc_fast_plan``: error words, capture check, alignment, epoch, launch).  False:
        not memoised or not launched — the full path decides, validates, raises or records.  A
        hit implies the ranges and root were validated when the shape was memoised."""
        if self._fast_pl is None or type(arrData) is not self._fast_tensor or not arrData.is_cuda or \
                not arrData.is_contiguous():
            return False
        fast = self._fast_ar
        base, n = arrData.data_ptr(), arrData.numel()
        try:
            ent = fast.get((kind, fast.addr_key(base, n * arrData.element_size()), arrData.get_device(), n,
                            arrData.dtype) + tail)
        except TypeError:               # unhashable ranges (e.g. arrays): the full path
            return False
        if ent is None:
            return False
        rc = self._fast_pl(ent, self._fast_stream(), base)
        if rc and not _fast_ok(rc, "mp4x_ipc_fast_plan"):
            return False
        self._fast_after(ent.stat, ent.api)
        return True

    def registerBuffer(self, tensor) -> bool:
        """Collective (extension, like ``ncclCommRegister``): map a device tensor into every peer
        so allreduces on it (or on [from, to) views of it) run the zero-copy xGMI two-shot — no
        staging copy and no pieces at any size.  Every rank registers its same-shaped tensor at
        the same point and keeps it alive until :meth:`deregisterBuffer`.  Returns False on every
        rank when the mesh refused it (the staged kernels are used then)."""
        if self.slaveNum == 1 or not _is_device_tensor(tensor):
            return False
        return self.device.register_buffer(tensor)

    def deregisterBuffer(self, tensor) -> None:
        if self._device_engine is not None:
            self._device_engine.deregister_buffer(tensor)

    register_buffer = registerBuffer
    deregister_buffer = deregisterBuffer

    def memAlloc(self, n: int, dtype=None, device=None):
        """Collective (extension, like ``ncclMemAlloc``): an ``n``-element device tensor that is
        registered with every peer from the start, at ANY size — also above the 2 GiB at which
        a caching-allocator tensor cannot be mapped (parallel/vmm.py).  Allreduce / reduce-
        scatter / all-gather on it (or on [from, to) views) run the zero-copy xGMI kernels: the
        in-place 8 GB arrays of the reference (README.md:313) with no staging.  Contents are
        uninitialised.  Free with :meth:`memFree` (collective).  Without a multi-rank GPU mesh it
        returns a plain tensor (``torch.empty``)."""
        import torch
        dtype = dtype or torch.float32
        want_dev = device is None or str(device).startswith("cuda")
        if self.slaveNum > 1 and want_dev and torch.cuda.is_available():
            try:
                t = self.device.mem_alloc(int(n), dtype)
            except Mp4jException as e:
                # agreed on every rank inside mem_alloc (the failure travels in its collectives),
                # so every rank falls back together: a plain tensor on the staged kernels / RCCL
                LOG.warning("memAlloc(%d) fell back to a plain tensor: %s", int(n), e)
                t = None
            if t is not None:
                return t
        dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
        return torch.empty(int(n), dtype=dtype, device=dev)

    def memFree(self, tensor) -> None:
        """Collective: release a :meth:`memAlloc` tensor (no-op for a plain tensor)."""
        if self._device_engine is not None:
            self._device_engine.mem_free(tensor)

    mem_alloc = memAlloc
    mem_free = memFree

    def _shm_engine(self, buf, operand: Operand, operator, nelems: int):
        """The shared-memory engine when this call qualifies (decision identical on every rank).
        The job-level inputs (``MP4X_SHM``, ``MP4X_SHM_MIN_BYTES``, all ranks on one host) are
        read once: the per-call check is a few attribute tests on the host latency path."""
        cfg = self._shm_cfg
        if cfg is None:
            from .shm import same_host
            cfg = self._shm_cfg = (os.environ.get("MP4X_SHM", "1") == "1" and self.slaveNum > 1 and
                                   same_host(self.addresses),
                                   int(os.environ.get("MP4X_SHM_MIN_BYTES", SHM_MIN_BYTES)))
        if not cfg[0] or not operand.is_primitive or operand.compress:
            return None
        if not isinstance(buf, np.ndarray) or buf.dtype != operand.np_dtype:
            return None
        if operator is not None and (getattr(operator, "is_custom", False) or operator.dtype != operand.dtype):
            return None
        if nelems * buf.itemsize < cfg[1]:
            return None
        if self._shm is None:
            from .shm import ShmEngine
            self._shm = ShmEngine(self)
        return self._shm

    def _tick(self, name: str):
        self._fault.tick(name)
        c = self.stats["calls"]
        c[name] = c.get(name, 0) + 1

    def _check_len(self, a, name):
        if len(a) != self.slaveNum:
            raise Mp4jException(f"{name} array length must be equal to slaveNum")

    # ================================================================ gather
    def gatherArray(self, arrData, operand: Operand, sendfroms: Sequence[int], sendtos: Sequence[int],
                    rootRank: int):
        if self._fast_ar and type(sendfroms) is list and type(sendtos) is list and \
                self._fast_plan_call("gather", arrData, (tuple(sendfroms), tuple(sendtos), rootRank)):
            return arrData
        self._tick("gatherArray")
        self._check_len(sendfroms, "sendfroms")
        self._check_len(sendtos, "sendtos")
        if self.slaveNum == 1:
            return arrData
        CommUtils.isfromsTosLegal(sendfroms, sendtos)
        self._check_root(rootRank)
        if _is_device_tensor(arrData):
            return self.device.gather(arrData, list(sendfroms), list(sendtos), rootRank,
                                      memo=self._fast_ar is not None)
        buf = _host_view(arrData, operand)
        self.engine.tree_gather(buf, sendfroms, sendtos, operand, rootRank)
        return arrData

    def _map_on_device(self, mapData: Dict, all_keys=None) -> bool:
        """Do this map collective's values live on the GPU?  A rank with an empty map cannot
        tell, so the ranks agree over the control plane — a round of a few bytes per rank: the
        placement flag, whether the rank has not-yet-numbered keys (``all_keys``: every key the
        device op will number; default the map's), and the value shape.  The new key strings
        themselves then travel PEER TO PEER (``sparse.allgather_keys`` over the host mesh), so
        the master's load does not grow with the keys, and the device op skips its own
        key-dictionary round (``_keys_presynced``)."""
        mine = -1 if not mapData else int(_is_torch(next(iter(mapData.values()))))
        new = []
        if mine == 1 and self._device_engine is None:
            # Creating the device engine is collective (process group, shared tuning table): it
            # must not start before this round, or a rank with an empty map (which learns only
            # here that the op is a device op) leaves this rank waiting in the engine's bootstrap
            # while it waits in the round.  No engine yet = an empty dictionary: every key is new.
            new = list(dict.fromkeys(mapData.keys() if all_keys is None else all_keys))
        elif mine == 1:
            from .sparse import TensorMap, _dictionary
            d = _dictionary(self.device)
            packed = None
            if all_keys is None:
                # the native walk finds the unseen keys AND the ids / rows the device op needs:
                # one pass over the map instead of two (sparse._map_tensors takes it up)
                from .sparse import _pack_native
                try:
                    packed = _pack_native(d, mapData)
                except Exception:   # noqa: BLE001 — never fail alone before the agreement round
                    packed = None
                self.device._prepacked = (mapData, packed) if packed is not None else None
            if packed is not None:
                if packed[1]:
                    keys = list(mapData.keys())
                    new = [keys[i] for i in np.flatnonzero(packed[0] < 0)]
            elif not (all_keys is None and isinstance(mapData, TensorMap) and mapData.pristine() and mapData._d is d):
                new = d.unknown(list(mapData.keys()) if all_keys is None else list(all_keys))
        # the value shape / dtype travels too: a rank with an empty map must still size its
        # (empty) rows like everyone else's for the device exchange
        meta = None
        if mine == 1:
            v0 = next(iter(mapData.values()))
            meta = (tuple(v0.shape), str(v0.dtype).replace("torch.", ""))
        res = self.server.call("allgather_obj", self.rank, (mine, len(new), meta))
        on_device = any(f == 1 for f, _, _ in res)
        if on_device:
            from .sparse import _dictionary, allgather_keys
            eng = self.device
            if any(nn for _, nn, _ in res):
                _dictionary(eng).learn_round(allgather_keys(eng, new))
            eng._keys_presynced = True
            eng._map_meta = next((m for _, _, m in res if m is not None), None)
        return on_device

    def gatherMap(self, mapData: Dict, operand: Operand, rootRank: int) -> Dict:
        self._tick("gatherMap")
        if self.slaveNum == 1:
            return mapData
        self._check_root(rootRank)
        if self._map_on_device(mapData):
            return self.device.gather_map(mapData, rootRank)
        return self.engine.tree_gather_map(mapData, operand, rootRank)

    # ================================================================ allgather
    def allgatherArray(self, arrData, operand: Operand, froms: Sequence[int], tos: Sequence[int]):
        if self._fast_ar and type(froms) is list and type(tos) is list and \
                self._fast_plan_call("allgather", arrData, (tuple(froms), tuple(tos))):
            return arrData
        self._tick("allgatherArray")
        self._check_len(froms, "froms")
        self._check_len(tos, "tos")
        if self.slaveNum == 1:
            return arrData
        CommUtils.isfromsTosLegal(froms, tos)
        if _is_device_tensor(arrData):
            return self.device.allgather(arrData, list(froms), list(tos), memo=self._fast_ar is not None)
        buf = _host_view(arrData, operand)
        shm = self._shm_engine(buf, operand, None, tos[-1] - froms[0])
        if shm is not None and buf.flags.c_contiguous:
            shm.allgather(buf, froms, tos)
            return arrData
        self.engine.ring_allgather(buf, froms, tos, operand)
        return arrData

    def allgatherMap(self, mapData: Dict, operand: Operand) -> List[Dict]:
        self._tick("allgatherMap")
        if self.slaveNum == 1:
            return [mapData]
        if self._map_on_device(mapData):
            return self.device.allgather_map(mapData)
        blocks = self.engine.ring_allgather_maps([mapData], operand)
        return [b[0] for b in blocks]

    # ================================================================ broadcast
    def broadcastArray(self, arrData, operand: Operand, frm: int, to: int, rootRank: int):
        if self._fast_ar and self._fast_plan_call("broadcast", arrData, (frm, to, rootRank)):
            return arrData
        self._tick("broadcastArray")
        if self.slaveNum == 1:
            return arrData
        CommUtils.isFromToLegal(frm, to)
        self._check_root(rootRank)
        if _is_device_tensor(arrData):
            return self.device.broadcast(arrData, frm, to, rootRank, memo=self._fast_ar is not None)
        buf = _host_view(arrData, operand)
        shm = self._shm_engine(buf, operand, None, to - frm)
        if shm is not None and buf.flags.c_contiguous:
            shm.broadcast(buf, frm, to, rootRank)
            return arrData
        nbytes = (to - frm) * (operand.np_dtype.itemsize if operand.is_primitive else 64)
        if nbytes <= BCAST_TREE_BYTES or (to - frm) < self.slaveNum:
            self.engine.tree_bcast(buf, frm, to, operand, rootRank)
        else:
            # van de Geijn: scatter + allgather (reference :750-775)
            froms, tos, _ = CommUtils.even_split(frm, to, self.slaveNum)
            self.engine.tree_scatter(buf, froms, tos, operand, rootRank)
            self.engine.ring_allgather(buf, froms, tos, operand)
        return arrData

    def broadcast(self, value, operand: Operand, rootRank: int):
        self._tick("broadcast")
        if self.slaveNum == 1:
            return value
        arr = operand.box(value)
        self.broadcastArray(arr, operand, 0, 1, rootRank)
        return operand.unbox(arr)

    def broadcastMap(self, mapData: Dict, operand: Operand, rootRank: int) -> Dict:
        """Root partitions by key hash → scatterMap → allgatherMap → merge (reference :842-883)."""
        self._tick("broadcastMap")
        if self.slaveNum == 1:
            return mapData
        self._check_root(rootRank)
        if self._map_on_device(mapData if self.rank == rootRank else {}):
            return self.device.broadcast_map(mapData, rootRank)
        p = self.slaveNum
        blocks = None
        if self.rank == rootRank:
            blocks = [[d] for d in self._partition(mapData)]
        mine = self.engine.tree_scatter_maps(blocks, operand, rootRank)
        allb = self.engine.ring_allgather_maps(mine, operand)
        out: Dict = {}
        for blk in allb:
            for d in blk:
                out.update(d)
        return out

    # ================================================================ scatter
    def scatterArray(self, arrData, operand: Operand, recvfroms: Sequence[int], recvtos: Sequence[int],
                     rootRank: int):
        if self._fast_ar and type(recvfroms) is list and type(recvtos) is list and \
                self._fast_plan_call("scatter", arrData, (tuple(recvfroms), tuple(recvtos), rootRank)):
            return arrData
        self._tick("scatterArray")
        self._check_len(recvfroms, "recvfroms")
        self._check_len(recvtos, "recvtos")
        if self.slaveNum == 1:
            return arrData
        CommUtils.isfromsTosLegal(recvfroms, recvtos)
        self._check_root(rootRank)
        if _is_device_tensor(arrData):
            return self.device.scatter(arrData, list(recvfroms), list(recvtos), rootRank,
                                       memo=self._fast_ar is not None)
        buf = _host_view(arrData, operand)
        self.engine.tree_scatter(buf, recvfroms, recvtos, operand, rootRank)
        return arrData

    def scatterMap(self, mapDataList: List[Dict], operand: Operand, rootRank: int) -> Dict:
        self._tick("scatterMap")
        if self.rank == rootRank and len(mapDataList) != self.slaveNum:
            raise Mp4jException("mapDataList size must be equal to slaveNum")
        if self.slaveNum == 1:
            return mapDataList[0]
        self._check_root(rootRank)
        probe = next((d for d in mapDataList if d), {}) if self.rank == rootRank and mapDataList else {}
        if self._map_on_device(probe, all_keys=(k for m in mapDataList for k in m.keys()) if probe else None):
            return self.device.scatter_map(mapDataList if self.rank == rootRank else None, rootRank)
        blocks = [[d] for d in mapDataList] if self.rank == rootRank else None
        got = self.engine.tree_scatter_maps(blocks, operand, rootRank)
        if not got:
            raise Mp4jException("scatter error retmap must not be null!")
        return got[0]

    def scatterMapSpecial(self, mapDataListList: List[List[Dict]], operand: Operand, rootRank: int) -> List[Dict]:
        """``list[rank][t]`` → rank receives its list of T maps (reference :999-1051)."""
        if self.slaveNum == 1:
            return mapDataListList[0]
        blocks = mapDataListList if self.rank == rootRank else None
        return self.engine.tree_scatter_maps(blocks, operand, rootRank)

    # ================================================================ reduce-scatter
    def reduceScatterArray(self, arrData, operand: Operand, operator, frm: int, counts: Sequence[int]):
        fast = self._fast_ar
        tail = None
        if fast is not None and type(counts) is list:
            tail = (frm, tuple(counts), operator, operand.codec, operand.compress)
            if fast and self._fast_rs is not None and type(arrData) is self._fast_tensor and arrData.is_cuda and \
                    arrData.is_contiguous():
                base, n = arrData.data_ptr(), arrData.numel()
                try:
                    ent = fast.get(("reduce_scatter", fast.addr_key(base, n * arrData.element_size()),
                                    arrData.get_device(), n, arrData.dtype) + tail)
                except TypeError:
                    ent = tail = None
                if ent is not None and _fast_ok(self._fast_rs(ent, self._fast_stream(), base), "mp4x_ipc_fast_rs"):
                    self._fast_after(ent.stat, ent.api)
                    return arrData
        self._tick("reduceScatterArray")
        self._check_len(counts, "counts")
        if self.slaveNum == 1:
            return arrData
        CommUtils.isFromCountsLegal(frm, counts)
        froms = CommUtils.getFromsFromCount(frm, counts, self.slaveNum)
        tos = CommUtils.getTosFromCount(frm, counts, self.slaveNum)
        if _is_device_tensor(arrData):
            return self.device.reduce_scatter(arrData, froms, tos, operator, operand, memo=tail)
        buf = _host_view(arrData, operand)
        shm = self._shm_engine(buf, operand, operator, tos[-1] - froms[0])
        if shm is not None and buf.flags.c_contiguous:
            shm.reduce_scatter(buf, froms, tos, int(operand.dtype), int(operator.code))
            return arrData
        self.engine.ring_reduce_scatter(buf, froms, tos, operand, operator)
        return arrData

    def reduceScatterMap(self, mapDataList: List[Dict], operand: Operand, operator) -> Dict:
        self._tick("reduceScatterMap")
        if self.slaveNum == 1:
            return mapDataList[0]
        if len(mapDataList) != self.slaveNum:
            raise Mp4jException(f"mapDataList size={len(mapDataList)}, must be equal to slaveNum={self.slaveNum}")
        if self._map_on_device(next((d for d in mapDataList if d), {}),
                               all_keys=(k for m in mapDataList for k in m.keys())):
            return self.device.reduce_scatter_map(mapDataList, operator)
        return self.engine.ring_reduce_scatter_maps([[d] for d in mapDataList], operand, operator)[0]

    def reduceScatterMapSpecial(self, mapDataListList: List[List[Dict]], operand: Operand, operator) -> List[Dict]:
        if self.slaveNum == 1:
            return mapDataListList[0]
        if len(mapDataListList) != self.slaveNum:
            raise Mp4jException(f"mapDataListList size={len(mapDataListList)}, must be equal to slaveNum={self.slaveNum}")
        return self.engine.ring_reduce_scatter_maps(mapDataListList, operand, operator)

    # ================================================================ reduce
    def reduceArray(self, arrData, operand: Operand, operator, frm: int, to: int, rootRank: int):
        """reduce-scatter + gather (reference :1390-1421)."""
        fast = self._fast_ar
        if fast and type(arrData) is self._fast_tensor and arrData.is_cuda and arrData.is_contiguous() and \
                0 <= rootRank < self.slaveNum:
            # the latency tier of a reduce is the staged IPC allreduce (every rank gets the sum;
            # non-root results are unspecified by contract): the same native launch
            base, n = arrData.data_ptr(), arrData.numel()
            ent = fast.get(("reduce", fast.addr_key(base, n * arrData.element_size()), arrData.get_device(), n, frm,
                            to, arrData.dtype, operator, operand.codec, operand.compress, 1.0))
            if ent is not None and _fast_ok(self._fast_lx(ent, self._fast_stream(), base), "mp4x_ipc_fast_allreduce"):
                self._fast_after(ent.stat, ent.api)
                return arrData
        self._tick("reduceArray")
        if self.slaveNum == 1:
            return arrData
        CommUtils.isFromToLegal(frm, to)
        self._check_root(rootRank)
        if _is_device_tensor(arrData):
            return self.device.reduce(arrData, frm, to, operator, operand, rootRank, memo=self._fast_ar is not None)
        buf = _host_view(arrData, operand)
        shm = self._shm_engine(buf, operand, operator, to - frm)
        if shm is not None and buf.flags.c_contiguous:
            # non-root results are unspecified by contract; the shm allreduce serves the root
            shm.allreduce(buf, frm, to, int(operand.dtype), int(operator.code))
            return arrData
        froms, tos, _ = CommUtils.even_split(frm, to, self.slaveNum)
        self.engine.ring_reduce_scatter(buf, froms, tos, operand, operator)
        self.engine.tree_gather(buf, froms, tos, operand, rootRank)
        return arrData

    def reduce(self, value, operand: Operand, operator, rootRank: int):
        self._tick("reduce")
        if self.slaveNum == 1:
            return value
        arr = operand.box(value)
        self.reduceArray(arr, operand, operator, 0, 1, rootRank)
        return operand.unbox(arr)

    def _partition(self, mapData: Dict) -> List[Dict]:
        """p maps by the reference's owner rule ``key.hashCode() % p`` (utils/hashing.owner_of),
        in ONE native walk for str keys (csrc/pyext/hostmap_ext.cpp ``partition``)."""
        p = self.slaveNum
        if type(mapData) is dict and mapData:
            from ..ops import native
            ext = native.hostmap_ext()
            parts = ext.partition(mapData, p) if ext is not None else None
            if parts is not None:
                return parts
        parts: List[Dict] = [{} for _ in range(p)]
        for k, v in mapData.items():
            parts[owner_of(k, p)][k] = v
        return parts

    def reduceMap(self, mapData: Dict, operand: Operand, operator, rootRank: int) -> Dict:
        """hash-partition → reduceScatterMap → gatherMap (reference :1490-1516)."""
        self._tick("reduceMap")
        if self.slaveNum == 1:
            return mapData
        self._check_root(rootRank)
        if self._map_on_device(mapData):
            return self.device.reduce_map(mapData, operator, rootRank)
        mine = self.engine.ring_reduce_scatter_maps([[d] for d in self._partition(mapData)], operand, operator)[0]
        return self.engine.tree_gather_map(mine, operand, rootRank)

    # ---- set / list specials (reference :1518-1720, :2099-2230)
    @staticmethod
    def _set_operand(elementSerializer=None) -> Operand:
        return Operands.OBJECT_OPERAND(elementSerializer or DEFAULT_SERIALIZER)

    _UNION = CustomOperator(lambda a, b: set(a) | set(b), name="set_union")
    _INTERSECT = CustomOperator(lambda a, b: set(a) & set(b), name="set_intersection")
    _CONCAT = CustomOperator(lambda a, b: list(a) + list(b), name="list_concat")

    def reduceMapSetUnion(self, mapData: Dict, rootRank: int, elementSerializer=None, elementType=None) -> Dict:
        return self.reduceMap(mapData, self._set_operand(elementSerializer), self._UNION, rootRank)

    def reduceSetUnion(self, setData, rootRank: int, elementSerializer=None, elementType=None):
        r = self.reduceMapSetUnion({"key": setData}, rootRank, elementSerializer, elementType)
        return None if r is None else r.get("key")

    def reduceMapSetIntersection(self, mapData: Dict, rootRank: int, elementSerializer=None, elementType=None) -> Dict:
        return self.reduceMap(mapData, self._set_operand(elementSerializer), self._INTERSECT, rootRank)

    def reduceSetIntersection(self, setData, rootRank: int, elementSerializer=None, elementType=None):
        r = self.reduceMapSetIntersection({"key": setData}, rootRank, elementSerializer, elementType)
        return None if r is None else r.get("key")

    def reduceMapListConcat(self, mapData: Dict, rootRank: int, elementSerializer=None, elementType=None) -> Dict:
        return self.reduceMap(mapData, self._set_operand(elementSerializer), self._CONCAT, rootRank)

    def reduceListConcat(self, listData, rootRank: int, elementSerializer=None, elementType=None):
        r = self.reduceMapListConcat({"key": listData}, rootRank, elementSerializer, elementType)
        return None if r is None else r.get("key")

    def allreduceMapSetUnion(self, mapData: Dict, elementSerializer=None, elementType=None) -> Dict:
        return self.allreduceMap(mapData, self._set_operand(elementSerializer), self._UNION)

    def allreduceSetUnion(self, setData, elementSerializer=None, elementType=None):
        if _is_torch(setData):   # int64 id tensor → GPU K7 path
            from .sparse import set_union
            return setData if self.slaveNum == 1 else set_union(self.device, setData)
        return self.allreduceMapSetUnion({"key": setData}, elementSerializer, elementType).get("key")

    def allreduceMapSetIntersection(self, mapData: Dict, elementSerializer=None, elementType=None) -> Dict:
        return self.allreduceMap(mapData, self._set_operand(elementSerializer), self._INTERSECT)

    def allreduceSetIntersection(self, setData, elementSerializer=None, elementType=None):
        if _is_torch(setData):
            from .sparse import set_intersection
            return setData if self.slaveNum == 1 else set_intersection(self.device, setData)
        return self.allreduceMapSetIntersection({"key": setData}, elementSerializer, elementType).get("key")

    def allreduceMapListConcat(self, mapData: Dict, elementSerializer=None, elementType=None) -> Dict:
        return self.allreduceMap(mapData, self._set_operand(elementSerializer), self._CONCAT)

    def allreduceListConcat(self, listData, elementSerializer=None, elementType=None):
        if _is_torch(listData):
            from .sparse import list_concat
            return listData if self.slaveNum == 1 else list_concat(self.device, listData)
        return self.allreduceMapListConcat({"key": listData}, elementSerializer, elementType).get("key")

    @staticmethod
    def _check_key_bits(keys, keyBits):
        if keyBits is None:
            return None
        keyBits = int(keyBits)
        if not 1 <= keyBits <= 63:
            raise Mp4jException(f"keyBits {keyBits} outside [1, 63]")
        if keys.numel() and (int(keys.min()) < 0 or int(keys.max()) >= (1 << keyBits)):
            raise Mp4jException(f"keys outside [0, 2**{keyBits}) with keyBits={keyBits}")
        return keyBits

    def allreduceSparse(self, keys, vals, operator, keyBits: Optional[int] = None):
        """Sparse allreduce of (int64 id, value-row) pairs on the device engine (extension).

        Every rank returns ``(keys, vals)`` holding the op-reduction over all ranks of the rows
        sharing an id (the tensor form of ``allreduceMap`` for ``Map<String, float[]>``).
        ``keyBits``: ids are known to lie in [0, 2**keyBits) (e.g. embedding rows), so the
        reduce-by-key radix sort covers only those bits.
        """
        self._tick("allreduceSparse")
        if self.slaveNum == 1:
            return keys, vals
        from .sparse import allreduce_sparse
        return allreduce_sparse(self.device, keys, vals, operator, self._check_key_bits(keys, keyBits))

    def reduceSparse(self, keys, vals, operator, rootRank: int, keyBits: Optional[int] = None):
        """Tensor form of ``reduceMap``: root gets the op-reduced union (others: their owned share)."""
        self._tick("reduceSparse")
        if self.slaveNum == 1:
            return keys, vals
        self._check_root(rootRank)
        from .sparse import reduce_sparse
        return reduce_sparse(self.device, keys, vals, operator, rootRank, self._check_key_bits(keys, keyBits))

    def gatherSparse(self, keys, vals, rootRank: int):
        """Tensor form of ``gatherMap``: union at root, duplicate ids keep the lowest rank's row (K8)."""
        self._tick("gatherSparse")
        if self.slaveNum == 1:
            return keys, vals
        self._check_root(rootRank)
        from .sparse import gather_sparse
        return gather_sparse(self.device, keys, vals, rootRank)

    def allgatherSparse(self, keys, vals):
        """Tensor form of ``allgatherMap``: (keys, rows, per-rank counts) concatenated in rank order."""
        self._tick("allgatherSparse")
        if self.slaveNum == 1:
            return keys, vals, [int(keys.shape[0])]
        from .sparse import allgather_sparse
        return allgather_sparse(self.device, keys, vals)

    def broadcastSparse(self, keys, vals, rootRank: int):
        """Tensor form of ``broadcastMap``: root's (keys, rows) everywhere (non-root inputs may be None)."""
        self._tick("broadcastSparse")
        if self.slaveNum == 1:
            return keys, vals
        self._check_root(rootRank)
        from .sparse import broadcast_sparse
        return broadcast_sparse(self.device, keys, vals, rootRank)

    def alltoallArray(self, sendData, sendCounts: Sequence[int], recvData=None):
        """Ragged all-to-all of a device tensor (extension; the exchange behind the sparse map
        collectives, exposed for expert-parallel style routing).  ``sendData`` rows are grouped
        by destination rank with ``sendCounts[j]`` rows for rank j.  Returns ``(recv, recvCounts)``
        with rows grouped by source rank (RCCL all-to-all, every link at once)."""
        self._tick("alltoallArray")
        self._check_len(sendCounts, "sendCounts")
        if not _is_torch(sendData):
            raise Mp4jException("alltoallArray needs a torch tensor (device engine)")
        return self.device.all_to_all_v(sendData, list(sendCounts), recvData)

    # ================================================================ allreduce
    def allreduceArray(self, arrData, operand: Operand, operator, frm: int, to: int, out=None, scale: float = 1.0):
        """reduce-scatter + allgather with the last rank taking the remainder (reference :1733-1763).

        ``out`` (extension): out-of-place form — ``out[from:to]`` receives the result and
        ``arrData`` is left untouched (with one rank this is a plain copy).
        ``scale`` (extension, float data): the result is multiplied by it — e.g. ``1/p`` for a
        gradient average; on the device it is fused into the collective's final write.
        """
        fast = self._fast_ar
        if fast and out is None and type(arrData) is self._fast_tensor and arrData.is_cuda and arrData.is_contiguous():
            base, n = arrData.data_ptr(), arrData.numel()
            ent = fast.get((fast.addr_key(base, n * arrData.element_size()), arrData.get_device(), n, frm, to,
                            arrData.dtype, operator, operand.codec, operand.compress, scale))
            if ent is not None:
                rc = self._fast_lx(ent, self._fast_stream(), base)
                if rc == 0 or _fast_ok(rc, "mp4x_ipc_fast_allreduce"):
                    self._fast_after(ent.stat, ent.api)
                    return arrData
            # not memoised, or not launched (rc 1003: an earlier collective failed; 1004: the stream
            # is being captured; 1001 / 1002: refused): the full path decides, raises or records
        self._tick("allreduceArray")
        if scale != 1.0:
            if _is_device_tensor(arrData) and self.slaveNum > 1:
                CommUtils.isFromToLegal(frm, to)
                return self.device.allreduce(arrData, frm, to, operator, operand, out=out, scale=scale,
                                             memo=out is None)
            res = self.allreduceArray(arrData, operand, operator, frm, to, out=out)
            tgt = res.view(-1)[frm:to] if _is_torch(res) else res[frm:to]
            tgt *= scale
            return res
        if out is not None and self.slaveNum > 1 and _is_device_tensor(out) and _is_device_tensor(arrData):
            # the device engine writes the result straight into ``out`` (no copy-then-in-place)
            CommUtils.isFromToLegal(frm, to)
            return self.device.allreduce(arrData, frm, to, operator, operand, out=out)
        if out is not None:
            CommUtils.isFromToLegal(frm, to)
            if _is_device_tensor(out):
                # the local data movement of an out-of-place allreduce runs through the K1 kernel
                from ..ops.device_ops import reduce_
                from ..operators import OpCode
                if to > frm:
                    reduce_(out.view(-1)[frm:to], [arrData.view(-1)[frm:to]], int(OpCode.SUM))
            elif _is_torch(out):
                out.view(-1)[frm:to].copy_(arrData.view(-1)[frm:to])
            else:
                out[frm:to] = arrData[frm:to]
            if self.slaveNum == 1:
                return out
            arrData = out
        if self.slaveNum == 1:
            return arrData
        CommUtils.isFromToLegal(frm, to)
        if _is_device_tensor(arrData):
            return self.device.allreduce(arrData, frm, to, operator, operand, memo=self._fast_ar is not None)
        buf = _host_view(arrData, operand)
        shm = self._shm_engine(buf, operand, operator, to - frm)
        if shm is not None and buf.flags.c_contiguous:
            shm.allreduce(buf, frm, to, int(operand.dtype), int(operator.code))
            return arrData
        nbytes = (to - frm) * (buf.itemsize if isinstance(buf, np.ndarray) else 64)
        if choose_allreduce(self.slaveNum, nbytes, getattr(operator, "is_custom", False)) == "rhd":
            self.engine.rhd_allreduce(buf, frm, to, operand, operator)
            return arrData
        froms, tos, _ = CommUtils.even_split(frm, to, self.slaveNum)
        self.engine.ring_reduce_scatter(buf, froms, tos, operand, operator)
        self.engine.ring_allgather(buf, froms, tos, operand)
        return arrData

    def allreduce(self, value, operand: Operand, operator):
        self._tick("allreduce")
        if self.slaveNum == 1:
            return value
        arr = operand.box(value)
        self.allreduceArray(arr, operand, operator, 0, 1)
        return operand.unbox(arr)

    def allreduceArrayRpc(self, arrData, operand: Operand, operator):
        """Small-data allreduce through the master (reference :1776-1926, Server.java:373-514).

        Every rank uploads its whole array; the master returns all p copies in
        RANK order; each rank folds them locally (op(op(r0, r1), r2) ...).  For
        device tensors the latency path is the device engine's small-message
        allreduce instead.
        """
        self._tick("allreduceArrayRpc")
        if self.slaveNum == 1:
            return arrData
        if _is_device_tensor(arrData):
            return self.device.allreduce(arrData, 0, arrData.numel(), operator, operand, small=True)
        buf = _host_view(arrData, operand)
        if operand.is_primitive:
            payload = np.ascontiguousarray(buf).tobytes()
        else:
            payload = operand.serializer.write_list(buf)
        copies = self.server.call("rpc_allreduce", self.rank, payload)
        if operand.is_primitive:
            acc = np.frombuffer(copies[0], dtype=operand.np_dtype).copy()
            for c in copies[1:]:
                x = np.frombuffer(c, dtype=operand.np_dtype)
                with np.errstate(over="ignore", invalid="ignore"):
                    operator.reduce_into(acc, x)
            buf[:] = acc
        else:
            acc = operand.serializer.read_list(copies[0])
            for c in copies[1:]:
                x = operand.serializer.read_list(c)
                acc = [operator.apply(a, b) for a, b in zip(acc, x)]
            buf[:] = acc
        return arrData

    def allreduceRpc(self, value, operand: Operand, operator):
        self._tick("allreduceRpc")
        if self.slaveNum == 1:
            return value
        arr = operand.box(value)
        self.allreduceArrayRpc(arr, operand, operator)
        return operand.unbox(arr)

    def allreduceMap(self, mapData: Dict, operand: Operand, operator) -> Dict:
        """partition → reduceScatterMap → allgatherMap → merge (reference :2053-2088)."""
        self._tick("allreduceMap")
        if self.slaveNum == 1:
            return mapData
        if self._map_on_device(mapData):
            return self.device.allreduce_map(mapData, operator)
        from . import hostmap
        if HOST_MAP_COLUMNAR and hostmap.supported(operand, operator):
            # primitive values: keys + one value column per block, vectorised owner merge
            return hostmap.allreduce_map(self.engine, mapData, operand, operator)
        mine = self.engine.ring_reduce_scatter_maps([[d] for d in self._partition(mapData)], operand, operator)
        allb = self.engine.ring_allgather_maps(mine, operand)
        out: Dict = {}
        for blk in allb:
            for d in blk:
                out.update(d)
        return out

    # ================================================================ helpers
    def _check_root(self, root: int):
        if not (0 <= root < self.slaveNum):
            raise RangeError(f"root rank {root} out of range [0, {self.slaveNum})")

    # torch-style conveniences ---------------------------------------------------
    def allreduce_tensor(self, tensor, operator=None, operand: Optional[Operand] = None):
        """Whole-tensor in-place allreduce (flattened view), SUM by default."""
        from ..operators import Operators
        op = operator or Operators.Float.SUM
        flat = tensor.view(-1) if _is_torch(tensor) else tensor.reshape(-1)
        opnd = operand or Operands.FLOAT_OPERAND()
        self.allreduceArray(flat, opnd, op, 0, flat.shape[0])
        return tensor


def _nbytes(x) -> int:
    if isinstance(x, np.ndarray):
        return int(x.nbytes)
    if _is_torch(x):
        return int(x.numel() * x.element_size())
    if isinstance(x, (list, dict, set)):
        return len(x)
    return 0


def _traced(name, fn):
    def wrapper(self, *args, **kwargs):
        a0 = args[0] if args else None
        tr = self.tracer
        if not tr.enabled:                       # counters only: keep the latency tier lean
            tr.count(name, _nbytes(a0))
            return fn(self, *args, **kwargs)
        with tr.span(name, _nbytes(a0), a0 if _is_device_tensor(a0) else None):
            return fn(self, *args, **kwargs)
    wrapper.__name__ = fn.__name__
    wrapper.__doc__ = fn.__doc__
    wrapper.__wrapped__ = fn
    return wrapper


_TRACED = ["gatherArray", "gatherMap", "allgatherArray", "allgatherMap", "broadcastArray", "broadcastMap",
           "scatterArray", "scatterMap", "reduceScatterArray", "reduceScatterMap", "reduceArray", "reduceMap",
           "allreduceArray", "allreduceArrayRpc", "allreduceMap", "allreduceSparse", "barrier"]
for _n in _TRACED:
    setattr(ProcessCommSlave, _n, _traced(_n, getattr(ProcessCommSlave, _n)))


def _trace_report(self):
    """Per-collective calls / bytes / host ms (+ device ms and algorithm mix with MP4X_TRACE=1)."""
    rep = self.tracer.report()
    if self._device_engine is not None:
        rep["_device_algorithms"] = dict(self._device_engine.stats)
    return rep


ProcessCommSlave.trace_report = _trace_report


# snake_case aliases --------------------------------------------------------------
def _snake(name: str) -> str:
    out = []
    for i, ch in enumerate(name):
        if ch.isupper() and i > 0:
            out.append("_")
        out.append(ch.lower())
    return "".join(out)


for _n in [n for n in dir(ProcessCommSlave) if not n.startswith("_")]:
    _sn = _snake(_n)
    if _sn != _n and not hasattr(ProcessCommSlave, _sn):
        setattr(ProcessCommSlave, _sn, getattr(ProcessCommSlave, _n))

ProcessComm = ProcessCommSlave
