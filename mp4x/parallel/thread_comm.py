"""ThreadComm — T worker threads per process on top of one ProcessComm.

Public API = the reference's ``ThreadCommSlave``
(/root/reference/src/main/java/com/fenbi/mp4j/comm/ThreadCommSlave.java): every
collective ``X`` has a hierarchical form taking ``[slaveNum][threadNum]`` range
tables and ``(rootRank, rootThreadId)``, plus an ``XProcess`` pass-through
that a single thread per process calls.

Choreography:

* thread phase — the T threads' contributions are combined into the *root
  thread* ``rt = rootThreadId if rank == rootRank else 0``
  (ThreadCommSlave.java:486).  The reference pairs threads through a
  ``java.util.concurrent.Exchanger`` tree and lets one thread of each pair
  do the whole reduce (:259-303).  Here the reduction is DATA-PARALLEL: every
  thread reduces its own 1/T slice of the range across all T inputs
  (numpy releases the GIL, so the slices run concurrently); for GPU tensors
  ``rt`` issues ONE multi-input HIP reduce kernel (K1b, ``NIN = T``);
* process phase — ``rt`` alone runs the ProcessComm collective (RCCL /
  TCP communicators are driven from a single thread);
* distribution — the other threads copy their slice / the whole array from
  ``rt`` (``threadCopy`` / ``threadArrayAllCopy``) or share the same Map object.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..exceptions import Mp4jException
from ..operands import Operand, Operands
from ..utils.commutils import CommUtils
from .process_comm import ProcessCommSlave, _is_device_tensor, _is_torch, _host_view
from . import wire


def _chunk(f: int, t: int, parts: int, i: int):
    avg = (t - f) // parts
    cf = f + i * avg
    ct = t if i == parts - 1 else cf + avg
    return cf, ct


class _TeamBarrier:
    """The thread barrier of a ThreadCommSlave: the native thread team (csrc/host/host_ops.cpp
    ``mp4x_team_*``) whose spin barrier both the Python-level choreography and the native
    host-array thread reductions use (GIL released while waiting); ``threading.Barrier`` when
    the host library is unavailable.  ``abort()`` breaks it, so a failing thread never leaves
    its peers waiting."""

    def __init__(self, n: int):
        self._py = threading.Barrier(n)
        self.team = None
        self._lib = None
        self.ext = None          # CPython binding of the team (csrc/pyext/team_ext.cpp), if built
        if n > 1:
            try:
                from ..ops import native
                self._lib = native.host()
                self.team = self._lib.mp4x_team_create(n, 0.0)
                self.ext = native.team_ext() if _TEAM_ON else None
            except Exception:
                self.team = None

    def wait(self, tid: int = 0):
        if self.team:            # the same native barrier the team phases use (GIL released)
            rc = self.ext.barrier(self.team, tid) if self.ext else self._lib.mp4x_team_barrier(self.team, tid)
            if rc:
                raise threading.BrokenBarrierError("thread barrier aborted")
            return 0
        return self._py.wait()

    def abort(self):
        self._py.abort()
        if self.team:
            self._lib.mp4x_team_abort(self.team)

    @property
    def broken(self) -> bool:
        if self.team:
            return bool(self._lib.mp4x_team_aborted(self.team))
        return self._py.broken

    def __del__(self):
        try:
            if self.team:
                self._lib.mp4x_team_destroy(self.team)
        except Exception:
            pass


_TEAM_DTYPES = None
_TEAM_ON = __import__("os").environ.get("MP4X_THREAD_TEAM", "1") == "1"
_EXT_NOT_ELIGIBLE, _EXT_OUT_OF_RANGE = -100, -101      # csrc/pyext/team_ext.cpp


def _team_dtype(buf, operator):
    """Native dtype code when ``buf`` / ``operator`` can take the native thread-team path."""
    global _TEAM_DTYPES
    if not isinstance(buf, np.ndarray) or buf.ndim != 1 or not buf.flags.c_contiguous:
        return None
    if getattr(operator, "is_custom", False) or not hasattr(operator, "code"):
        return None
    if _TEAM_DTYPES is None:
        from ..operators import DType
        _TEAM_DTYPES = {np.dtype(np.float64): int(DType.F64), np.dtype(np.float32): int(DType.F32),
                        np.dtype(np.int64): int(DType.I64), np.dtype(np.int32): int(DType.I32),
                        np.dtype(np.int16): int(DType.I16), np.dtype(np.int8): int(DType.I8)}
    dt = _TEAM_DTYPES.get(buf.dtype)
    if dt is None or int(getattr(operator, "dtype", dt)) != dt:
        return None
    return dt


_OPINFO: Dict[int, tuple] = {}


def _op_team_info(operator):
    """``(operator, op code, dtype code)`` of a built-in operator (cached by identity), or None
    for a custom one: what the native team binding takes."""
    e = _OPINFO.get(id(operator))
    if e is not None and e[0] is operator:
        return e
    if getattr(operator, "is_custom", False) or getattr(operator, "code", None) is None:
        return None
    if len(_OPINFO) > 4096:
        _OPINFO.clear()
    e = _OPINFO[id(operator)] = (operator, int(operator.code), int(operator.dtype))
    return e


class ThreadCommSlave:
    """Process × thread communicator (reference ``ThreadCommSlave``)."""

    def __init__(self, loginName: Optional[str], threadNum: int, masterHost: str = "127.0.0.1",
                 masterPort: int = 61235, *, process_comm: Optional[ProcessCommSlave] = None, **kw):
        if threadNum < 1:
            raise Mp4jException("threadNum must be >= 1")
        self.threadNum = threadNum
        self._barrier = _TeamBarrier(threadNum)
        self.processCommSlave = process_comm or ProcessCommSlave(loginName, masterHost, masterPort, **kw)
        self.rank = self.processCommSlave.getRank()
        self.slaveNum = self.processCommSlave.getSlaveNum()
        self._tls = threading.local()
        self._slots: List[object] = [None] * threadNum
        self._delegate = None
        self._close_lock = threading.Lock()
        self._isClosed = False

    # ------------------------------------------------------------------ basics
    def getThreadNum(self) -> int:
        return self.threadNum

    def isClosed(self) -> bool:
        return self._isClosed

    def setThreadId(self, threadId: int) -> None:
        if not (0 <= threadId < self.threadNum):
            raise Mp4jException(f"threadId {threadId} out of range")
        self._tls.tid = threadId

    def getThreadId(self) -> int:
        return getattr(self._tls, "tid", 0)

    def threadBarrier(self) -> None:
        try:
            self._barrier.wait(self.getThreadId())
        except threading.BrokenBarrierError as e:
            raise Mp4jException("thread barrier broken") from e

    def abort(self) -> None:
        """Break the thread barriers (a failing thread releases its peers with an error)."""
        self._barrier.abort()

    def _team_fail(self, rc: int, frm: int, to: int):
        self._barrier.abort()
        if rc == _EXT_OUT_OF_RANGE:
            CommUtils.isFromToLegal(frm, to)
            raise Mp4jException(f"[{frm}, {to}) is out of the array's bounds")
        raise Mp4jException(f"thread team collective failed ({rc})")

    def _team_call(self, fn, *args) -> None:
        rc = fn(self._barrier.team, self.getThreadId(), *args)
        if rc:
            self._barrier.abort()
            raise Mp4jException(f"thread team collective failed ({rc})")

    def barrier(self) -> None:
        self.threadBarrier()
        if self.getThreadId() == 0:
            self.processCommSlave.barrier()
        self.threadBarrier()

    def getRank(self) -> int:
        return self.rank

    def getSlaveNum(self) -> int:
        return self.slaveNum

    def info(self, s: str, onlyRank0Thread0: bool = True) -> None:
        if onlyRank0Thread0:
            if self.getThreadId() == 0:
                self.processCommSlave.info(s)
        else:
            self.processCommSlave.info(f"[threadId={self.getThreadId()}] {s}", False)

    def debug(self, s: str, onlyRank0Thread0: bool = True) -> None:
        if onlyRank0Thread0:
            if self.getThreadId() == 0:
                self.processCommSlave.debug(s)
        else:
            self.processCommSlave.debug(f"[threadId={self.getThreadId()} ] {s}", False)

    def error(self, s: str) -> None:
        self.processCommSlave.error(s)

    def exception(self, e: BaseException) -> None:
        self.processCommSlave.exception(e)

    def close(self, code: int = 0) -> None:
        with self._close_lock:
            if not self._isClosed:
                self.processCommSlave.close(code)
                self._isClosed = True

    @property
    def process(self) -> ProcessCommSlave:
        return self.processCommSlave

    def registerBuffer(self, tensor) -> bool:
        """Pass-through to ``ProcessCommSlave.registerBuffer`` (one thread per process, collective
        over the processes): the tensor the process phase allreduces (the root thread's) runs
        zero-copy."""
        return self.processCommSlave.registerBuffer(tensor)

    def deregisterBuffer(self, tensor) -> None:
        self.processCommSlave.deregisterBuffer(tensor)

    def memAlloc(self, n: int, dtype=None, device=None):
        """Pass-through to ``ProcessCommSlave.memAlloc`` (one thread per process, collective over
        the processes)."""
        return self.processCommSlave.memAlloc(n, dtype, device)

    def memFree(self, tensor) -> None:
        self.processCommSlave.memFree(tensor)

    # ------------------------------------------------------------------ thread-phase primitives
    def _publish(self, obj) -> None:
        self._slots[self.getThreadId()] = obj
        self.threadBarrier()

    def _thread_reduce_array(self, arr, operand: Operand, operator, f: int, t: int, rt: int):
        """All T arrays' [f, t) reduced into thread rt's array (rt's value first, then threads in order)."""
        tid = self.getThreadId()
        ext = self._barrier.ext
        if ext is not None and type(arr) is np.ndarray:
            oi = _op_team_info(operator)
            if oi is not None:
                self._slots[tid] = arr
                rc = ext.reduce(self._barrier.team, tid, arr, f, t, oi[2], oi[1], rt)
                if rc == 0:
                    return self._slots[rt]
                if rc != _EXT_NOT_ELIGIBLE:
                    self._team_fail(rc, f, t)
        if self._barrier.team and _TEAM_ON and not _is_device_tensor(arr):
            buf = _host_view(arr, operand)
            dt = _team_dtype(buf, operator)
            if dt is not None:     # native: publish + chunked reduce into rt's buffer + barrier
                self._slots[tid] = arr
                self._team_call(self._barrier._lib.mp4x_team_reduce, buf.ctypes.data, f, t, dt,
                                int(operator.code), rt)
                return self._slots[rt]
        self._publish(arr)
        T = self.threadNum
        order = [j for j in range(T) if j != rt]
        root = self._slots[rt]
        if _is_device_tensor(root):
            if tid == rt:
                from .device_engine import local_reduce
                local_reduce(root, [self._slots[j] for j in order], f, t, operator)
        else:
            bufs = [_host_view(self._slots[j], operand) for j in range(T)]
            cf, ct = _chunk(f, t, T, tid)
            if ct > cf:
                acc = bufs[rt]
                if isinstance(acc, np.ndarray):
                    with np.errstate(over="ignore", invalid="ignore"):
                        for j in order:
                            operator.reduce_into(acc[cf:ct], bufs[j][cf:ct])
                else:
                    for i in range(cf, ct):
                        v = acc[i]
                        for j in order:
                            v = operator.apply(v, bufs[j][i])
                        acc[i] = v
        self.threadBarrier()
        return root

    def _thread_merge_array(self, arr, operand: Operand, segs: Sequence, rt: int):
        """Each thread t copies its segment segs[t] = (from, to) into thread rt's array."""
        tid = self.getThreadId()
        self._publish(arr)
        root = self._slots[rt]
        f, t = segs[tid]
        if tid != rt and t > f:
            _copy_range(root, arr, f, t)
        self.threadBarrier()
        return root

    def _thread_reduce_maps(self, maps: List[Dict], operator, rt: int) -> Optional[List[Dict]]:
        """Per-position map reduce of every thread's list of maps into a copy at rt."""
        tid = self.getThreadId()
        self._publish(maps)
        out = None
        if tid == rt:
            out = [dict(m) for m in self._slots[rt]]
            for j in range(self.threadNum):
                if j == rt:
                    continue
                for pos, m in enumerate(self._slots[j]):
                    if _tensor_valued(m) or _tensor_valued(out[pos]):
                        _merge_reduce_tensors(out[pos], m, operator)
                        continue
                    keys, vals = _map_kv(m, operator)
                    wire.merge_reduce(out[pos], keys, vals, operator)
        self.threadBarrier()
        return out

    def _thread_merge_maps(self, m: Dict, rt: int) -> Optional[Dict]:
        tid = self.getThreadId()
        self._publish(m)
        out = None
        if tid == rt:
            out = {}
            for j in range(self.threadNum):
                out.update(self._slots[j])
        self.threadBarrier()
        return out

    def _distribute(self, value, rt: int):
        """rt publishes ``value``; everyone returns it after the barrier."""
        if self.getThreadId() == rt:
            self._delegate = value
        self.threadBarrier()
        v = self._delegate
        self.threadBarrier()
        return v

    # ================================================================== gather
    def gatherArray(self, arrData, operand: Operand, sendfroms, sendtos, rootRank: int, rootThreadId: int):
        self._check2d(sendfroms, sendtos, "sendfroms", "sendtos")
        pf, pt = CommUtils.getProcessFroms(sendfroms), CommUtils.getProcessTos(sendtos)
        if self.threadNum == 1:
            return self.processCommSlave.gatherArray(arrData, operand, pf, pt, rootRank)
        rt = rootThreadId if self.rank == rootRank else 0
        segs = list(zip(sendfroms[self.rank], sendtos[self.rank]))
        root = self._thread_merge_array(arrData, operand, segs, rt)
        res = None
        if self.getThreadId() == rt:
            res = self.processCommSlave.gatherArray(root, operand, pf, pt, rootRank)
        self.threadBarrier()
        if self.getThreadId() == rt and self.rank == rootRank:
            return res
        return arrData

    def gatherMap(self, mapData: Dict, operand: Operand, rootRank: int, rootThreadId: int) -> Dict:
        if self.threadNum == 1:
            return self.processCommSlave.gatherMap(mapData, operand, rootRank)
        rt = rootThreadId if self.rank == rootRank else 0
        merged = self._thread_merge_maps(mapData, rt)
        res = None
        if self.getThreadId() == rt:
            res = self.processCommSlave.gatherMap(merged, operand, rootRank)
        self.threadBarrier()
        if self.getThreadId() == rt and self.rank == rootRank:
            return res
        return mapData

    # ================================================================== allgather
    def allgatherArray(self, arrData, operand: Operand, sendfroms, sendtos):
        self._check2d(sendfroms, sendtos, "sendfroms", "sendtos")
        pf, pt = CommUtils.getProcessFroms(sendfroms), CommUtils.getProcessTos(sendtos)
        if self.threadNum == 1:
            return self.processCommSlave.allgatherArray(arrData, operand, pf, pt)
        segs = list(zip(sendfroms[self.rank], sendtos[self.rank]))
        root = self._thread_merge_array(arrData, operand, segs, 0)
        if self.getThreadId() == 0:
            self.processCommSlave.allgatherArray(root, operand, pf, pt)
        self.threadBarrier()
        if self.getThreadId() != 0:
            _copy_all(arrData, root)   # reference threadArrayAllCopy (whole array)
        self.threadBarrier()
        return arrData

    def allgatherMap(self, mapData: Dict, operand: Operand) -> List[Dict]:
        if self.threadNum == 1:
            return self.processCommSlave.allgatherMap(mapData, operand)
        merged = self._thread_merge_maps(mapData, 0)
        res = None
        if self.getThreadId() == 0:
            res = self.processCommSlave.allgatherMap(merged, operand)
        return self._distribute(res, 0)  # shared list (reference :757)

    # ================================================================== broadcast
    def broadcastArray(self, arrData, operand: Operand, frm: int, to: int, rootRank: int, rootThreadId: int):
        if self.threadNum == 1:
            return self.processCommSlave.broadcastArray(arrData, operand, frm, to, rootRank)
        rt = rootThreadId if self.rank == rootRank else 0
        self._publish(arrData)
        root = self._slots[rt]
        if self.getThreadId() == rt:
            self.processCommSlave.broadcastArray(root, operand, frm, to, rootRank)
        self.threadBarrier()
        if self.getThreadId() != rt:
            _copy_all(arrData, root)
        self.threadBarrier()
        return arrData

    def broadcast(self, value, operand: Operand, rootRank: int, rootThreadId: int):
        arr = operand.box(value)
        self.broadcastArray(arr, operand, 0, 1, rootRank, rootThreadId)
        return operand.unbox(arr)

    def broadcastMap(self, mapData: Dict, operand: Operand, rootRank: int, rootThreadId: int) -> Dict:
        if self.threadNum == 1:
            return self.processCommSlave.broadcastMap(mapData, operand, rootRank)
        rt = rootThreadId if self.rank == rootRank else 0
        res = None
        if self.getThreadId() == rt:
            res = self.processCommSlave.broadcastMap(mapData, operand, rootRank)
        return self._distribute(res, rt)

    # ================================================================== scatter
    def scatterArray(self, arrData, operand: Operand, recvfroms, recvtos, rootRank: int, rootThreadId: int):
        self._check2d(recvfroms, recvtos, "recvfroms", "recvtos")
        pf, pt = CommUtils.getProcessFroms(recvfroms), CommUtils.getProcessTos(recvtos)
        if self.threadNum == 1:
            return self.processCommSlave.scatterArray(arrData, operand, pf, pt, rootRank)
        rt = rootThreadId if self.rank == rootRank else 0
        self._publish(arrData)
        root = self._slots[rt]
        tid = self.getThreadId()
        if tid == rt:
            self.processCommSlave.scatterArray(root, operand, pf, pt, rootRank)
        self.threadBarrier()
        if tid != rt:
            _copy_range(arrData, root, recvfroms[self.rank][tid], recvtos[self.rank][tid])
        self.threadBarrier()
        return arrData

    def scatterMap(self, mapDataListList, operand: Operand, rootRank: int, rootThreadId: int) -> Dict:
        tid = self.getThreadId()
        if self.rank == rootRank and tid == rootThreadId and len(mapDataListList) != self.slaveNum:
            raise Mp4jException(f"mapDataListList's size:{len(mapDataListList)} must be equal slaveNum:{self.slaveNum}!")
        if self.threadNum == 1:
            lst = [ml[0] for ml in mapDataListList] if self.rank == rootRank else None
            return self.processCommSlave.scatterMap(lst, operand, rootRank)
        rt = rootThreadId if self.rank == rootRank else 0
        res = None
        if tid == rt:
            res = self.processCommSlave.scatterMapSpecial(mapDataListList, operand, rootRank)
        lst = self._distribute(res, rt)
        return lst[tid]

    # ================================================================== reduce-scatter
    def reduceScatterArray(self, arrData, operand: Operand, operator, frm: int, counts):
        if len(counts) != self.slaveNum:
            raise Mp4jException("counts.length must be equal to slaveNum!")
        CommUtils.isFromCountsLegal(frm, counts)
        if self.threadNum == 1:
            return self.processCommSlave.reduceScatterArray(arrData, operand, operator, frm,
                                                            [c[0] for c in counts])
        allto = frm + sum(sum(c) for c in counts)
        rank_from = frm + sum(sum(counts[r]) for r in range(self.rank))
        tfroms = CommUtils.getFromsFromCount(rank_from, counts[self.rank], self.threadNum)
        ttos = CommUtils.getTosFromCount(rank_from, counts[self.rank], self.threadNum)
        root = self._thread_reduce_array(arrData, operand, operator, frm, allto, 0)
        tid = self.getThreadId()
        if tid == 0:
            self.processCommSlave.reduceScatterArray(root, operand, operator, frm, [sum(c) for c in counts])
        self.threadBarrier()
        if tid != 0:
            _copy_range(arrData, root, tfroms[tid], ttos[tid])
        self.threadBarrier()
        return arrData

    def reduceScatterMap(self, mapDataListList, operand: Operand, operator) -> Dict:
        if len(mapDataListList) != self.slaveNum or any(len(l) != self.threadNum for l in mapDataListList):
            raise Mp4jException("mapDataListList dimension must be equal to slaveNum * threadNum!")
        if self.threadNum == 1:
            return self.processCommSlave.reduceScatterMap([l[0] for l in mapDataListList], operand, operator)
        flat = [m for l in mapDataListList for m in l]
        red = self._thread_reduce_maps(flat, operator, 0)
        res = None
        if self.getThreadId() == 0:
            T = self.threadNum
            blocks = [red[r * T:(r + 1) * T] for r in range(self.slaveNum)]
            res = self.processCommSlave.reduceScatterMapSpecial(blocks, operand, operator)
        lst = self._distribute(res, 0)
        return lst[self.getThreadId()]

    # ================================================================== reduce
    def reduceArray(self, arrData, operand: Operand, operator, frm: int, to: int, rootRank: int, rootThreadId: int):
        if self.threadNum == 1:
            return self.processCommSlave.reduceArray(arrData, operand, operator, frm, to, rootRank)
        CommUtils.isFromToLegal(frm, to)
        rt = rootThreadId if self.rank == rootRank else 0
        root = self._thread_reduce_array(arrData, operand, operator, frm, to, rt)
        if self.getThreadId() == rt:
            self.processCommSlave.reduceArray(root, operand, operator, frm, to, rootRank)
        self.threadBarrier()
        return arrData

    def reduce(self, value, operand: Operand, operator, rootRank: int, rootThreadId: int):
        arr = operand.box(value)
        self.reduceArray(arr, operand, operator, 0, 1, rootRank, rootThreadId)
        return operand.unbox(arr)

    def reduceMap(self, mapData: Dict, operand: Operand, operator, rootRank: int, rootThreadId: int):
        if self.threadNum == 1:
            return self.processCommSlave.reduceMap(mapData, operand, operator, rootRank)
        rt = rootThreadId if self.rank == rootRank else 0
        red = self._thread_reduce_maps([mapData], operator, rt)
        res = None
        if self.getThreadId() == rt:
            res = self.processCommSlave.reduceMap(red[0], operand, operator, rootRank)
        self.threadBarrier()
        if self.getThreadId() == rt and self.rank == rootRank:
            return res
        return None   # reference returns null for non-root threads (ThreadCommSlave.java:1583)

    # ---- set / list specials
    _UNION = ProcessCommSlave._UNION
    _INTERSECT = ProcessCommSlave._INTERSECT
    _CONCAT = ProcessCommSlave._CONCAT

    def reduceMapSetUnion(self, mapData, rootRank, rootThreadId, elementSerializer=None, elementType=None):
        return self.reduceMap(mapData, Operands.OBJECT_OPERAND(elementSerializer), self._UNION, rootRank, rootThreadId)

    def reduceSetUnion(self, setData, rootRank, rootThreadId, elementSerializer=None, elementType=None):
        r = self.reduceMapSetUnion({"key": setData}, rootRank, rootThreadId, elementSerializer)
        return None if r is None else r.get("key")

    def reduceMapSetIntersection(self, mapData, rootRank, rootThreadId, elementSerializer=None, elementType=None):
        return self.reduceMap(mapData, Operands.OBJECT_OPERAND(elementSerializer), self._INTERSECT, rootRank,
                              rootThreadId)

    def reduceSetIntersection(self, setData, rootRank, rootThreadId, elementSerializer=None, elementType=None):
        r = self.reduceMapSetIntersection({"key": setData}, rootRank, rootThreadId, elementSerializer)
        return None if r is None else r.get("key")

    def reduceMapListConcat(self, mapData, rootRank, rootThreadId, elementSerializer=None, elementType=None):
        return self.reduceMap(mapData, Operands.OBJECT_OPERAND(elementSerializer), self._CONCAT, rootRank, rootThreadId)

    def reduceListConcat(self, listData, rootRank, rootThreadId, elementSerializer=None, elementType=None):
        r = self.reduceMapListConcat({"key": listData}, rootRank, rootThreadId, elementSerializer)
        return None if r is None else r.get("key")

    def allreduceMapSetUnion(self, mapData, elementSerializer=None, elementType=None):
        return self.allreduceMap(mapData, Operands.OBJECT_OPERAND(elementSerializer), self._UNION)

    def allreduceSetUnion(self, setData, elementSerializer=None, elementType=None):
        return self.allreduceMapSetUnion({"key": setData}, elementSerializer).get("key")

    def allreduceMapSetIntersection(self, mapData, elementSerializer=None, elementType=None):
        return self.allreduceMap(mapData, Operands.OBJECT_OPERAND(elementSerializer), self._INTERSECT)

    def allreduceSetIntersection(self, setData, elementSerializer=None, elementType=None):
        return self.allreduceMapSetIntersection({"key": setData}, elementSerializer).get("key")

    def allreduceMapListConcat(self, mapData, elementSerializer=None, elementType=None):
        return self.allreduceMap(mapData, Operands.OBJECT_OPERAND(elementSerializer), self._CONCAT)

    def allreduceListConcat(self, listData, elementSerializer=None, elementType=None):
        return self.allreduceMapListConcat({"key": listData}, elementSerializer).get("key")

    # ================================================================== allreduce
    def allreduceArray(self, arrData, operand: Operand, operator, frm: int, to: int):
        if self.threadNum == 1:
            return self.processCommSlave.allreduceArray(arrData, operand, operator, frm, to)
        ext = self._barrier.ext
        if ext is not None and type(arrData) is np.ndarray:
            # the hot path (BASELINE config 1): one FASTCALL into the team per phase; the binding
            # checks the array (1-D, C-contiguous, the operator's dtype, [frm, to) in bounds)
            oi = _op_team_info(operator)
            if oi is not None:
                team, tid = self._barrier.team, getattr(self._tls, "tid", 0)
                if self.slaveNum == 1:
                    rc = ext.allreduce(team, tid, arrData, frm, to, oi[2], oi[1])
                    if rc == 0:
                        return arrData
                    if rc != _EXT_NOT_ELIGIBLE:
                        self._team_fail(rc, frm, to)
                else:
                    rc = ext.reduce(team, tid, arrData, frm, to, oi[2], oi[1], 0)
                    if rc == 0:
                        if tid == 0:
                            try:
                                self.processCommSlave.allreduceArray(arrData, operand, operator, frm, to)
                            except BaseException:
                                self._barrier.abort()
                                raise
                        rc = ext.bcast(team, tid, arrData, frm, to, oi[2], 0)
                        if rc:
                            self._team_fail(rc, frm, to)
                        return arrData
                    if rc != _EXT_NOT_ELIGIBLE:
                        self._team_fail(rc, frm, to)
        CommUtils.isFromToLegal(frm, to)
        if self._barrier.team and _TEAM_ON and not _is_device_tensor(arrData):
            buf = _host_view(arrData, operand)
            dt = _team_dtype(buf, operator)
            if dt is not None:       # native thread team through ctypes (binding not built)
                lib = self._barrier._lib
                if self.slaveNum == 1:
                    self._team_call(lib.mp4x_team_allreduce, buf.ctypes.data, frm, to, dt, int(operator.code))
                    return arrData
                self._team_call(lib.mp4x_team_reduce, buf.ctypes.data, frm, to, dt, int(operator.code), 0)
                if self.getThreadId() == 0:
                    self.processCommSlave.allreduceArray(arrData, operand, operator, frm, to)
                self._team_call(lib.mp4x_team_bcast, buf.ctypes.data, frm, to, buf.itemsize, 0)
                return arrData
        root = self._thread_reduce_array(arrData, operand, operator, frm, to, 0)
        tid = self.getThreadId()
        if tid == 0:
            self.processCommSlave.allreduceArray(root, operand, operator, frm, to)
        self.threadBarrier()
        if tid != 0:
            _copy_range(arrData, root, frm, to)
        self.threadBarrier()
        return arrData

    def allreduceArrayRpc(self, arrData, operand: Operand, operator):
        if self.threadNum == 1:
            return self.processCommSlave.allreduceArrayRpc(arrData, operand, operator)
        n = _length(arrData)
        root = self._thread_reduce_array(arrData, operand, operator, 0, n, 0)
        tid = self.getThreadId()
        if tid == 0:
            self.processCommSlave.allreduceArrayRpc(root, operand, operator)
        self.threadBarrier()
        if tid != 0:
            _copy_all(arrData, root)
        self.threadBarrier()
        return arrData

    def allreduce(self, value, operand: Operand, operator):
        arr = operand.box(value)
        self.allreduceArray(arr, operand, operator, 0, 1)
        return operand.unbox(arr)

    def allreduceRpc(self, value, operand: Operand, operator):
        arr = operand.box(value)
        self.allreduceArrayRpc(arr, operand, operator)
        return operand.unbox(arr)

    def allreduceMap(self, mapData: Dict, operand: Operand, operator) -> Dict:
        if self.threadNum == 1:
            return self.processCommSlave.allreduceMap(mapData, operand, operator)
        red = self._thread_reduce_maps([mapData], operator, 0)
        res = None
        if self.getThreadId() == 0:
            res = self.processCommSlave.allreduceMap(red[0], operand, operator)
        return self._distribute(res, 0)   # shared result map (reference :2217)

    # ================================================================== helpers
    def _check2d(self, froms, tos, nf, nt):
        if len(froms) != self.slaveNum:
            raise Mp4jException(f"{nf} array length:{len(froms)} must be equal to slaveNum:{self.slaveNum}")
        if len(tos) != self.slaveNum:
            raise Mp4jException(f"{nt} array length:{len(tos)} must be equal to slaveNum:{self.slaveNum}")
        CommUtils.isfromsTosLegal2D(froms, tos, self.threadNum)


def _tensor_valued(m: Dict) -> bool:
    return bool(m) and _is_torch(next(iter(m.values())))


def _torch_reduce_(a, b, operator) -> None:
    """a = op(a, b) in place for two equal [n, ...] tensors: ONE K1 launch on the GPU
    (``device_ops.reduce_``, every built-in op incl. the *_LOC ones), numpy's reduce on CPU
    tensors it can view, plain torch elementwise ops otherwise."""
    from ..operators import OpCode
    if a.is_cuda:
        from ..ops import device_ops
        device_ops.reduce_(a, [a, b], int(operator.code))
        return
    try:
        operator.reduce_into(a.numpy().reshape(-1), b.numpy().reshape(-1))
        return
    except (TypeError, RuntimeError):          # e.g. bf16 CPU tensors: no numpy view
        pass
    import torch
    name = {OpCode.SUM: "add", OpCode.PROD: "mul", OpCode.MAX: "maximum", OpCode.MIN: "minimum",
            OpCode.BAND: "bitwise_and", OpCode.BOR: "bitwise_or", OpCode.BXOR: "bitwise_xor"}.get(operator.code)
    if name is None:
        raise Mp4jException(f"{operator} on {a.dtype} CPU tensors is not supported")
    getattr(torch, name)(a, b, out=a)


def _merge_reduce_tensors(local: Dict, m: Dict, operator) -> None:
    """Thread-phase map merge for tensor values (reference MapReduce merge,
    J/comm/ThreadCommSlave.java:259-303): the shared keys' rows are stacked and reduced with ONE
    kernel (not one launch per key), new keys are inserted as they are.  Results of shared keys
    are row views of one fresh tensor.  Custom operators apply per key."""
    import torch
    keys = list(m.keys())
    vals = list(m.values())
    cur = list(map(local.get, keys))
    shared = [i for i, c in enumerate(cur) if c is not None]
    if shared:
        if getattr(operator, "is_custom", False):
            for i in shared:
                local[keys[i]] = operator.apply(cur[i], vals[i])
        else:
            a = torch.stack([cur[i] for i in shared])
            b = torch.stack([vals[i] for i in shared])
            if b.dtype != a.dtype or b.device != a.device:
                b = b.to(device=a.device, dtype=a.dtype)
            _torch_reduce_(a, b, operator)
            for i, row in zip(shared, a.unbind(0)):
                local[keys[i]] = row
    if len(shared) != len(keys):
        for k, c, v in zip(keys, cur, vals):
            if c is None:
                local[k] = v


def _map_kv(m: Dict, operator):
    """(keys, values) of a map in the representation wire.merge_reduce vectorises."""
    from ..operators import NP_DTYPE
    keys = list(m.keys())
    vals = list(m.values())
    if vals and not operator.is_custom and operator.dtype is not None:
        if np.isscalar(vals[0]):
            return keys, np.asarray(vals, dtype=NP_DTYPE[operator.dtype])
        if isinstance(vals[0], np.ndarray):
            return keys, wire.stack_rows(vals, NP_DTYPE[operator.dtype])
    return keys, vals


def _length(a) -> int:
    if _is_torch(a):
        return int(a.numel())
    return len(a)


def _copy_range(dst, src, f: int, t: int) -> None:
    if t <= f or dst is src:
        return
    if _is_torch(dst):
        dst[f:t].copy_(src[f:t])
    else:
        dst[f:t] = src[f:t]


def _copy_all(dst, src) -> None:
    if dst is src:
        return
    if _is_torch(dst):
        dst.copy_(src)
    else:
        dst[:] = src[:]


# *Process pass-throughs: XProcess(...) == processCommSlave.X(...) (reference :429, :526, ...)
_PROCESS_OPS = [
    "gatherArray", "gatherMap", "allgatherArray", "allgatherMap", "broadcastArray", "broadcast", "broadcastMap",
    "scatterArray", "scatterMap", "reduceScatterArray", "reduceScatterMap", "reduceArray", "reduce", "reduceMap",
    "reduceMapSetUnion", "reduceSetUnion", "reduceMapSetIntersection", "reduceSetIntersection",
    "reduceMapListConcat", "reduceListConcat", "allreduceArray", "allreduceArrayRpc", "allreduce",
    "allreduceRpc", "allreduceMap", "allreduceMapSetUnion", "allreduceSetUnion", "allreduceMapSetIntersection",
    "allreduceSetIntersection", "allreduceMapListConcat", "allreduceListConcat",
]


def _mk_passthrough(name):
    def f(self, *args, **kwargs):
        return getattr(self.processCommSlave, name)(*args, **kwargs)
    f.__name__ = name + "Process"
    f.__doc__ = f"Pass-through to ``ProcessCommSlave.{name}`` (called by one thread per process)."
    return f


for _n in _PROCESS_OPS:
    setattr(ThreadCommSlave, _n + "Process", _mk_passthrough(_n))

ThreadComm = ThreadCommSlave
