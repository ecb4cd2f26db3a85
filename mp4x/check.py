"""CommCheckTool — the reference's integration check harness as a CLI.

Reference: J/check/CommCheckTool.java:40-321 (+ 16 checks per element type in J/check/check*/).

    python -m mp4x.check <login> <masterHost> <port> <arrSize> <objSize> <runTime> \\
                         <threadNum> <process|thread> <compress> <testRpc> [--device cpu|cuda]

Every slave runs gather / scatter / allgather / reduce-scatter / broadcast / reduce /
allreduce (+ RPC allreduce) for double, float, long, int, short, byte, string and object
operands on arrays of ``arrSize`` and maps of ``objSize`` keys, ``runTime`` times each,
checks the exact expected values (deterministic inputs, as the reference does) and reports
timings to the master log.  Any failure calls ``exception(e)`` → the master exits 1.
``--device cuda`` runs the primitive array checks on MI355X tensors (device engine), in process
and in thread mode.
"""
from __future__ import annotations

import argparse
import sys
import threading
import time

import numpy as np

from . import CommUtils, Operands, Operators, ProcessCommSlave, ThreadCommSlave
from .operators import IObjectOperator, IStringOperator

PRIM = [("double", np.float64, Operands.DOUBLE_OPERAND, Operators.Double),
        ("float", np.float32, Operands.FLOAT_OPERAND, Operators.Float),
        ("long", np.int64, Operands.LONG_OPERAND, Operators.Long),
        ("int", np.int32, Operands.INT_OPERAND, Operators.Int),
        ("short", np.int16, Operands.SHORT_OPERAND, Operators.Short),
        ("byte", np.int8, Operands.BYTE_OPERAND, Operators.Byte)]


class CheckFailed(AssertionError):
    pass


def _ok(cond, msg):
    if not cond:
        raise CheckFailed(msg)


class _Arr:
    """numpy or torch array factory so the same checks run on host or device."""

    def __init__(self, device: str):
        self.device = device
        if device != "cpu":
            import torch
            self.torch = torch

    def full(self, n, v, dt):
        if self.device == "cpu":
            return np.full(n, v, dt)
        return self.torch.full((n,), v, dtype=getattr(self.torch, np.dtype(dt).name), device=self.device)

    def all_eq(self, a, v) -> bool:
        if self.device == "cpu":
            return bool((a == v).all())
        return bool((a == v).all().item())


def process_checks(comm: ProcessCommSlave, arr_size: int, obj_size: int, run_time: int, compress: bool,
                   test_rpc: bool, device: str = "cpu"):
    p, r = comm.getSlaveNum(), comm.getRank()
    device = _device_for(r, device)
    A = _Arr(device)
    froms = CommUtils.createProcessArrayFroms(arr_size, p)
    tos = CommUtils.createProcessArrayTos(arr_size, p)
    root = p - 1 if p > 1 else 0
    for name, dt, mk, ops in PRIM:
        operand = mk(compress)
        for it in range(run_time):
            t0 = time.perf_counter()
            a = A.full(arr_size, -1, dt)
            a[froms[r]:tos[r]] = r
            comm.gatherArray(a, operand, froms, tos, root)
            if r == root:
                for i in range(p):
                    _ok(A.all_eq(a[froms[i]:tos[i]], i), f"{name} gather")
            a = A.full(arr_size, -1, dt)
            if r == root:
                for i in range(p):
                    a[froms[i]:tos[i]] = i
            comm.scatterArray(a, operand, froms, tos, root)
            _ok(A.all_eq(a[froms[r]:tos[r]], r), f"{name} scatter")
            a = A.full(arr_size, -1, dt)
            a[froms[r]:tos[r]] = r
            comm.allgatherArray(a, operand, froms, tos)
            for i in range(p):
                _ok(A.all_eq(a[froms[i]:tos[i]], i), f"{name} allgather")
            counts = [t - f for f, t in zip(froms, tos)]
            a = A.full(arr_size, 1, dt)
            comm.reduceScatterArray(a, operand, ops.SUM, 0, counts)
            _ok(A.all_eq(a[froms[r]:tos[r]], p), f"{name} reduceScatter")
            a = A.full(arr_size, 1 if r == root else -1, dt)
            comm.broadcastArray(a, operand, 0, arr_size, root)
            _ok(A.all_eq(a, 1), f"{name} broadcast")
            a = A.full(arr_size, 1, dt)
            comm.reduceArray(a, operand, ops.SUM, 0, arr_size, root)
            if r == root:
                _ok(A.all_eq(a, p), f"{name} reduce")
            a = A.full(arr_size, 1, dt)
            comm.allreduceArray(a, operand, ops.SUM, 0, arr_size)
            _ok(A.all_eq(a, p), f"{name} allreduce")
            if test_rpc:
                a = A.full(min(arr_size, 1 << 16), 1, dt)
                comm.allreduceArrayRpc(a, operand, ops.SUM)
                _ok(A.all_eq(a, p), f"{name} rpc allreduce")
            # map (shared keys + a unique key per rank; size == objSize + p)
            m = {str(k): dt(1).item() for k in range(obj_size)}
            m[str(-(r + 1))] = dt(1).item()
            res = comm.allreduceMap(m, operand, ops.SUM)
            _ok(len(res) == obj_size + p and all(res[str(k)] == p for k in range(obj_size)), f"{name} allreduceMap")
            comm.info(f"{name} check round {it} takes: {(time.perf_counter() - t0) * 1e3:.1f} ms")
    # string / object operands (host)
    sop = Operands.STRING_OPERAND(compress)
    add = IStringOperator(lambda a, b: str(int(a) + int(b)))
    s = ["1"] * min(arr_size, 10000)
    comm.allreduceArray(s, sop, add, 0, len(s))
    _ok(all(x == str(p) for x in s), "string allreduce")
    oop = Operands.OBJECT_OPERAND(compress=compress)
    o = [[1] for _ in range(min(arr_size, 2000))]
    comm.allreduceArray(o, oop, IObjectOperator(lambda a, b: [a[0] + b[0]]), 0, len(o))
    _ok(all(x == [p] for x in o), "object allreduce")
    _ok(comm.allreduceSetUnion({r}) == set(range(p)), "set union")
    comm.info("process checks passed")


def _device_for(rank: int, device: str) -> str:
    """``cuda`` -> this rank's GPU (``MP4X_DEVICE_INDEX`` / ``LOCAL_RANK`` / rank mod count)."""
    if device == "cpu" or ":" in device:
        return device
    import os
    import torch
    idx = os.environ.get("MP4X_DEVICE_INDEX", os.environ.get("LOCAL_RANK"))
    return f"cuda:{int(idx) if idx is not None else rank % max(1, torch.cuda.device_count())}"


def thread_checks(tc: ThreadCommSlave, arr_size: int, obj_size: int, run_time: int, compress: bool, test_rpc: bool,
                  device: str = "cpu"):
    """Every reference Thread*Check (J/check/check*/Thread{Gather,Scatter,AllGather,ReduceScatter,
    Broadcast,Reduce,AllReduce}Check.java + the map / set / list / scalar / RPC variants) with
    roots (rootRank, rootThreadId) = (p-1, T-1), then every ``*Process`` pass-through from thread 0
    (J/check/checkbyte/ThreadAllReduceCheck.java:156-241).  ``device`` = cuda: the arrays are
    tensors on this rank's GPU (the thread phase is the K1 multi-input kernel)."""
    p, r, T = tc.getSlaveNum(), tc.getRank(), tc.getThreadNum()
    device = _device_for(r, device)
    A = _Arr(device)
    froms = CommUtils.createThreadArrayFroms(arr_size, p, T)
    tos = CommUtils.createThreadArrayTos(arr_size, p, T)
    pf = CommUtils.createProcessArrayFroms(arr_size, p)
    pt = CommUtils.createProcessArrayTos(arr_size, p)
    rr, rt = p - 1, T - 1
    errs = []

    def body(t):
        try:
            tc.setThreadId(t)
            if device != "cpu":
                A.torch.cuda.set_device(A.torch.device(device))
            me = r == rr and t == rt
            for name, dt, mk, ops in PRIM:
                operand = mk(compress)
                for it in range(run_time):
                    t0 = time.perf_counter()
                    a = A.full(arr_size, -1, dt)
                    a[froms[r][t]:tos[r][t]] = r * T + t
                    g = tc.gatherArray(a, operand, froms, tos, rr, rt)
                    if me:
                        for i in range(p):
                            for j in range(T):
                                _ok(A.all_eq(g[froms[i][j]:tos[i][j]], i * T + j), f"thread {name} gather")
                    a = A.full(arr_size, -1, dt)
                    if me:
                        for i in range(p):
                            for j in range(T):
                                a[froms[i][j]:tos[i][j]] = i * T + j
                    tc.scatterArray(a, operand, froms, tos, rr, rt)
                    _ok(A.all_eq(a[froms[r][t]:tos[r][t]], r * T + t), f"thread {name} scatter")
                    a = A.full(arr_size, -1, dt)
                    a[froms[r][t]:tos[r][t]] = r * T + t
                    tc.allgatherArray(a, operand, froms, tos)
                    for i in range(p):
                        for j in range(T):
                            _ok(A.all_eq(a[froms[i][j]:tos[i][j]], i * T + j), f"thread {name} allgather")
                    counts = [[tos[i][j] - froms[i][j] for j in range(T)] for i in range(p)]
                    a = A.full(arr_size, 1, dt)
                    tc.reduceScatterArray(a, operand, ops.SUM, 0, counts)
                    _ok(A.all_eq(a[froms[r][t]:tos[r][t]], p * T), f"thread {name} reduceScatter")
                    a = A.full(arr_size, 1 if me else -1, dt)
                    tc.broadcastArray(a, operand, 0, arr_size, rr, rt)
                    _ok(A.all_eq(a, 1), f"thread {name} broadcast")
                    a = A.full(arr_size, 1, dt)
                    tc.reduceArray(a, operand, ops.SUM, 0, arr_size, rr, rt)
                    if me:
                        _ok(A.all_eq(a, p * T), f"thread {name} reduce")
                    a = A.full(arr_size, 1, dt)
                    tc.allreduceArray(a, operand, ops.SUM, 0, arr_size)
                    _ok(A.all_eq(a, p * T), f"thread {name} allreduce")
                    a = A.full(arr_size, r * T + t, dt)
                    tc.allreduceArray(a, operand, ops.MAX, 0, arr_size)
                    _ok(A.all_eq(a, p * T - 1), f"thread {name} allreduce MAX")
                    if test_rpc:
                        a = A.full(min(arr_size, 4096), 1, dt)
                        tc.allreduceArrayRpc(a, operand, ops.SUM)
                        _ok(A.all_eq(a, p * T), f"thread {name} rpc")
                        _ok(tc.allreduceRpc(dt(1).item(), operand, ops.SUM) == p * T, f"thread {name} rpc scalar")
                    _ok(tc.allreduce(dt(1).item(), operand, ops.SUM) == p * T, f"thread {name} allreduce scalar")
                    v = tc.reduce(dt(1).item(), operand, ops.SUM, rr, rt)
                    _ok(not me or v == p * T, f"thread {name} reduce scalar")
                    _ok(tc.broadcast(dt(7 if me else 0).item(), operand, rr, rt) == 7, f"thread {name} broadcast scalar")
                    # maps: shared keys + one unique key per (rank, thread)
                    m = {str(k): dt(1).item() for k in range(obj_size)}
                    m[f"u{r}_{t}"] = dt(1).item()
                    res = tc.allreduceMap(m, operand, ops.SUM)
                    _ok(len(res) == obj_size + p * T and res.get("0", p * T) == p * T, f"thread {name} allreduceMap")
                    red = tc.reduceMap(m, operand, ops.SUM, rr, rt)
                    _ok((red is not None and len(red) == obj_size + p * T) if me else red is None,
                        f"thread {name} reduceMap")
                    gm = tc.gatherMap({f"g{r}_{t}": dt(1).item()}, operand, rr, rt)
                    _ok(not me or len(gm) == p * T, f"thread {name} gatherMap")
                    ag = tc.allgatherMap({f"a{r}_{t}": dt(1).item()}, operand)
                    _ok(len(ag) == p and set(ag[r]) == {f"a{r}_{j}" for j in range(T)}, f"thread {name} allgatherMap")
                    bm = tc.broadcastMap({"b": dt(3).item()} if me else {}, operand, rr, rt)
                    _ok(bm == {"b": 3}, f"thread {name} broadcastMap")
                    lists = [[{f"s{i}_{j}": dt(1).item()} for j in range(T)] for i in range(p)] if me else None
                    sm = tc.scatterMap(lists, operand, rr, rt)
                    _ok(sm == {f"s{r}_{t}": 1}, f"thread {name} scatterMap")
                    rsl = [[{"c": dt(1).item()} for _ in range(T)] for _ in range(p)]
                    rs = tc.reduceScatterMap(rsl, operand, ops.SUM)
                    _ok(rs == {"c": p * T}, f"thread {name} reduceScatterMap")
                    if t == 0:
                        tc.info(f"thread {name} check round {it} takes: {(time.perf_counter() - t0) * 1e3:.1f} ms")
            # set / list specials (object operands, host)
            _ok(tc.allreduceSetUnion({r * T + t}) == set(range(p * T)), "thread set union")
            _ok(tc.allreduceSetIntersection({-1, r * T + t}) == ({-1} if p * T > 1 else {-1, 0}),
                "thread set intersection")
            _ok(sorted(tc.allreduceListConcat([r * T + t])) == list(range(p * T)), "thread list concat")
            u = tc.reduceSetUnion({r * T + t}, rr, rt)
            _ok((u == set(range(p * T))) if me else u is None, "thread reduce set union")
            # string / object operands
            sop = Operands.STRING_OPERAND(compress)
            add = IStringOperator(lambda a, b: str(int(a) + int(b)))
            s = ["1"] * min(arr_size, 1000)
            tc.allreduceArray(s, sop, add, 0, len(s))
            _ok(all(x == str(p * T) for x in s), "thread string allreduce")
            # *Process pass-throughs: one thread per process
            if t == 0:
                D, ops = Operands.DOUBLE_OPERAND(compress), Operators.Double
                b = A.full(arr_size, 1, np.float64)
                tc.allreduceArrayProcess(b, D, ops.SUM, 0, arr_size)
                _ok(A.all_eq(b, p), "allreduceArrayProcess")
                b = A.full(arr_size, -1, np.float64)
                b[pf[r]:pt[r]] = r
                tc.allgatherArrayProcess(b, D, pf, pt)
                _ok(all(A.all_eq(b[pf[i]:pt[i]], i) for i in range(p)), "allgatherArrayProcess")
                b = A.full(arr_size, -1, np.float64)
                b[pf[r]:pt[r]] = r
                tc.gatherArrayProcess(b, D, pf, pt, rr)
                _ok(r != rr or all(A.all_eq(b[pf[i]:pt[i]], i) for i in range(p)), "gatherArrayProcess")
                b = A.full(arr_size, -1, np.float64)
                if r == rr:
                    for i in range(p):
                        b[pf[i]:pt[i]] = i
                tc.scatterArrayProcess(b, D, pf, pt, rr)
                _ok(A.all_eq(b[pf[r]:pt[r]], r), "scatterArrayProcess")
                b = A.full(arr_size, 2 if r == rr else 0, np.float64)
                tc.broadcastArrayProcess(b, D, 0, arr_size, rr)
                _ok(A.all_eq(b, 2), "broadcastArrayProcess")
                b = A.full(arr_size, 1, np.float64)
                tc.reduceScatterArrayProcess(b, D, ops.SUM, 0, [y - x for x, y in zip(pf, pt)])
                _ok(A.all_eq(b[pf[r]:pt[r]], p), "reduceScatterArrayProcess")
                b = A.full(arr_size, 1, np.float64)
                tc.reduceArrayProcess(b, D, ops.SUM, 0, arr_size, rr)
                _ok(r != rr or A.all_eq(b, p), "reduceArrayProcess")
                b = A.full(min(arr_size, 64), 1, np.float64)
                tc.allreduceArrayRpcProcess(b, D, ops.SUM)
                _ok(A.all_eq(b, p), "allreduceArrayRpcProcess")
                _ok(tc.allreduceProcess(1.0, D, ops.SUM) == p, "allreduceProcess")
                _ok(tc.broadcastProcess(5.0 if r == rr else 0.0, D, rr) == 5.0, "broadcastProcess")
                _ok(tc.allreduceMapProcess({"k": 1.0}, D, ops.SUM) == {"k": float(p)}, "allreduceMapProcess")
                _ok(tc.allreduceSetUnionProcess({r}) == set(range(p)), "allreduceSetUnionProcess")
            tc.threadBarrier()
            if t == 0:
                tc.info("thread checks passed")
        except BaseException as e:  # noqa
            errs.append(e)
            tc.abort()

    ths = [threading.Thread(target=body, args=(t,)) for t in range(T)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise errs[0]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    for a in ("login", "master_host"):
        ap.add_argument(a)
    ap.add_argument("port", type=int)
    ap.add_argument("arr_size", type=int)
    ap.add_argument("obj_size", type=int)
    ap.add_argument("run_time", type=int)
    ap.add_argument("thread_num", type=int)
    ap.add_argument("mode", choices=["process", "thread"])
    ap.add_argument("compress", type=lambda s: s.lower() == "true")
    ap.add_argument("test_rpc", type=lambda s: s.lower() == "true")
    ap.add_argument("--device", default="cpu")
    a = ap.parse_args(argv)
    # log/slave{,_warn,_error}.log when MP4X_LOG_DIR or MP4X_LOG_CONFIG is set (reference:
    # config/log4j_slave.properties); stdout only otherwise
    import os
    from .utils.logconf import configure_logging
    configure_logging("slave", log_dir=os.environ.get("MP4X_LOG_DIR", "-"))
    comm = None
    code = 0
    try:
        if a.mode == "process":
            comm = ProcessCommSlave(a.login, a.master_host, a.port)
            process_checks(comm, a.arr_size, a.obj_size, a.run_time, a.compress, a.test_rpc, a.device)
        else:
            comm = ThreadCommSlave(a.login, a.thread_num, a.master_host, a.port)
            thread_checks(comm, a.arr_size, a.obj_size, a.run_time, a.compress, a.test_rpc, a.device)
    except BaseException as e:  # noqa
        code = 1
        print(f"check failed: {e!r}", file=sys.stderr)
        if comm is not None:
            try:
                comm.exception(e)
            except Exception:
                pass
    finally:
        if comm is not None:
            try:
                comm.close(code)
            except Exception:
                pass
    return code


if __name__ == "__main__":
    sys.exit(main())
