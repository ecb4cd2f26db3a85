"""CommCheckTool — the reference's integration check harness as a CLI.

Reference: J/check/CommCheckTool.java:40-321 (+ 16 checks per element type in J/check/check*/).

    python -m mp4x.check <login> <masterHost> <port> <arrSize> <objSize> <runTime> \\
                         <threadNum> <process|thread> <compress> <testRpc> [--device cpu|cuda]

Every slave runs gather / scatter / allgather / reduce-scatter / broadcast / reduce /
allreduce (+ RPC allreduce) for double, float, long, int, short, byte, string and object
operands on arrays of ``arrSize`` and maps of ``objSize`` keys, ``runTime`` times each,
checks the exact expected values (deterministic inputs, as the reference does) and reports
timings to the master log.  Any failure calls ``exception(e)`` → the master exits 1.
``--device cuda`` runs the primitive array checks on MI355X tensors (device engine).
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


def thread_checks(tc: ThreadCommSlave, arr_size: int, obj_size: int, run_time: int, compress: bool, test_rpc: bool):
    p, r, T = tc.getSlaveNum(), tc.getRank(), tc.getThreadNum()
    froms = CommUtils.createThreadArrayFroms(arr_size, p, T)
    tos = CommUtils.createThreadArrayTos(arr_size, p, T)
    errs = []

    def body(t):
        try:
            tc.setThreadId(t)
            for name, dt, mk, ops in PRIM:
                operand = mk(compress)
                for it in range(run_time):
                    a = np.ones(arr_size, dt)
                    tc.allreduceArray(a, operand, ops.SUM, 0, arr_size)
                    _ok((a == p * T).all(), f"thread {name} allreduce")
                    a = np.full(arr_size, -1, dt)
                    a[froms[r][t]:tos[r][t]] = r * T + t
                    tc.allgatherArray(a, operand, froms, tos)
                    for i in range(p):
                        for j in range(T):
                            _ok((a[froms[i][j]:tos[i][j]] == i * T + j).all(), f"thread {name} allgather")
                    counts = [[tos[i][j] - froms[i][j] for j in range(T)] for i in range(p)]
                    a = np.ones(arr_size, dt)
                    tc.reduceScatterArray(a, operand, ops.SUM, 0, counts)
                    _ok((a[froms[r][t]:tos[r][t]] == p * T).all(), f"thread {name} reduceScatter")
                    if test_rpc:
                        a = np.ones(min(arr_size, 4096), dt)
                        tc.allreduceArrayRpc(a, operand, ops.SUM)
                        _ok((a == p * T).all(), f"thread {name} rpc")
                    m = {str(k): dt(1).item() for k in range(obj_size)}
                    res = tc.allreduceMap(m, operand, ops.SUM)
                    _ok(res["0"] == p * T, f"thread {name} allreduceMap")
            tc.info("thread checks passed")
        except BaseException as e:  # noqa
            errs.append(e)
            tc._barrier.abort()

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
            thread_checks(comm, a.arr_size, a.obj_size, a.run_time, a.compress, a.test_rpc)
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
