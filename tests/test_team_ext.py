"""The native thread-team binding (csrc/pyext/team_ext.cpp) behind ThreadCommSlave's host-array
collectives, and its GIL hand-off chain (csrc/host/host_ops.cpp ``team_leave``).

Reference: the thread level of ThreadCommSlave.allreduceArray (ThreadCommSlave.java:259-303,
448-520)."""
import os
import threading

import numpy as np
import pytest

from mp4x import Mp4jException, Operands, Operators
from mp4x.ops import native
from mp4x.parallel.thread_comm import ThreadCommSlave

pytestmark = pytest.mark.skipif(not os.path.exists(native.HOST_LIB), reason="host library not built")


class _Solo:
    """A one-process stand-in for the ProcessCommSlave under a ThreadCommSlave."""

    def getRank(self):
        return 0

    def getSlaveNum(self):
        return 1

    def close(self, code=0):
        pass

    def allreduceArray(self, a, *args):
        return a

    def reduceArray(self, a, *args):
        return a


def _team(T):
    return ThreadCommSlave("t", T, process_comm=_Solo())


def _run(tc, fn):
    T = tc.getThreadNum()
    res, errs = [None] * T, [None] * T

    def body(t):
        tc.setThreadId(t)
        try:
            res[t] = fn(t)
        except BaseException as e:   # noqa: B902
            errs[t] = e
            tc.abort()

    ths = [threading.Thread(target=body, args=(t,)) for t in range(T)]
    [x.start() for x in ths]
    [x.join(60) for x in ths]
    assert not any(x.is_alive() for x in ths), "thread team hung"
    return res, errs


def test_binding_is_built_and_used():
    ext = native.team_ext()
    assert ext is not None, "csrc/pyext/team_ext.cpp not built: run tools/build_native.py"
    tc = _team(2)
    assert tc._barrier.ext is ext


@pytest.mark.parametrize("T", [2, 3, 5])
@pytest.mark.parametrize("dt,opnd,ops", [(np.float32, Operands.FLOAT_OPERAND(), Operators.Float),
                                         (np.float64, Operands.DOUBLE_OPERAND(), Operators.Double),
                                         (np.int64, Operands.LONG_OPERAND(), Operators.Long),
                                         (np.int32, Operands.INT_OPERAND(), Operators.Int),
                                         (np.int16, Operands.SHORT_OPERAND(), Operators.Short),
                                         (np.int8, Operands.BYTE_OPERAND(), Operators.Byte)])
def test_allreduce_many_iterations(T, dt, opnd, ops):
    """Back-to-back calls (the hand-off chain's steady state), sub-ranges, SUM and MAX."""
    n = 1000

    def body(t):
        for it in range(200):
            a = np.full(n, (t + it) % 7, dt)
            f, to = it % 5, n - (it % 3)
            tc.allreduceArray(a, opnd, ops.SUM, f, to)
            want = sum((j + it) % 7 for j in range(T))
            assert (a[f:to] == want).all() and (a[:f] == (t + it) % 7).all()
            b = np.full(n, t, dt)
            tc.allreduceArray(b, opnd, ops.MAX, 0, n)
            assert (b == T - 1).all()
        return True

    tc = _team(T)
    res, errs = _run(tc, body)
    assert errs == [None] * T and res == [True] * T


def test_out_of_range_fails_every_thread():
    """[from, to) past the array: the binding refuses it before touching memory; the team is
    aborted so no peer waits forever."""
    def body(t):
        a = np.ones(10 if t == 0 else 100, np.float32)
        tc.allreduceArray(a, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, 50)

    tc = _team(2)
    _, errs = _run(tc, body)
    assert isinstance(errs[0], Mp4jException) and "bounds" in str(errs[0])
    assert isinstance(errs[1], Mp4jException)


def test_not_eligible_takes_generic_path():
    """A strided view or a dtype the operator does not match goes the generic path, same result."""
    def body(t):
        base = np.ones(40, np.float64)
        v = base[::2]
        tc.allreduceArray(v, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, 20)
        assert (v == 2).all() and (base[1::2] == 1).all()
        return True

    tc = _team(2)
    res, errs = _run(tc, body)
    assert errs == [None, None] and res == [True, True]


def test_handoff_off_still_correct(monkeypatch):
    """MP4X_TEAM_HANDOFF_US=0 (no chain): same results."""
    monkeypatch.setenv("MP4X_TEAM_HANDOFF_US", "0")

    def body(t):
        for it in range(100):
            a = np.full(64, t + it, np.float32)
            tc.allreduceArray(a, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, 64)
            assert (a == 2 * it + 1).all()
        tc.threadBarrier()
        return True

    tc = _team(2)
    res, errs = _run(tc, body)
    assert errs == [None, None] and res == [True, True]


def test_reduce_to_nonzero_root_thread():
    """The team reduce phase with root thread != 0 (reduceArray's thread level)."""
    def body(t):
        a = np.full(33, t + 1, np.int32)
        tc.reduceArray(a, Operands.INT_OPERAND(), Operators.Int.SUM, 0, 33, 0, 2)
        return int(a[0])

    tc = _team(3)
    res, errs = _run(tc, body)
    assert errs == [None] * 3 and res[2] == 6
