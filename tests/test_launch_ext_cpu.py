"""The ctypes-free launcher (csrc/pyext/launch_ext.cpp) passes every argument of
mp4x_ipc_allreduce_ex2 through unchanged (the 15-argument form with slots 0 / 0, or the
17-argument form with the one-shot's double-buffered slots): bound here to a ctypes callback with
the same C signature (CPU, no HIP) that records what it receives."""
import ctypes

import pytest

from mp4x.ops import native

PROTO = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p,
                         ctypes.c_int64, ctypes.c_int64)


def test_allreduce_ex_marshals_every_argument():
    try:
        mod = native._load_ext("_mp4x_launch")
    except native.NativeUnavailable:
        pytest.skip("_mp4x_launch not built")
    seen = []

    def fake(*args):
        seen.append(args)
        return 7

    cb = PROTO(fake)
    mod.bind(ctypes.cast(cb, ctypes.c_void_p).value)
    try:
        _check(mod, seen)
    finally:
        mod.bind(0)                 # the callback dies with this test: unbind (calls then raise)
    with pytest.raises(RuntimeError):
        mod.allreduce_ex(*([0] * 13 + [1.0, 0]))
    native._launch_ext = None       # the next native.launch_ext() binds the real library again


def _check(mod, seen):
    rc = mod.allreduce_ex(1, 2, 3, 0x1000, 0x2000, 5, 8, (5 << 32) + 16, None, 0x3000, 0xFFFFFFF0, 48, None, 0.125,
                          0x4000)
    assert rc == 7
    (a,) = seen
    assert a[:3] == (1, 2, 3) and a[3] == 0x1000 and a[4] == 0x2000 and a[5:8] == (5, 8, (5 << 32) + 16)
    assert a[8] is None and a[9] == 0x3000 and a[10] == 0xFFFFFFF0 and a[11] == 48 and a[12] is None
    assert a[13] == pytest.approx(0.125) and a[14] == 0x4000 and a[15:] == (0, 0)
    mod.allreduce_ex(0, 2, 0, 0x1000, 0x2000, 1, 2, 4096, 0x5000, 0x5000, 3, 0, None, 1.0, 0x4000, 1 << 22, 1 << 15)
    assert seen[1][15:] == (1 << 22, 1 << 15)
    with pytest.raises(TypeError):
        mod.allreduce_ex(1, 2, 3)


PLAN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                        ctypes.c_void_p)
RS = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p)


def test_fast_plan_and_fast_rs_marshal_the_memo_entry():
    """fast_plan / fast_rs read the memoised entry positionally (a named tuple is a tuple) and the
    call's stream and tensor address; a wrong shape is a TypeError, an unbound launcher raises."""
    try:
        mod = native._load_ext("_mp4x_launch")
    except native.NativeUnavailable:
        pytest.skip("_mp4x_launch not built")
    if not hasattr(mod, "fast_plan"):
        pytest.skip("old _mp4x_launch build")
    from mp4x.parallel.device_engine import _PlanEntry, _RsEntry
    seen = []
    cbp = PLAN(lambda *a: seen.append(("plan",) + a) or 0)
    cbr = RS(lambda *a: seen.append(("rs",) + a) or 5)
    mod.bind_fast_plan(ctypes.cast(cbp, ctypes.c_void_p).value)
    mod.bind_fast_rs(ctypes.cast(cbr, ctypes.c_void_p).value)
    try:
        pe = _PlanEntry(0x10, 0x20, 1, 0x30, 2, 0, -1, 4096, 1 << 22, 64, "broadcast.ipc", "broadcastArray",
                        None, None, None)
        assert mod.fast_plan(pe, 0x40, 0x5000) == 0
        re_ = _RsEntry(0x11, 2, 3, 0x21, 0x31, 16, 32, 8, "reduce_scatter.ipc", "reduceScatterArray", None, None,
                       None)
        assert mod.fast_rs(re_, 0x41, 0x6000) == 5
        p, r = seen
        assert p == ("plan", 0x10, 0x20, 1, 0x30, 2, 0, -1, 0x5000, 4096, 1 << 22, 64, 0x40)
        assert r == ("rs", 0x11, 2, 3, 0x21, 0x31, 16, 32, 0x6000, 8, 0x41)
        with pytest.raises(TypeError):
            mod.fast_plan(pe, 0x40)
        with pytest.raises(TypeError):
            mod.fast_rs((1, 2), 0x40, 0x6000)
    finally:
        mod.bind_fast_plan(0)
        mod.bind_fast_rs(0)
    with pytest.raises(RuntimeError):
        mod.fast_plan(pe, 0x40, 0x5000)
    native._launch_ext = None
