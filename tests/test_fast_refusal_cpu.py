"""Every refusal of the native latency fast paths happens BEFORE the epoch moves (VERDICT r5
Next #3 / weak #4): a refused call leaves the instance's epoch box, the stream-order
guard and the instance's error word untouched, and only the "nothing launched" codes send a call
to the full path — any other code raises at once.  CPU: the real libmp4x_hip.so, called with a
fake instance state (the refusals are host-side checks; the capture query, which needs a GPU,
comes after them)."""
import ctypes

import pytest

torch = pytest.importorskip("torch")

from mp4x.operators import DType, OpCode  # noqa: E402
from mp4x.ops import native  # noqa: E402


def _lib():
    try:
        return native.hip()
    except Exception as e:   # noqa: BLE001
        pytest.skip(f"libmp4x_hip.so not loadable: {e}")


def _state(p=2, rank=0, herr=None):
    from mp4x.parallel.ipc import FastAr
    from mp4x.parallel.order import CommOrder
    s = FastAr()
    box = (ctypes.c_uint32 * 1)(7)
    own = (ctypes.c_uint32 * 1)(0)
    ptrs = (ctypes.c_void_p * 8)(*([0x10000] * 8))
    if herr is not None:
        s.herr[0] = ctypes.addressof(herr)
    s.epoch = ctypes.addressof(box)
    s.data_ptrs = s.signal_ptrs = ctypes.addressof(ptrs)
    s.rank, s.p = rank, p
    order = CommOrder()
    s.order = order.addr
    s.own_err = ctypes.addressof(own)
    return s, box, own, order, ptrs


def _fast_ar(lib, s, algo, dtype, op, buf, nbytes, scale=1.0):
    f = lib.mp4x_ipc_fast_allreduce
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                  ctypes.c_int, ctypes.c_float, ctypes.c_void_p]
    return f(ctypes.addressof(s), algo, int(dtype), int(op), buf, nbytes, 0, scale, None)


@pytest.mark.parametrize("case,want", [
    (dict(buf=0x1008), 1001),                                   # unaligned buffer
    (dict(nbytes=1000), 1001),                                  # not a 16-byte multiple
    (dict(nbytes=0), 1001),
    (dict(algo=2), 1001),                                       # no such algorithm
    (dict(dtype=DType.I32, scale=0.5), 1001),                   # fused scale needs a float dtype
    (dict(op=OpCode.BAND), 1002),                               # BITS_AND of f32: not an operator of the table
    (dict(dtype=99), 1002),
    (dict(p=9), 1001),                                          # rank count out of range
    (dict(p=2, rank=2), 1001),
])
def test_refused_allreduce_leaves_the_epoch_alone(case, want):
    lib = _lib()
    s, box, own, order, _keep = _state(p=case.get("p", 2), rank=case.get("rank", 0))
    rc = _fast_ar(lib, s, case.get("algo", 0), case.get("dtype", DType.F32), case.get("op", OpCode.SUM),
                  case.get("buf", 0x1000), case.get("nbytes", 4096), case.get("scale", 1.0))
    assert rc == want
    assert box[0] == 7 and own[0] == 0                 # epoch unchanged, instance not marked
    assert not order.s.have_last and order.switches == 0    # the stream order was not touched


def test_failed_earlier_is_refused_first():
    lib = _lib()
    w = ctypes.c_uint32(1)
    s, box, own, order, _keep = _state(herr=w)
    assert _fast_ar(lib, s, 0, DType.F32, OpCode.SUM, 0x1000, 4096) == 1003
    assert box[0] == 7 and not order.s.have_last


def test_valid_call_without_a_gpu_stops_at_the_capture_query():
    """A valid call passes every host check; without a GPU the capture query fails and the call is
    refused as 1004 — still before the stream join and the epoch bump."""
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    lib = _lib()
    s, box, own, order, _keep = _state()
    assert _fast_ar(lib, s, 1, DType.BF16, OpCode.MAX, 0x1000, 1 << 16) == 1004
    assert box[0] == 7 and own[0] == 0 and not order.s.have_last


def test_refused_plan_and_rs_leave_the_epoch_alone():
    lib = _lib()
    s, box, own, order, _keep = _state(p=2)
    I64 = ctypes.c_int64
    plan = lib.mp4x_ipc_fast_plan
    plan.restype = ctypes.c_int
    plan.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, I64, I64,
                     ctypes.c_void_p, I64, I64, ctypes.c_int, ctypes.c_void_p]
    pull = (I64 * 4)(0, 0, 16, 5)                      # peer 5 of 2 ranks
    assert plan(ctypes.addressof(s), None, 0, pull, 1, -1, 0, 0x1000, 16, 64, 0, None) == 1001
    pull = (I64 * 4)(60, 0, 16, 1)                     # past the peer's buffer (64 vectors)
    assert plan(ctypes.addressof(s), None, 0, pull, 1, -1, 0, 0x1000, 16, 64, 0, None) == 1001
    pull = (I64 * 4)(0, 0, 16, 1)
    assert plan(ctypes.addressof(s), None, 0, pull, 1, -1, 8, 0x1000, 16, 64, 0, None) == 1001   # unaligned out
    rs = lib.mp4x_ipc_fast_rs
    rs.restype = ctypes.c_int
    rs.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, I64, I64,
                   ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lo, hi = (I64 * 2)(0, 4), (I64 * 2)(4, 8)
    assert rs(ctypes.addressof(s), int(DType.F32), int(OpCode.BXOR), lo, hi, 0, 0, 0x1000, 0, None) == 1002
    bad_hi = (I64 * 2)(4, 2)
    assert rs(ctypes.addressof(s), int(DType.F32), int(OpCode.SUM), lo, bad_hi, 0, 0, 0x1000, 0, None) == 1001
    assert box[0] == 7 and own[0] == 0 and not order.s.have_last


def test_fast_ok_falls_back_only_when_nothing_was_launched(monkeypatch):
    from mp4x.parallel.process_comm import _fast_ok
    monkeypatch.setattr(native, "_hip", None)
    assert _fast_ok(0, "x") is True
    for rc in (1001, 1002, 1003, 1004):
        assert _fast_ok(rc, "x") is False
    with pytest.raises(native.NativeError):
        _fast_ok(1, "mp4x_ipc_fast_allreduce")          # a HIP launch error after the epoch moved
    with pytest.raises(native.NativeError):
        _fast_ok(1005, "mp4x_ipc_fast_allreduce")


def test_copy_plan_takes_two_pulls_per_peer_at_eight_ranks():
    """The sparse exchanges pull a row block and a key block from every peer: 2p pulls at p = 8
    must pass the plan check on every rank (a refusal on the ranks with more non-empty blocks
    than the others would leave the rest waiting in the kernel's barrier)."""
    import mp4x.parallel.ipc  # noqa: F401  (registers the ipc signatures)
    lib = _lib()
    c64 = ctypes.c_int64

    def check(npull, p=8):
        pa = (c64 * (4 * npull))(*[x for j in range(npull) for x in (j, j, 1, j % p)])
        sa = (c64 * 4)()
        return lib.mp4x_ipc_copy_plan_check(0, p, sa, 0, pa, npull, None, 0x1000, 1 << 20)
    assert check(16) == 0
    assert check(17) == 1001                              # MP4X_E_BADARG


def test_refused_plan_leaves_the_epoch_in_step(monkeypatch):
    """IpcForms._plan runs the plan check before the epoch moves: a refused plan raises with the
    epoch (and the stream order) untouched."""
    from mp4x.exceptions import NativeError
    from mp4x.parallel import ipc_forms
    import mp4x.parallel.ipc  # noqa: F401
    lib = _lib()

    class _Inst(ipc_forms.IpcForms):
        def __init__(self):
            self.lib, self.rank, self.p, self.nbytes, self.epoch = lib, 0, 8, 1 << 20, 5
            self._plan_sink = None

        def raise_if_failed(self):
            pass

        def _launch_stream(self):
            raise AssertionError("stream joined before the check")

    inst = _Inst()
    pulls = [(j, j, 1, j % 8) for j in range(17)]
    with pytest.raises(NativeError):
        inst._plan([], pulls, None, 0x1000, 1)
    assert inst.epoch == 5
