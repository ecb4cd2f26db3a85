"""The stream-order guard's host side (mp4x/parallel/order.py), with a fake native entry: the steady
state (same stream, not capturing) never leaves Python; a stream switch or a capture goes to the
native join with the capture state; a switch inside one capture raises a named error; the
communicator shares ONE guard between its IPC instances and its RCCL calls."""
import pytest

from mp4x.exceptions import Mp4jException
from mp4x.ops import native
from mp4x.parallel import order as order_mod


class _Native:
    def __init__(self, rc=0):
        self.calls = []
        self.rc = rc

    def __call__(self, addr, stream, cap):
        self.calls.append((stream, cap))
        if self.rc:
            return self.rc
        o = order_mod.StreamOrder.from_address(addr)
        if not cap:
            if o.have_last and (o.last or 0) != stream:
                o.switches += 1
            o.last, o.have_last = stream, 1
        return 0


def _order(monkeypatch, cap=False, rc=0):
    o = order_mod.CommOrder()
    fake = _Native(rc)
    o._enter = fake
    monkeypatch.setattr(native, "capturing_now", lambda: cap)
    return o, fake


def test_steady_state_stays_in_python(monkeypatch):
    o, fake = _order(monkeypatch)
    o.enter(0x10)                      # first launch: native (nothing recorded yet)
    for _ in range(100):
        o.enter(0x10)                  # same stream: no native call
    assert fake.calls == [(0x10, 0)]
    o.enter(0x20)                      # a switch: native join
    o.enter(0x20)
    o.enter(0)                         # the null stream is a stream too
    assert fake.calls == [(0x10, 0), (0x20, 0), (0, 0)] and o.switches == 2


def test_capture_always_reaches_the_native_check(monkeypatch):
    o, fake = _order(monkeypatch)
    o.enter(0x10)
    monkeypatch.setattr(native, "capturing_now", lambda: True)
    o.enter(0x10)                      # same stream, but capturing: the capture id is tracked natively
    assert fake.calls[-1] == (0x10, 1)


def test_switch_inside_a_capture_raises(monkeypatch):
    o, _ = _order(monkeypatch, cap=True, rc=order_mod.STREAM_SWITCH)
    with pytest.raises(Mp4jException, match="ONE stream"):
        o.enter(0x30)


def test_disabled_by_env_only_for_tests(monkeypatch):
    monkeypatch.setenv("MP4X_TEST_NO_STREAM_ORDER", "1")
    assert order_mod.CommOrder().s.disabled == 1
    monkeypatch.delenv("MP4X_TEST_NO_STREAM_ORDER")
    assert order_mod.CommOrder().s.disabled == 0


def test_torchcoll_enters_the_order_for_device_tensors(monkeypatch):
    from mp4x.parallel import coll
    seen = []

    class _O:
        def enter(self, st):
            seen.append(st)
    c = coll.TorchColl(None, "nccl")
    c.order = _O()
    monkeypatch.setattr(native, "stream_ptr", lambda *a: 0x77)
    monkeypatch.setattr(coll.dist, "all_reduce", lambda *a, **k: None)

    class _T:
        is_cuda = True
    c.all_reduce(_T(), 0)
    assert seen == [0x77]
    c.all_reduce(type("C", (), {"is_cuda": False})(), 0)      # host tensors: no device order
    assert seen == [0x77]
