"""IPC setup failures are decided collectively (CPU, fake native library).

A rank whose IPC buffer allocation fails must still join the handle allgather, so every rank
raises the same error instead of its peers waiting forever for it
(`mp4x/parallel/ipc.py` `IpcAllreduce.__init__`).
"""
import threading
from ctypes import c_void_p

import pytest

from mp4x.exceptions import Mp4jException
from mp4x.parallel import ipc as ipc_mod


class _Server:
    """In-process stand-in for the master's allgather_obj / barrier RPCs."""

    def __init__(self, p):
        self.p = p
        self.bar = threading.Barrier(p, timeout=10)
        self.slots = [None] * p

    def call(self, name, rank, *args):
        if name == "barrier":
            self.bar.wait()
            return None
        assert name == "allgather_obj"
        self.slots[rank] = args[0]
        self.bar.wait()
        out = list(self.slots)
        self.bar.wait()
        return out


class _Comm:
    def __init__(self, server, rank):
        self.server, self.rank, self.slaveNum = server, rank, server.p


class _FakeLib:
    def __init__(self, fail_rank_of):
        self.fail_rank_of = fail_rank_of
        self.freed = []

    def mp4x_ipc_handle_size(self):
        return 8

    def mp4x_ipc_signal_bytes(self):
        return 4096

    def mp4x_ipc_alloc(self, nbytes, out):
        if self.fail_rank_of():
            return 2                      # hipErrorOutOfMemory
        out._obj.value = 0x1000
        return 0

    def mp4x_ipc_alloc_data(self, nbytes, coarse, out):
        return self.mp4x_ipc_alloc(nbytes, out)

    def mp4x_ipc_get_handle(self, ptr, buf):
        return 0

    def mp4x_device_pci_id(self, buf, n):
        return 0

    def mp4x_ipc_open_handle(self, h, out):
        out._obj.value = 0x2000
        return 0

    def mp4x_ipc_close_handle(self, ptr):
        return 0

    def mp4x_ipc_free(self, ptr):
        self.freed.append(ptr)
        return 0

    def mp4x_ipc_set_spin(self, s):
        return 0

    def mp4x_host_word_alloc(self, hptr, dptr):
        return 0

    def mp4x_host_word_free(self, hptr):
        return 0

    def mp4x_ipc_set_host_error(self, sig, dev):
        return 0


def test_alloc_failure_on_one_rank_raises_on_every_rank(monkeypatch):
    p = 3
    tls = threading.local()
    lib = _FakeLib(lambda: tls.rank == 1)
    monkeypatch.setattr(ipc_mod.native, "hip", lambda: lib)
    monkeypatch.setattr(ipc_mod.torch.cuda, "current_device", lambda: 0)
    server = _Server(p)
    errors = [None] * p

    def run(r):
        tls.rank = r
        try:
            ipc_mod.IpcAllreduce(_Comm(server, r), nbytes=1 << 16)
        except Mp4jException as e:
            errors[r] = str(e)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(p)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(20)
    assert not any(t.is_alive() for t in threads), "a rank is stuck waiting for its peers"
    assert all(e is not None and "failed on ranks [(1," in e for e in errors), errors


def test_native_load_failure_before_first_collective_raises_on_every_rank(monkeypatch):
    """native.hip() / current_device() failing on ONE rank happen before any collective: the
    error must travel in the first allgather so no peer is left waiting (ipc.py:74)."""
    p = 3
    tls = threading.local()
    lib = _FakeLib(lambda: False)

    def hip():
        if tls.rank == 2:
            raise OSError("libmp4x_hip.so: cannot open shared object file")
        return lib
    monkeypatch.setattr(ipc_mod.native, "hip", hip)
    monkeypatch.setattr(ipc_mod.torch.cuda, "current_device", lambda: 0)
    server = _Server(p)
    errors = [None] * p

    def run(r):
        tls.rank = r
        try:
            ipc_mod.IpcAllreduce(_Comm(server, r), nbytes=1 << 16)
        except Mp4jException as e:
            errors[r] = str(e)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(p)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(20)
    assert not any(t.is_alive() for t in threads), "a rank is stuck waiting for its peers"
    assert all(e is not None and "setup failed on ranks [(2," in e for e in errors), errors
