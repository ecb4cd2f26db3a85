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

    def mp4x_ipc_set_spin(self, sig, seconds, stream):
        self.spin = seconds
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


class _CountingLib(_FakeLib):
    """Fake native library that hands out distinct addresses and counts opens / closes / frees."""

    def __init__(self):
        super().__init__(lambda: False)
        self.next = 0x10000
        self.opens = 0
        self.closes = 0
        self.allocs = 0
        self.lock = threading.Lock()

    def _addr(self):
        with self.lock:
            self.next += 0x100000
            return self.next

    def mp4x_ipc_alloc(self, nbytes, out):
        with self.lock:
            self.allocs += 1
        out._obj.value = self._addr()
        return 0

    def mp4x_ipc_get_handle(self, ptr, buf):
        v = ptr.value if hasattr(ptr, "value") else int(ptr)
        buf.raw = v.to_bytes(8, "little")
        return 0

    def mp4x_ipc_open_handle(self, h, out):
        with self.lock:
            self.opens += 1
        out._obj.value = self._addr()
        return 0

    def mp4x_ipc_close_handle(self, ptr):
        with self.lock:
            self.closes += 1
        return 0

    def mp4x_mem_range(self, ptr, base, size):
        base._obj.value = ptr.value
        size._obj.value = 1 << 20
        return 0


class _FakeTensor:
    is_cuda = True

    def __init__(self, ptr, nbytes):
        self.ptr, self.nbytes = ptr, nbytes

    def is_contiguous(self):
        return True

    def data_ptr(self):
        return self.ptr

    def numel(self):
        return self.nbytes // 4

    def element_size(self):
        return 4


@pytest.mark.parametrize("close_peers", [True, False])
def test_registration_lifecycle(monkeypatch, close_peers):
    """CLOSE_PEERS (default): deregister() closes this rank's mappings of the peers' allocations
    once no registration uses them and frees the push scratch, so nothing accumulates per
    registration.  Without it (the round-3 policy): scratch pooled per size, mappings cached until
    close().  Either way a registration holds its tensor and close() releases everything."""
    p = 2
    lib = _CountingLib()
    monkeypatch.setattr(ipc_mod, "CLOSE_PEERS", close_peers)
    monkeypatch.setattr(ipc_mod.native, "hip", lambda: lib)
    monkeypatch.setattr(ipc_mod.torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(ipc_mod.torch.cuda, "synchronize", lambda *a, **k: None)
    server = _Server(p)
    res = [None] * p

    def run(r):
        inst = ipc_mod.IpcAllreduce(_Comm(server, r), nbytes=1 << 16)
        base_allocs = lib.allocs
        server.call("barrier", r)
        a = _FakeTensor(0x7000000 + r * 0x1000000, 1 << 16)
        b = _FakeTensor(0x7100000 + r * 0x1000000, 1 << 16)
        ok1 = inst.register(a)
        keeps = inst._find(a)[0].keep is a
        opened = len(inst._peer_bases)
        inst.deregister(a)
        server.call("barrier", r)
        after_dereg = (len(inst._peer_bases), sum(len(v) for v in inst._scratch_pool.values()))
        ok2 = inst.register(b)
        server.call("barrier", r)
        inst.deregister(b)
        ok3 = inst.register(a)
        server.call("barrier", r)
        inst.deregister(a)
        server.call("barrier", r)
        res[r] = (ok1, ok2, ok3, keeps, opened, after_dereg, lib.allocs - base_allocs, inst)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(p)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(20)
    assert not any(t.is_alive() for t in threads)
    for ok1, ok2, ok3, keeps, opened, after_dereg, allocs, inst in res:
        assert ok1 and ok2 and ok3 and keeps
        assert opened == 2                           # the peer's tensor segment + its push scratch
        if close_peers:
            assert after_dereg == (0, 0)             # mappings closed, scratch freed
            assert not inst._peer_refs and not inst._peer_bases
            assert allocs >= 3                       # one scratch per registration (freed at each)
        else:
            assert after_dereg == (2, 1)             # cached mappings, pooled scratch
            assert allocs <= p                       # the pooled scratch came back
        assert not inst._regs
    for *_, inst in res:
        inst.close(sync=False)
    assert lib.closes >= lib.opens                   # every mapping closed by close() at the latest


def test_hier_submesh_failure_on_one_node_is_agreed_job_wide(monkeypatch):
    """the per-node IPC meshes of the node-aware allreduce are built over
    GLOBAL control-plane calls.  When one node's setup fails, every node must raise at the same
    agreement point, so the global calls that follow stay paired (a node raising alone would pair
    its next global call with the other nodes' setup calls)."""
    from mp4x.parallel.hier import _GroupComm
    p = 4
    nodes = [[0, 1], [2, 3]]
    tls = threading.local()
    lib = _FakeLib(lambda: tls.rank == 2)          # rank 2's buffer allocation fails (node 1)
    monkeypatch.setattr(ipc_mod.native, "hip", lambda: lib)
    monkeypatch.setattr(ipc_mod.torch.cuda, "current_device", lambda: 0)
    server = _Server(p)
    errors, after = [None] * p, [None] * p

    def run(r):
        tls.rank = r
        try:
            ipc_mod.IpcAllreduce(_GroupComm(_Comm(server, r), nodes[r // 2], 1), nbytes=1 << 16)
        except Mp4jException as e:
            errors[r] = str(e)
        after[r] = server.call("allgather_obj", r, ("after", r))     # the next global call

    threads = [threading.Thread(target=run, args=(r,)) for r in range(p)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(20)
    assert not any(t.is_alive() for t in threads), "a rank is stuck waiting for its peers"
    assert all(e is not None for e in errors), errors
    assert "another node" in errors[0] and "(0," in errors[2], errors     # node-local rank 0 of node 1
    assert all(a == [("after", j) for j in range(p)] for a in after), after
