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
    """CLOSE_PEERS (default): deregister() closes this rank's mappings of the peers' tensors once
    no registration uses them; push scratches are pooled per size class (never freed before
    close(), the peers' mappings of them kept: releasing them was round 4's corruption trigger),
    so nothing accumulates per registration.  Without it (the round-3 policy): scratch pooled per size, mappings cached until
    close().  Either way a registration holds its tensor and close() releases everything."""
    p = 2
    lib = _CountingLib()
    monkeypatch.setattr(ipc_mod, "CLOSE_PEERS", close_peers)
    monkeypatch.setenv("MP4X_IPC_FLUSH_ON_CLOSE", "0")      # (its map / unmap would count as allocs)
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
            # the tensor mapping closed; the push scratches pooled (never freed before close), the
            # peer's pooled scratch still mapped for the next registration it serves
            assert after_dereg == (1, 1)
            assert not inst._peer_refs and len(inst._peer_bases) == 1
            assert allocs <= p                       # one scratch per rank, reused by every registration
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


class _OrderLib(_CountingLib):
    """Logs, in global order, every close of a mapping (by the OWNER's address it maps) and every
    free, so a test can check that no owner frees memory a peer still maps."""

    def __init__(self, slow_close=0.0):
        super().__init__()
        self.log = []
        self.maps = {}                  # mapped address -> owner's allocation address
        self.slow_close = slow_close

    def mp4x_ipc_open_handle(self, h, out):
        owner = int.from_bytes(bytes(h.raw[:8]), "little")
        super().mp4x_ipc_open_handle(h, out)
        with self.lock:
            self.maps[out._obj.value] = owner
        return 0

    def mp4x_ipc_close_handle(self, ptr):
        import time
        time.sleep(self.slow_close)
        v = ptr.value if hasattr(ptr, "value") else int(ptr)
        with self.lock:
            self.log.append(("close", self.maps.get(v)))
        return super().mp4x_ipc_close_handle(ptr)

    def mp4x_ipc_free(self, ptr):
        v = ptr.value if hasattr(ptr, "value") else int(ptr)
        with self.lock:
            self.log.append(("free", v))
        return super().mp4x_ipc_free(ptr)

    def violations(self):
        """Frees of an allocation that some peer closed only AFTERWARDS."""
        bad = []
        for i, (kind, addr) in enumerate(self.log):
            if kind == "free" and any(k == "close" and a == addr for k, a in self.log[i + 1:]):
                bad.append(addr)
        return bad


def _register_cycle(monkeypatch, lib, p=3):
    monkeypatch.setattr(ipc_mod, "CLOSE_PEERS", True)
    monkeypatch.setattr(ipc_mod.native, "hip", lambda: lib)
    monkeypatch.setattr(ipc_mod.torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(ipc_mod.torch.cuda, "synchronize", lambda *a, **k: None)
    server = _Server(p)
    done = [False] * p

    def run(r):
        inst = ipc_mod.IpcAllreduce(_Comm(server, r), nbytes=1 << 16)
        for k in range(3):
            t = _FakeTensor(0x7000000 + r * 0x1000000 + k * 0x100000, 1 << 16)
            assert inst.register(t)
            inst.deregister(t)
        inst.close(sync=False, collective=True)
        done[r] = True

    threads = [threading.Thread(target=run, args=(r,)) for r in range(p)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(30)
    assert not any(t.is_alive() for t in threads), "a rank is stuck in the release barriers"
    assert all(done)


def test_deregistration_and_collective_close_never_free_what_a_peer_maps(monkeypatch):
    """VERDICT r4 Next #1: deregisterBuffer is collective and ordered like memFree — every rank
    closes its mappings of the peers' push scratches (and, at a collective close, of their staging
    and signal buffers), a barrier, and only then does an owner free its memory."""
    monkeypatch.setattr(ipc_mod, "UNORDERED_RELEASE", False)
    lib = _OrderLib(slow_close=0.002)
    _register_cycle(monkeypatch, lib)
    assert sum(1 for k, _ in lib.log if k == "free") >= 3 * 3, lib.log    # the scratches really went
    assert lib.violations() == [], lib.violations()


def test_unordered_release_knob_reproduces_round_4_order(monkeypatch):
    """The test-only knob (MP4X_TEST_UNORDERED_RELEASE) brings back round 4's order: an owner frees
    its push scratch while a peer still maps it — what the checker above exists to catch."""
    monkeypatch.setattr(ipc_mod, "UNORDERED_RELEASE", True)
    lib = _OrderLib(slow_close=0.02)
    _register_cycle(monkeypatch, lib)
    assert lib.violations(), lib.log


class _FakeInst:
    """An IPC instance with nothing to move (0-byte buffer): the first-use probe's exact checks
    pass trivially, so only the agreement / drop / fallback logic is under test."""
    nbytes = 0
    _epoch_dev = None
    made = []

    def __init__(self, comm, nbytes=None, tag="", slots=True):
        self.comm, self.tag, self.closed = comm, tag, None
        _FakeInst.made.append(self)

    def use_order(self, order):
        pass

    def set_spin(self, s, on_current_stream=True):
        pass

    def raise_if_failed(self):
        pass

    def fp8_ok(self, t):
        return False

    def allreduce(self, *a, **k):
        pass

    broadcast_large = scatter_large = gather_large = reduce_scatter_large = allgather_large = allreduce

    def close(self, sync=True, collective=False):
        self.closed = "collective" if collective else "local"
        if collective:
            self.comm.server.call("barrier", self.comm.rank)


def _engines_ipc_large(monkeypatch, inject):
    import torch as _torch
    from mp4x.parallel.device_engine import DeviceEngine
    p = 3
    server = _Server(p)
    monkeypatch.setattr(ipc_mod, "IpcAllreduce", _FakeInst)
    monkeypatch.setattr(_torch.cuda, "synchronize", lambda *a, **k: None)
    if inject is None:
        monkeypatch.delenv("MP4X_IPC_PROBE_INJECT", raising=False)
    else:
        monkeypatch.setenv("MP4X_IPC_PROBE_INJECT", str(inject))
    _FakeInst.made = []
    out = [None] * p

    def run(r):
        e = object.__new__(DeviceEngine)
        e.comm, e.rank, e.p, e.device = _Comm(server, r), r, p, _torch.device("cpu")
        e.ipc_enabled, e._ipc_large, e._ipc_large_failed, e.probe_failures = True, None, False, []
        e._ipc_obj = _FakeInst(e.comm, tag="default")
        got = e.ipc_large()
        out[r] = (got, e)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(p)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(30)
    assert not any(t.is_alive() for t in threads), "a rank is stuck in the probe agreement"
    return out


def test_ipc_large_first_use_probe_failure_falls_back_on_every_rank(monkeypatch):
    """VERDICT r4 Next #2: a lazily created instance is probed before first use; a failure on ONE
    rank drops it on EVERY rank (ordered, collective close) and the default instance serves."""
    out = _engines_ipc_large(monkeypatch, inject=1)
    for got, e in out:
        assert got is e._ipc_obj and got.tag == "default"
        assert e._ipc_large is None and e._ipc_large_failed
        assert e.probe_failures and "rank 1: injected" in e.probe_failures[0]["failures"][0]
    large = [i for i in _FakeInst.made if i.tag == "large"]
    assert len(large) == 3 and all(i.closed == "collective" for i in large)


def test_ipc_large_first_use_probe_pass_keeps_the_instance(monkeypatch):
    out = _engines_ipc_large(monkeypatch, inject=None)
    for got, e in out:
        assert got.tag == "large" and e._ipc_large is got and not e._ipc_large_failed
        assert got.closed is None and not e.probe_failures
