"""memAlloc under the chunk pool (``MP4X_VMM_POLICY=chunks``, the default) on CPU: a fake native
library stands in for the VMM calls (memfd files for the exported dmabuf fds, tagged with the
owning rank and chunk), the fd exchange is the real SCM_RIGHTS one between rank threads.

Pinned: the chunk sizes (power-of-two decomposition); a freed chunk serves a later allocation of
ANOTHER size; only NEW chunks' fds travel (a reused chunk is mapped again from the handle every
peer kept); every rank's view of a peer maps exactly that peer's chunks, in order; memFree unmaps
every view and releases nothing; close() releases every chunk and imported handle once.
"""
import os
import threading

import pytest

from mp4x.exceptions import Mp4jException
from mp4x.parallel import ipc as ipc_mod
from mp4x.parallel import vmm
from mp4x.parallel.vmm import chunk_sizes

from test_ipc_setup_consensus import _CountingLib, _Comm, _Server

MiB = 1 << 20


def test_chunk_sizes():
    g = 2 * MiB
    assert chunk_sizes(1, g, 512 * MiB) == [2 * MiB]
    assert chunk_sizes(10 * MiB, g, 512 * MiB) == [8 * MiB, 2 * MiB]
    assert chunk_sizes(12 * MiB + 1, g, 512 * MiB) == [8 * MiB, 4 * MiB, 2 * MiB]
    assert chunk_sizes((1 << 30) + 6 * MiB, g, 512 * MiB) == [512 * MiB] * 2 + [4 * MiB, 2 * MiB]
    # a cap that is not a power-of-two number of units rounds down to one
    assert chunk_sizes(20 * MiB, g, 7 * MiB) == [4 * MiB] * 5
    # 4 KiB granularity: still 2 MiB units (large fragments)
    assert chunk_sizes(3 * MiB, 4096, 512 * MiB) == [4 * MiB]
    # a granularity that does not divide 2 MiB is the unit itself
    assert chunk_sizes(10 * 3 * MiB, 3 * MiB, 12 * MiB) == [12 * MiB, 12 * MiB, 6 * MiB]
    for n in (1, 5 * MiB, 77 * MiB + 3, 3 << 30):
        cs = chunk_sizes(n, g, 512 * MiB)
        assert sum(cs) >= n and sum(cs) - n < 2 * MiB and cs == sorted(cs, reverse=True)
    with pytest.raises(Mp4jException):
        chunk_sizes(0, g)


class _VmmLib(_CountingLib):
    def __init__(self, tls):
        super().__init__()
        self.tls = tls
        self.tags = {}            # handle -> "owner:chunk serial"
        self.maps = {}            # va -> [tags]
        self.unmapped = []
        self.released = []
        self.imports = 0
        self.creates = 0
        self.serial = {}
        self.by_rank = {}         # rank -> [creates, imports]

    def _h(self, tag):
        h = self._addr()
        self.tags[h] = tag
        return h

    def mp4x_vmm_granularity(self, g):
        g._obj.value = 2 * MiB
        return 0

    def mp4x_vmm_chunk_create(self, size, h, fd):
        r = self.tls.rank
        with self.lock:
            k = self.serial.get(r, 0)
            self.serial[r] = k + 1
            self.creates += 1
            self.by_rank.setdefault(r, [0, 0])[0] += 1
        tag = f"{r}:{k}:{size}"
        f = os.memfd_create(tag)
        os.write(f, tag.encode())
        h._obj.value = self._h(tag)
        fd._obj.value = f
        return 0

    def mp4x_vmm_chunk_import(self, fd, h):
        with self.lock:
            self.imports += 1
            self.by_rank.setdefault(self.tls.rank, [0, 0])[1] += 1
        h._obj.value = self._h(os.pread(fd, 64, 0).decode())
        return 0

    def mp4x_vmm_map_chunks(self, handles, sizes, n, va):
        v = self._addr()
        self.maps[v] = [self.tags[handles[i]] for i in range(n)]
        va._obj.value = v
        return 0

    def mp4x_vmm_unmap_chunks(self, va, sizes, n):
        self.unmapped.append(va.value)
        return 0

    def mp4x_vmm_chunk_release(self, h):
        self.released.append(h)
        return 0


class _T:
    """What vmm.tensor_at returns here: slicing / view keep the base pointer."""

    def __init__(self, ptr):
        self.ptr = ptr

    def __getitem__(self, _):
        return self

    def view(self, _):
        return self

    def data_ptr(self):
        return self.ptr


def test_chunk_pool_reuses_chunks_across_sizes_and_sends_only_new_ones(monkeypatch):
    p = 3
    tls = threading.local()
    lib = _VmmLib(tls)
    monkeypatch.setattr(ipc_mod, "VMM_POLICY", "chunks")
    monkeypatch.setattr(ipc_mod, "PUSH_ON", True)
    monkeypatch.setattr(ipc_mod.native, "hip", lambda: lib)
    monkeypatch.setattr(ipc_mod.torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(ipc_mod.torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(vmm, "tensor_at", lambda ptr, nb, dt, dev, owner=None: _T(ptr))
    server = _Server(p)
    out = [None] * p
    errs = []
    q0 = vmm.quarantined_bytes()

    def run(r):
        tls.rank = r
        try:
            inst = ipc_mod.IpcAllreduce(_Comm(server, r), nbytes=1 << 16)
            rows = []
            for mb in (10, 12, 10, 3):
                before = list(lib.by_rank.get(r, [0, 0]))
                t = inst.mem_alloc(mb * MiB, ipc_mod.torch.float32)
                reg = inst._regs[(t.data_ptr(), mb * MiB)]
                views = [lib.maps[v] for v in reg.peers]
                scr = [lib.maps[v] for v in reg.scratch]
                now = lib.by_rank.get(r, [0, 0])
                rows.append((mb, views, scr, (now[0] - before[0], now[1] - before[1])))
                inst.mem_free(t)
                assert all(v in lib.unmapped for v in reg.peers + reg.scratch)
            out[r] = (rows, sorted(c.size for c in inst._chunk_pool.owned), inst)
        except Exception as e:   # noqa: BLE001
            errs.append((r, repr(e)))
            raise

    threads = [threading.Thread(target=run, args=(r,)) for r in range(p)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    assert not any(t.is_alive() for t in threads), "a rank is stuck"
    assert not errs, errs
    for r, (rows, owned, _) in enumerate(out):
        for k, (mb, views, scr, _) in enumerate(rows):
            for j in range(p):
                # rank r's view of rank j: rank j's chunks, the decomposition of the size, and
                # the very chunks rank j mapped for itself
                assert [int(tag.split(":")[0]) for tag in views[j]] == [j] * len(views[j])
                assert [int(tag.split(":")[2]) for tag in views[j]] == chunk_sizes(mb * MiB, 2 * MiB)
                assert views[j] == out[j][0][k][1][j] and scr[j] == out[j][0][k][2][j]
        # 10 MiB = 8+2 (+ 8 MiB of scratch), 12 MiB = 8+4 (+8): one new 4 MiB chunk, imported by
        # each of the 2 peers; 10 MiB again and 3 MiB (4, +2 scratch) reuse everything
        assert rows[0][3] == (3, 2 * 3)
        assert rows[1][3] == (1, 2 * 1)
        assert rows[2][3] == (0, 0) and rows[3][3] == (0, 0)
        assert owned == [2 * MiB, 4 * MiB, 8 * MiB, 8 * MiB]
    # the VA the cycles keep reserved (documented growth, vmm._VaQuarantine): per rank and cycle,
    # its own range and p - 1 imported views of the tensor and of the push scratch
    def span(nbytes):
        return sum(chunk_sizes(nbytes, 2 * MiB))
    per_cycle = {mb: p * (span(mb * MiB) + span((p - 1) * (-(-(mb * MiB // 16) // p)) * 16)) for mb in (10, 12, 3)}
    assert vmm.quarantined_bytes() - q0 == p * sum(per_cycle[mb] for mb in (10, 12, 10, 3))
    for _, _, inst in out:
        inst.close(sync=False)
    owned_handles = {h for h, tag in lib.tags.items()}
    assert len(set(lib.released)) == len(lib.released)          # nothing released twice
    assert len(lib.released) == lib.creates + lib.imports        # ... and everything once, at close
    assert set(lib.released) <= owned_handles


def test_chunks_sent_by_a_failed_allocation_are_never_reused(monkeypatch):
    """A peer fails to import a new chunk: memAlloc raises on every rank, the chunks that
    allocation sent are released and dropped (a peer may not hold them), and the next memAlloc
    of that size creates and sends new ones — it does not map a chunk some peer never got."""
    p = 3
    tls = threading.local()
    lib = _VmmLib(tls)
    orig_import = lib.mp4x_vmm_chunk_import
    fail = {"on": False}

    def flaky_import(fd, h):
        if fail["on"] and tls.rank == 2:
            return 1
        return orig_import(fd, h)
    lib.mp4x_vmm_chunk_import = flaky_import
    monkeypatch.setattr(ipc_mod, "VMM_POLICY", "chunks")
    monkeypatch.setattr(ipc_mod, "PUSH_ON", True)
    monkeypatch.setattr(ipc_mod.native, "hip", lambda: lib)
    monkeypatch.setattr(ipc_mod.torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(ipc_mod.torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(vmm, "tensor_at", lambda ptr, nb, dt, dev, owner=None: _T(ptr))
    server = _Server(p)
    out = [None] * p
    errs = []

    def run(r):
        tls.rank = r
        try:
            inst = ipc_mod.IpcAllreduce(_Comm(server, r), nbytes=1 << 16)
            t = inst.mem_alloc(10 * MiB, ipc_mod.torch.float32)
            inst.mem_free(t)
            server.call("barrier", r)
            if r == 0:
                fail["on"] = True
            server.call("barrier", r)
            raised = False
            try:
                inst.mem_alloc(12 * MiB, ipc_mod.torch.float32)      # a new 4 MiB chunk: import fails on rank 2
            except Mp4jException:
                raised = True
            server.call("barrier", r)
            if r == 0:
                fail["on"] = False
            server.call("barrier", r)
            released_before = len(lib.released)
            t = inst.mem_alloc(12 * MiB, ipc_mod.torch.float32)
            reg = inst._regs[(t.data_ptr(), 12 * MiB)]
            views = [lib.maps[v] for v in reg.peers]
            inst.mem_free(t)
            out[r] = (raised, views, sorted(c.size for c in inst._chunk_pool.owned), released_before, inst)
        except Exception as e:   # noqa: BLE001
            errs.append((r, repr(e)))
            raise

    threads = [threading.Thread(target=run, args=(r,)) for r in range(p)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    assert not any(t.is_alive() for t in threads) and not errs, errs
    for r, (raised, views, owned, released_before, _) in enumerate(out):
        assert raised                                             # every rank, together
        for j in range(p):                                        # the retry maps real chunks everywhere
            assert [int(tag.split(":")[0]) for tag in views[j]] == [j] * len(views[j])
            assert views[j] == out[j][1][j]
        assert owned.count(4 * MiB) == 1                          # the discarded 4 MiB chunk is gone
        assert released_before >= p                               # ... released (one per rank at least)
    for *_, inst in out:
        inst.close(sync=False)
