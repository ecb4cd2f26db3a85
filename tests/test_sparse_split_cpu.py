"""The split staging layout of the sparse IPC exchanges (mp4x/parallel/sparse.py _split_exchange):
every rank stages its rows at vector 0 and its keys as 16-byte vectors from nmax * V, then ONE
copy plan pulls a row block and a key block from every peer.  CPU: p fake ranks in threads share
host staging buffers; the plan is executed in Python exactly as the kernel's pulls would (after
every rank staged, as the kernel's start barrier guarantees).  Ragged, empty, p up to 8, with and
without rows — against the expected blocks, and the plans' shapes against the kernel's limits."""
import ctypes
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from mp4x.parallel import sparse  # noqa: E402

PLAN_MAX_PULLS = 16            # kPlanMaxPulls (csrc/runtime/ipc.hip)


class _World:
    def __init__(self, p, nbytes):
        self.p = p
        self.bufs = [np.zeros(nbytes, dtype=np.uint8) for _ in range(p)]
        self.bar = threading.Barrier(p)
        self.plans = []


class _Inst:
    def __init__(self, world, rank):
        self.w, self.rank, self.p = world, rank, world.p
        self.nbytes = world.bufs[rank].nbytes
        self._data = ctypes.c_void_p(world.bufs[rank].ctypes.data)

    def _launch_stream(self):
        return 0

    def _plan(self, stage, pulls, src, out_ptr, grid):
        assert not stage and len(pulls) <= PLAN_MAX_PULLS
        assert all(ln <= grid for _, _, ln, _ in pulls)          # the grid covers every item
        self.w.plans.append((self.rank, list(pulls), grid))
        self.w.bar.wait()                                         # every rank staged (start barrier)
        for s0, d0, ln, j in pulls:
            peer = self.w.bufs[j]
            assert (s0 + ln) * 16 <= peer.nbytes
            ctypes.memmove(out_ptr + d0 * 16, peer.ctypes.data + s0 * 16, ln * 16)
        self.w.bar.wait()


class _Engine:
    def __init__(self, world, rank):
        self.p, self.rank = world.p, rank
        self._ipc_obj = _Inst(world, rank)
        self.stats = {}

    def ipc_large(self):
        return None

    def _count(self, k):
        self.stats[k] = self.stats.get(k, 0) + 1


def _stage_split_cpu(keys, vals, vals_ptr, keys16_ptr):
    n = keys.shape[0]
    if vals is not None and n:
        ctypes.memmove(vals_ptr, vals.data_ptr(), vals.numel() * vals.element_size())
    k16 = np.zeros((n, 2), dtype=np.int64)
    k16[:, 0] = keys.numpy()
    if n:
        ctypes.memmove(keys16_ptr, k16.ctypes.data, k16.nbytes)


def _keys_from16_cpu(k16):
    return k16.view(torch.int64).view(-1, 2)[:, 0].clone()


@pytest.fixture(autouse=True)
def _cpu_kernels(monkeypatch):
    from mp4x.ops import device_ops
    monkeypatch.setattr(device_ops, "stage_split", _stage_split_cpu)
    monkeypatch.setattr(device_ops, "keys_from16", _keys_from16_cpu)


def _run(p, fn):
    out, errs = [None] * p, []

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:   # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=body, args=(r,)) for r in range(p)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errs, errs
    return out


def _rows(r, n, dim, dtype):
    if dim == 0:
        return None
    g = torch.Generator().manual_seed(7 + r)
    return torch.randint(-50, 50, (n, dim), generator=g).to(dtype)


@pytest.mark.parametrize("p", [2, 3, 8])
@pytest.mark.parametrize("dim,dtype", [(64, torch.float32), (8, torch.bfloat16), (0, None)])
def test_alltoallv_split_layout(p, dim, dtype):
    rng = np.random.default_rng(p * 100 + dim)
    mat = rng.integers(0, 40, size=(p, p)).tolist()
    mat[p - 1] = [0] * p                                          # an empty sender
    if p > 2:
        for i in range(p):
            mat[i][1] = 0                                         # a rank that receives nothing
    n = [sum(row) for row in mat]
    keys = [torch.arange(n[r], dtype=torch.int64) * 10 + r * 100_000 - 5 for r in range(p)]
    vals = [_rows(r, n[r], dim, dtype) for r in range(p)]
    rb = dim * (torch.empty((), dtype=dtype).element_size() if dtype is not None else 0)
    w = _World(p, max(n) * (rb + 16) + 4096)
    engines = [_Engine(w, r) for r in range(p)]
    got = _run(p, lambda r: sparse._ipc_alltoallv(engines[r], keys[r], vals[r], mat))
    for r in range(p):
        rk, rv = got[r]
        ek = torch.cat([keys[j][sum(mat[j][:r]):sum(mat[j][:r]) + mat[j][r]] for j in range(p)])
        assert torch.equal(rk, ek), r
        if dim:
            ev = torch.cat([vals[j][sum(mat[j][:r]):sum(mat[j][:r]) + mat[j][r]] for j in range(p)])
            assert torch.equal(rv, ev), r
        else:
            assert rv is None
    grids = {g for _, _, g in w.plans}
    assert len(grids) <= 1                                        # one grid on every rank


@pytest.mark.parametrize("p", [2, 8])
def test_allgatherv_split_layout(p):
    sizes = [(7 * r + 3) % 11 for r in range(p)]
    sizes[0] = 0
    keys = [torch.arange(s, dtype=torch.int64) + 1000 * r for r, s in enumerate(sizes)]
    vals = [_rows(r, s, 4, torch.float32) for r, s in enumerate(sizes)]
    w = _World(p, max(sizes) * 32 + 4096)
    engines = [_Engine(w, r) for r in range(p)]
    got = _run(p, lambda r: sparse._ipc_allgatherv(engines[r], keys[r], vals[r], sizes))
    for r in range(p):
        gk, gv = got[r]
        assert torch.equal(gk, torch.cat(keys)) and torch.equal(gv, torch.cat(vals))
        assert engines[r].stats == {"sparse.allgatherv.ipc": 1}


def test_rows_of_odd_width_take_the_transport():
    assert sparse._row_bytes(torch.zeros(3, 3)) == -1
    assert sparse._row_bytes(torch.zeros(3, 4)) == 16
    assert sparse._row_bytes(None) == 0
