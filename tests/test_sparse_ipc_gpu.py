"""The sparse map collectives' ragged exchanges over the IPC mesh (copy-plan kernel pulling a row
block and a 16-byte key block from every peer) with real processes on one GPU, against a
reference built from every rank's seed: exact for integer-valued rows, f32 and bf16,
p = 2 / 3 / 4 / 8 (8: 2p = 16 pulls per plan), plus the fallback for rows that are not whole
16-byte vectors and empty ranks."""
import pytest

torch = pytest.importorskip("torch")

from spawn_ranks import run_spawn  # noqa: E402

pytestmark = pytest.mark.gpu


def _data(r, dim, dtype, n, shift=0):
    g = torch.Generator().manual_seed(100 + r)
    keys = torch.randperm(3 * n, generator=g)[:n].to(torch.int64) + shift  # overlapping id ranges
    vals = torch.randint(-8, 8, (n, dim), generator=g).to(dtype)
    return keys, vals


def _sparse_fn(comm, dim, dtype_name, n, empty_rank, shift):
    from mp4x import Operators
    dtype = getattr(torch, dtype_name)
    r, p = comm.getRank(), comm.getSlaveNum()
    k, v = _data(r, dim, dtype, 0 if r == empty_rank else n, shift)
    eng = comm.device
    before = dict(eng.stats)
    op = Operators.Float.SUM if dtype == torch.float32 else Operators.BFloat16.SUM
    rk, rv = comm.allreduceSparse(k.cuda(), v.cuda(), op)
    gk, gv, sizes = comm.allgatherSparse(k.cuda(), v.cuda())
    torch.cuda.synchronize()
    used = {x: c - before.get(x, 0) for x, c in eng.stats.items() if c != before.get(x, 0)}
    # numpy, not tensors: a torch tensor crosses the result queue as a shared-memory fd that
    # dies with the worker process
    return rk.cpu().numpy(), rv.float().cpu().numpy(), gk.cpu().numpy(), gv.float().cpu().numpy(), sizes, used


# shift: the keys' range — non-negative ids let the reduce-by-key sort only the bits the ranks'
# key ranges (carried by the count exchange) need; negative ids (-2**40 + ...) the full width
@pytest.mark.parametrize("p,dim,dtype,empty,shift", [(2, 64, "float32", -1, 0), (3, 8, "bfloat16", -1, -(1 << 40)),
                                                     (4, 64, "float32", 2, 1 << 50), (3, 3, "float32", -1, 0),
                                                     (8, 16, "float32", 5, 0)])
def test_sparse_exchange_over_ipc_exact(p, dim, dtype, empty, shift):
    n = 20000
    out = run_spawn(p, _sparse_fn, args=(dim, dtype, n, empty, shift))
    dt = getattr(torch, dtype)
    ins = [_data(j, dim, dt, 0 if j == empty else n, shift) for j in range(p)]
    ref = {}
    for k, v in ins:
        for kk, vv in zip(k.tolist(), v.float()):
            ref[kk] = ref[kk] + vv if kk in ref else vv.clone()
    allk = torch.cat([k for k, _ in ins])
    allv = torch.cat([v.float() for _, v in ins])
    ipc = dim * torch.empty((), dtype=dt).element_size() % 16 == 0
    for r, (rk, rv, gk, gv, sizes, used) in out.items():
        rk, rv, gk, gv = (torch.from_numpy(x) for x in (rk, rv, gk, gv))
        assert sorted(rk.tolist()) == sorted(ref)
        got = dict(zip(rk.tolist(), rv))
        assert all(torch.equal(got[kk], ref[kk]) for kk in ref), r
        assert torch.equal(gk, allk) and torch.equal(gv, allv) and sizes == [k.numel() for k, _ in ins]
        if ipc:
            assert used.get("sparse.a2a.ipc") == 1 and used.get("sparse.allgatherv.ipc") == 2, used
        else:
            assert "sparse.a2a.ipc" not in used, used


def _a2a_fn(comm, dim, dtype_name):
    import torch
    from mp4x import Mp4jException  # noqa: F401
    r, p = comm.getRank(), comm.getSlaveNum()
    dt = getattr(torch, dtype_name)
    counts = [(r + 1) * 37 + 11 * j for j in range(p)]
    rows = []
    for j in range(p):
        blk = torch.arange(counts[j] * dim, device="cuda").view(counts[j], dim).to(dt) + 1000 * r + 100 * j
        rows.append(blk)
    send = torch.cat(rows)
    recv, rc = comm.alltoallArray(send, counts)
    exp_counts = [(j + 1) * 37 + 11 * r for j in range(p)]
    ok = rc == exp_counts
    off = 0
    for j in range(p):
        exp = torch.arange(exp_counts[j] * dim, device="cuda").view(exp_counts[j], dim).to(dt) + 1000 * j + 100 * r
        ok = ok and bool(torch.equal(recv[off:off + exp_counts[j]], exp))
        off += exp_counts[j]
    torch.cuda.synchronize()
    return ok, dict(comm.device.stats)


@pytest.mark.parametrize("p,dim,dtype_name,ipc", [(2, 16, "float32", True), (4, 8, "bfloat16", True),
                                                   (3, 3, "float32", False)])
def test_alltoallv_rows_over_ipc(p, dim, dtype_name, ipc):
    """alltoallArray (expert-parallel routing): rows of whole 16-byte vectors go through ONE IPC
    copy-plan kernel (every rank pulls its block from every peer at once); other row widths take
    the transport's all-to-all.  Ragged counts, exact."""
    out = run_spawn(p, _a2a_fn, args=(dim, dtype_name))
    for r, (ok, st) in out.items():
        assert ok, r
        assert (st.get("all_to_all_v.ipc", 0) == 1) == ipc, st


def test_sparse_exchange_too_large_for_staging_takes_the_transport():
    """Payloads above both staging buffers (shrunk here to 1 / 2 MiB): the owner exchange counts
    (K4b first half), finds no instance that fits on ANY rank, scatters into plain tensors and
    runs the transport's all-to-all; results exact, no IPC exchange counted."""
    p, dim, n = 3, 64, 20000
    env = {"MP4X_IPC_BYTES": str(1 << 20), "MP4X_IPC_LARGE_BYTES": str(2 << 20)}
    out = run_spawn(p, _sparse_fn, args=(dim, "float32", n, -1, 0), env=env)
    ins = [_data(j, dim, torch.float32, n) for j in range(p)]
    ref = {}
    for k, v in ins:
        for kk, vv in zip(k.tolist(), v.float()):
            ref[kk] = ref[kk] + vv if kk in ref else vv.clone()
    for r, (rk, rv, gk, gv, sizes, used) in out.items():
        rk, rv = torch.from_numpy(rk), torch.from_numpy(rv)
        assert sorted(rk.tolist()) == sorted(ref)
        got = dict(zip(rk.tolist(), rv))
        assert all(torch.equal(got[kk], ref[kk]) for kk in ref), r
        assert "sparse.a2a.ipc" not in used and "sparse.allgatherv.ipc" not in used, used


def _setops_fn(comm, n):
    g = torch.Generator().manual_seed(50 + comm.getRank())
    ids = torch.randint(0, 3 * n, (n,), generator=g).cuda()          # dense ids, duplicates
    u = comm.allreduceSetUnion(ids)
    i = comm.allreduceSetIntersection(ids)
    torch.cuda.synchronize()
    return u.cpu().numpy(), i.cpu().numpy()


def test_set_ops_over_ipc_with_dense_ids():
    """Set union / intersection of dense ids across real processes: the owners' de-duplication
    runs K5d keys-only (unique keys ascending + counts); against Python sets."""
    p, n = 3, 30000
    out = run_spawn(p, _setops_fn, args=(n,))
    sets = []
    for r in range(p):
        g = torch.Generator().manual_seed(50 + r)
        sets.append(set(torch.randint(0, 3 * n, (n,), generator=g).tolist()))
    union, inter = set.union(*sets), set.intersection(*sets)
    for r, (u, i) in out.items():
        assert sorted(u.tolist()) == sorted(union) and len(u) == len(union), r
        assert sorted(i.tolist()) == sorted(inter) and len(i) == len(inter), r
