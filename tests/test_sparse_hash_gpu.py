"""K5h, the hash reduce-by-key (csrc/kernels/sparse_hash.hip, VERDICT r5 Next #6): exact against
the deterministic sort path (K5) on integer-valued rows, for SUM / MAX / MIN of f32 / f64 / i32 /
i64, and bit-identical on random floats (both combine in input order), on the BASELINE config-4
shape (the rows one owner receives at 8 ranks: 200k keys x float[64] per rank, half of them
shared) and on small / odd shapes; a key equal to the table's EMPTY marker (-1) is served as a
run of its own."""
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _config4_owner_rows(p=8, nkeys=200_000, dim=64, owner=3, dtype=torch.float32):
    """The (keys, rows) owner ``owner`` receives in config 4: every rank's keys with id % p ==
    owner, rank after rank; integer-valued rows."""
    shared = nkeys // 2
    ks, vs = [], []
    for r in range(p):
        ids = torch.cat([torch.arange(shared), 10_000_000 + r * nkeys + torch.arange(nkeys - shared)])
        ids = ids[ids % p == owner]
        ks.append(ids)
        vs.append(((ids.view(-1, 1) * 7 + torch.arange(dim) + r) % 23 - 11).to(dtype))
    return torch.cat(ks).cuda(), torch.cat(vs).cuda()


def _sorted(k, v, c):
    o = torch.argsort(k)
    return k[o], v[o], c[o]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int32, torch.int64])
@pytest.mark.parametrize("op", [0, 1, 2])           # SUM, MAX, MIN
def test_hash_matches_sort_path(dtype, op):
    from mp4x.ops.device_ops import hash_reduce_by_key, reduce_by_key
    cases = [_config4_owner_rows(dtype=dtype)]
    g = torch.Generator().manual_seed(7)
    for n, dim, nk in ((1, 1, 1), (1000, 3, 50), (4096, 16, 4096), (70000, 5, 900)):
        keys = torch.randint(0, nk, (n,), generator=g) * 7919 - 123456
        rows = torch.randint(-50, 50, (n, dim), generator=g).to(dtype)
        cases.append((keys.cuda(), rows.cuda()))
    for keys, rows in cases:
        hk, hv, hc = _sorted(*hash_reduce_by_key(keys, rows, op))
        sk, sv, sc = reduce_by_key(keys, rows, op)
        assert torch.equal(hk, sk)
        assert torch.equal(hc, sc)
        assert torch.equal(hv, sv), (dtype, op, keys.numel(), (hv != sv).sum().item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float64])
def test_hash_is_bit_identical_to_sort_on_random_floats(dtype):
    """Rows combine in input order in both paths (runs up to 64 rows), through the same segmented
    reduce: random (non-integer) floats give the same bits, for SUM and PROD."""
    from mp4x.ops.device_ops import hash_reduce_by_key, reduce_by_key
    g = torch.Generator(device="cuda").manual_seed(3)
    for n, dim, nk in ((200_000, 64, 60_000), (50_000, 7, 3000), (4096, 16, 512)):   # (runs well under 64)
        keys = torch.randint(0, nk, (n,), device="cuda", generator=g) * 1_000_003
        rows = torch.randn(n, dim, device="cuda", generator=g).to(dtype)
        for op in (0, 3):
            hk, hv, hc = _sorted(*hash_reduce_by_key(keys, rows, op))
            sk, sv, sc = reduce_by_key(keys, rows, op)
            assert torch.equal(hk, sk) and torch.equal(hc, sc)
            assert torch.equal(hv.view(torch.uint8), sv.view(torch.uint8)), (dtype, n, op)


def test_the_empty_marker_key_is_a_key_too():
    """-1 is the table's EMPTY marker: rows keyed -1 bypass the table and form a run of their own."""
    from mp4x.ops.device_ops import hash_reduce_by_key
    keys = torch.tensor([5, -1, 5, 9, -1, -1], device="cuda")
    rows = torch.arange(6, device="cuda").float().view(6, 1).repeat(1, 8)
    k, v, c = _sorted(*hash_reduce_by_key(keys, rows, 0))
    assert k.tolist() == [-1, 5, 9] and c.tolist() == [3, 2, 1]
    assert v[:, 0].tolist() == [1 + 4 + 5, 0 + 2, 3]
    k, v, c = _sorted(*hash_reduce_by_key(torch.full((5,), -1, device="cuda"), torch.ones(5, 4, device="cuda"), 0))
    assert k.tolist() == [-1] and c.tolist() == [5] and v.tolist() == [[5.0] * 4]


def test_sparse_allreduce_in_hash_mode(monkeypatch):
    """The map path with MP4X_SPARSE_RBK=hash: the same set of (key, row) pairs as the sort path."""
    from mp4x.parallel import sparse
    keys, rows = _config4_owner_rows(p=4, nkeys=20000, dim=16)
    from mp4x.operators import Operators, for_dtype, DType
    op = for_dtype(Operators.Float.SUM, DType.F32)
    monkeypatch.setattr(sparse, "RBK_MODE", "sort")
    sk, sv, _ = sparse._reduce_by_key(keys, rows, op)
    monkeypatch.setattr(sparse, "RBK_MODE", "hash")
    hk, hv, _ = sparse._reduce_by_key(keys, rows, op)
    o = torch.argsort(hk)
    assert torch.equal(hk[o], sk) and torch.equal(hv[o], sv)


def _dense_owner_rows(p, owner, nids, ranks, dim, dtype, seed):
    """An owner's received rows of DENSE ids (dictionary numbering): every rank holds a random
    subset of [0, nids); the owner gets the ids with id % p == owner, rank after rank."""
    g = torch.Generator().manual_seed(seed)
    ks, vs = [], []
    for r in range(ranks):
        ids = torch.randperm(nids, generator=g)[: nids * 2 // 3]
        ids = ids[ids % p == owner]
        ks.append(ids)
        vs.append(torch.randn(ids.numel(), dim, generator=g).to(dtype))
    return torch.cat(ks).cuda(), torch.cat(vs).cuda()


@pytest.mark.parametrize("p,dim,dtype", [(8, 64, torch.float32), (2, 3, torch.float32), (4, 8, torch.bfloat16),
                                         (1, 16, torch.float64)])
@pytest.mark.parametrize("op", [0, 1])
def test_dense_reduce_by_key_is_the_sort_path_bit_for_bit(p, dim, dtype, op):
    """K5d (direct addressing of dense ids): the same keys IN THE SAME ORDER (ascending), the same
    values bit for bit (rows combine in input order) and the same counts as the sort path, on
    random floats."""
    from mp4x.ops.device_ops import dense_reduce_by_key, reduce_by_key
    owner = p - 1
    keys, vals = _dense_owner_rows(p, owner, 300_000, 8, dim, dtype, seed=p * 10 + op)
    base, T = int(keys.min()) // p, int(keys.max()) // p - int(keys.min()) // p + 1
    got = dense_reduce_by_key(keys, vals, op, base, p, T)
    assert got is not None
    ref = reduce_by_key(keys, vals, op)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def test_dense_reduce_by_key_refuses_keys_that_are_not_dense():
    """A key outside the table, or two keys on one slot (a wrong stride), is reported (None) —
    the caller takes the sort path."""
    from mp4x.ops.device_ops import dense_reduce_by_key
    keys = torch.tensor([4, 8, 12, 8], device="cuda")
    vals = torch.ones(4, 4, device="cuda")
    assert dense_reduce_by_key(keys, vals, 0, 1, 4, 3) is not None          # slots 0, 1, 2
    assert dense_reduce_by_key(keys, vals, 0, 1, 4, 2) is None              # 12 // 4 - 1 = 2: outside
    assert dense_reduce_by_key(keys + torch.tensor([0, 1, 0, 0], device="cuda"), vals, 0, 1, 4, 3) is None  # 9, 8
    assert dense_reduce_by_key(keys - 20, vals, 0, 0, 4, 3) is None         # negative keys


def test_sparse_allreduce_of_dense_ids_takes_k5d(monkeypatch):
    """allreduce_sparse on dense ids routes the owner's reduce-by-key through K5d (keys ascending
    per owner as before); the fallback on non-dense keys keeps the sort path."""
    from mp4x.ops import device_ops
    from mp4x.parallel import sparse
    calls = []
    real = device_ops.dense_reduce_by_key

    def spy(*a, **k):
        out = real(*a, **k)
        calls.append(out is not None)
        return out
    monkeypatch.setattr(device_ops, "dense_reduce_by_key", spy)
    keys, vals = _dense_owner_rows(4, 1, 100_000, 4, 16, torch.float32, seed=5)
    rng = sparse.KeyRange(int(keys.min()), int(keys.max()), None)
    plan = sparse._dense_plan(rng, 4, keys)
    assert plan is not None
    from mp4x import Operators
    from mp4x.operators import dtype_of_torch, for_dtype
    op = for_dtype(Operators.Float.SUM, dtype_of_torch(vals.dtype))
    uk, uv, _ = sparse._reduce_by_key(keys, vals, op, None, plan)
    rk, rv, _ = device_ops.reduce_by_key(keys, vals, 0)
    assert calls == [True] and torch.equal(uk, rk) and torch.equal(uv, rv)
    # a range 100x wider: the table would be > DENSE_FACTOR x the rows -> no plan (the sort path)
    assert sparse._dense_plan(sparse.KeyRange(0, int(keys.max()) * 100, None), 4, keys) is None
    assert sparse._dense_plan(sparse.KeyRange(-5, int(keys.max()), None), 4, keys) is None


def test_dense_keys_only_is_the_sort_paths_unique_and_counts():
    """K5d without rows (the set operations): unique keys ascending + run lengths, as the sort."""
    from mp4x.ops.device_ops import dense_reduce_by_key, reduce_by_key
    g = torch.Generator().manual_seed(11)
    keys = (torch.randint(0, 50_000, (120_000,), generator=g) * 4 + 1).cuda()     # owner 1 of p = 4
    got = dense_reduce_by_key(keys, None, 0, int(keys.min()) // 4, 4, int(keys.max()) // 4 - int(keys.min()) // 4 + 1)
    ref = reduce_by_key(keys, None, 0)
    assert got is not None and got[1] is None
    assert torch.equal(got[0], ref[0]) and torch.equal(got[2], ref[2])
