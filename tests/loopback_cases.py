"""Device-engine scenarios driven by p virtual ranks (threads) over LoopbackColl.

Shared by tests/test_loopback_cpu.py (CPU tensors) and tests/test_loopback_gpu.py (one MI355X,
real HIP kernels): a2a two-shot with rank-ordered reduce, fp8 / bf16 codecs, p2p
gather/scatter/allgather-v, RCCL-shaped paths, sparse map / set ops.
"""
import threading

import torch

from mp4x import CommUtils, Operators
from mp4x.operands import Operands
from mp4x.operators import CustomOperator
from mp4x.parallel.coll import loopback_engines


def run_virtual(p, fn, device="cpu"):
    engines = loopback_engines(p, device=device)
    out = [None] * p
    errs = []

    def body(r):
        try:
            if device != "cpu":
                torch.cuda.set_device(torch.device(device))
            out[r] = fn(engines[r], r, p)
        except BaseException as e:  # noqa
            import traceback
            errs.append(traceback.format_exc())
            engines[r].coll.hub.bar.abort()

    ths = [threading.Thread(target=body, args=(r,)) for r in range(p)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    if errs:
        raise AssertionError(errs[0])
    return out


def dense_cases(eng, r, p):
    dev = eng.device
    n = 4099
    for algo in ("rccl", "a2a", "rhd"):
        eng.algo = algo
        t = torch.full((n,), float(r + 1), device=dev)
        eng.allreduce(t, 2, n - 3, Operators.Float.SUM)
        assert torch.all(t[2:n - 3] == p * (p + 1) / 2) and t[0] == r + 1
    # recursive halving/doubling with ops / dtypes RCCL lacks (K1 combines every round)
    eng.algo = "rhd"
    x = torch.full((n,), 1 << r, dtype=torch.int16, device=dev)
    eng.allreduce(x, 0, n, Operators.Short.BITS_OR)
    assert torch.all(x == (1 << p) - 1)
    b = torch.full((7,), float(r + 1), dtype=torch.bfloat16, device=dev)
    eng.allreduce(b, 0, 7, Operators.BFloat16.MAX)
    assert torch.all(b == p)
    eng.algo = "auto"
    x = torch.full((n,), 1 << r, dtype=torch.int16, device=dev)
    eng.allreduce(x, 0, n, Operators.Short.BITS_OR)
    assert torch.all(x == (1 << p) - 1)
    # rank-ordered non-commutative op
    op = CustomOperator(lambda a, b: a * 10 + b, vectorized=True)
    t = torch.full((p * 5,), float(r + 1), dtype=torch.float64, device=dev)
    eng.allreduce(t, 0, p * 5, op)
    e = 1.0
    for i in range(1, p):
        e = e * 10 + (i + 1)
    assert torch.all(t == e)
    # ragged reduce-scatter / allgather, gather / scatter / broadcast / reduce
    counts = [300 + 17 * i for i in range(p)]
    fr = CommUtils.getFromsFromCount(1, counts, p)
    to = CommUtils.getTosFromCount(1, counts, p)
    t = torch.zeros(2 + sum(counts), device=dev)
    for i in range(p):
        t[fr[i]:to[i]] = i + 1
    eng.reduce_scatter(t, fr, to, Operators.Float.SUM)
    assert torch.all(t[fr[r]:to[r]] == (r + 1) * p)
    t = torch.full((2 + sum(counts),), -1.0, device=dev)
    t[fr[r]:to[r]] = r
    eng.allgather(t, fr, to)
    for i in range(p):
        assert torch.all(t[fr[i]:to[i]] == i)
    root = p - 1
    t = torch.full((2 + sum(counts),), -1.0, device=dev)
    t[fr[r]:to[r]] = r
    eng.gather(t, fr, to, root)
    if r == root:
        for i in range(p):
            assert torch.all(t[fr[i]:to[i]] == i)
    t = torch.full((2 + sum(counts),), -1.0, device=dev)
    if r == root:
        for i in range(p):
            t[fr[i]:to[i]] = i
    eng.scatter(t, fr, to, root)
    assert torch.all(t[fr[r]:to[r]] == r)
    t = torch.full((n,), 7.0 if r == 0 else 0.0, device=dev)
    eng.broadcast(t, 0, n, 0)
    assert torch.all(t == 7)
    t = torch.full((n,), 1 << r, dtype=torch.int64, device=dev)
    eng.reduce(t, 0, n, Operators.Long.BITS_XOR, None, root)
    if r == root:
        assert torch.all(t == (1 << p) - 1)
    return True


def codec_cases(eng, r, p):
    dev = eng.device
    n = 256 * 40 + 64
    g = torch.Generator(device=dev).manual_seed(100 + r)
    x = torch.randn(n, device=dev, generator=g)
    xs = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(100 + j)) for j in range(p)]
    ref = sum(xs)
    y = x.clone()
    eng.allreduce(y, 0, n, Operators.Float.SUM, Operands.FLOAT_OPERAND(codec="fp8"))
    assert eng.stats.get("allreduce.fp8", 0) == 1
    err = (y - ref).abs().max().item()
    assert err < 0.25 * p, err                   # e4m3: ~2^-4 relative per block, twice quantised
    # unaligned [from, to) view: the staged (padded) form; the aligned call above quantised in place
    w = x.clone()
    eng.allreduce(w, 1, n - 2, Operators.Float.SUM, Operands.FLOAT_OPERAND(codec="fp8"))
    assert (w[1:n - 2] - ref[1:n - 2]).abs().max().item() < 0.25 * p
    assert w[0] == x[0] and torch.equal(w[n - 2:], x[n - 2:])
    z = x.clone()
    eng.allreduce(z, 0, n, Operators.Float.SUM, Operands.FLOAT_OPERAND(codec="bf16"))
    assert (z - ref).abs().max().item() < 0.05 * p
    return True


def sparse_cases(eng, r, p):
    from mp4x.parallel.sparse import allreduce_sparse, set_intersection, set_union, allreduce_map_device
    dev = eng.device
    ids = torch.tensor(list(range(50)) + [10_000 + r], dtype=torch.int64, device=dev)
    vals = torch.ones(51, 8, device=dev) * (r + 1)
    k, v = allreduce_sparse(eng, ids, vals, Operators.Float.SUM)
    got = dict(zip(k.tolist(), v[:, 0].tolist()))
    assert len(got) == 50 + p and got[3] == p * (p + 1) / 2 and got[10_000 + r] == r + 1
    u = set_union(eng, torch.tensor([r, 99, 99], dtype=torch.int64, device=dev))
    assert sorted(u.tolist()) == sorted(set(range(p)) | {99})
    i = set_intersection(eng, torch.tensor([4, 5, 77 + r], dtype=torch.int64, device=dev))
    assert sorted(i.tolist()) == [4, 5]
    m = {f"w{j}": torch.full((3,), float(r), device=dev) for j in range(20)}
    out = allreduce_map_device(eng, m, Operators.Float.MAX)
    assert len(out) == 20 and torch.all(out["w7"] == p - 1)
    map_family_cases(eng, r, p)
    return True


def map_family_cases(eng, r, p):
    """reduce / gather (K8 dedupe) / allgather / broadcast maps and their tensor forms, ragged
    and empty inputs, every value dtype the segment kernels take."""
    from mp4x.parallel import sparse as S
    dev = eng.device
    root = p - 1
    # reduceMap: union reduced at root; rank r contributes keys 0..r (rank 0: a single key)
    m = {f"k{j}": torch.full((2,), float(j + r), device=dev) for j in range(r + 1)}
    out = S.reduce_map_device(eng, m, Operators.Float.SUM, root)
    if r == root:
        assert len(out) == p
        for j in range(p):   # key j is present on ranks j..p-1
            assert torch.all(out[f"k{j}"] == sum(j + q for q in range(j, p)))
    # gatherMap: duplicate key "dup" keeps the lowest rank's value; rank 1 sends an empty map
    g = {} if r == 1 else {"dup": torch.tensor([float(r)], device=dev), f"own{r}": torch.ones(1, device=dev)}
    got = S.gather_map_device(eng, g, root)
    if r == root:
        expect_dup = 0.0
        assert float(got["dup"]) == expect_dup and len(got) == 1 + sum(1 for q in range(p) if q != 1)
    # allgatherMap: list indexed by rank
    lst = S.allgather_map_device(eng, {f"a{r}": torch.full((4,), r, dtype=torch.int16, device=dev)})
    assert len(lst) == p and all(int(lst[q][f"a{q}"][0]) == q for q in range(p))
    # broadcastMap: non-root ranks start empty
    b = {"x": torch.arange(6, dtype=torch.float64, device=dev).view(2, 3)} if r == 0 else {}
    bb = S.broadcast_map_device(eng, b, 0)
    assert list(bb) == ["x"] and bb["x"].shape == (2, 3) and float(bb["x"][1, 2]) == 5.0
    # tensor forms: gather with int8 rows (scalar segment kernel), allgather counts
    keys = torch.tensor([7, 100 + r], dtype=torch.int64, device=dev)
    vals = torch.full((2, 3), r, dtype=torch.int8, device=dev)
    gk, gv = S.gather_sparse(eng, keys, vals, 0)
    if r == 0:
        d = dict(zip(gk.tolist(), gv[:, 0].tolist()))
        assert d[7] == 0 and len(d) == 1 + p and d[100 + p - 1] == p - 1
    ak, av, sizes = S.allgather_sparse(eng, keys, vals)
    assert sizes == [2] * p and ak.tolist()[2 * r + 1] == 100 + r
    # ragged all-to-all (EP-style routing): rank r sends j+1 rows to rank j
    counts = [j + 1 for j in range(p)]
    send = torch.cat([torch.full((j + 1, 2), float(r * 10 + j), device=dev) for j in range(p)])
    recv, rc = eng.all_to_all_v(send, counts)
    assert rc == [r + 1] * p
    for q in range(p):
        assert torch.all(recv[q * (r + 1):(q + 1) * (r + 1)] == q * 10 + r)


def zs_cases(eng, r, p):
    """Lossless zero-suppression allreduce (compress=True on device tensors): exact results for
    sparse, dense and all-zero data, 1/2/8-byte words, ragged chunks."""
    dev = eng.device
    n = 3 * 256 * p + 77
    g = torch.Generator().manual_seed(7 + r)
    dense = torch.randn(n, generator=g).to(dev)
    sparse = dense * (torch.rand(n, generator=g) < 0.05).to(dev)
    for x, name in ((sparse, "sparse"), (dense, "dense")):
        xs = []
        for q in range(p):
            gq = torch.Generator().manual_seed(7 + q)
            d = torch.randn(n, generator=gq)
            xs.append((d * (torch.rand(n, generator=gq) < 0.05)) if name == "sparse" else d)
        y = x.clone()
        eng.allreduce(y, 0, n, Operators.Float.MAX, Operands.FLOAT_OPERAND(compress=True))
        ref = xs[0].clone()
        for q in range(1, p):
            ref = torch.maximum(ref, xs[q])
        assert torch.equal(y.cpu(), ref), name
    assert eng.stats.get("allreduce.zs", 0) >= 2
    for dt, op in ((torch.int8, Operators.Byte.BITS_XOR), (torch.int16, Operators.Short.SUM),
                   (torch.int64, Operators.Long.SUM)):
        v = torch.zeros(n, dtype=dt, device=dev)
        v[r::97] = r + 1
        eng.allreduce(v, 0, n, op, Operands.LONG_OPERAND(compress=True))
        exp = torch.zeros(n, dtype=torch.int64)
        for q in range(p):
            if op is Operators.Byte.BITS_XOR:
                exp[q::97] ^= q + 1
            else:
                exp[q::97] += q + 1
        assert torch.equal(v.cpu().long(), exp), dt
    z = torch.zeros(n, device=dev)
    eng.allreduce(z, 0, n, Operators.Float.SUM, Operands.FLOAT_OPERAND(codec="zs"))   # all-zero input
    assert torch.all(z == 0)
    return True


def scatter_family_cases(eng, r, p):
    """scatterMap / reduceScatterMap with tensor values (explicit destinations)."""
    from mp4x.parallel import sparse as S
    dev = eng.device
    lst = [{f"k{j}": torch.full((2,), float(r * 10 + j), device=dev), "common": torch.ones(2, device=dev)}
           for j in range(p)]
    got = S.reduce_scatter_map_device(eng, lst, Operators.Float.SUM)
    assert set(got) == {f"k{r}", "common"}
    assert torch.all(got["common"] == p) and torch.all(got[f"k{r}"] == sum(q * 10 + r for q in range(p)))
    root = p - 1
    sl = [({f"s{j}": torch.full((3,), float(j), device=dev)} if j != 1 else {}) for j in range(p)] \
        if r == root else None
    mine = S.scatter_map_device(eng, sl, root)
    if r == 1:
        assert mine == {}
    else:
        assert list(mine) == [f"s{r}"] and torch.all(mine[f"s{r}"] == r)
    return True
