"""Numerics of the hand-written HIP kernels vs plain PyTorch references (GPU only)."""
import pytest

torch = pytest.importorskip("torch")

from mp4x.operators import OpCode, DType  # noqa: E402

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _native():
    from mp4x.ops import device_ops, native
    native.hip()
    return device_ops


def _ref_reduce(xs, code, dtype):
    acc = xs[0].clone()
    for x in xs[1:]:
        if code == OpCode.SUM:
            acc = acc + x
        elif code == OpCode.PROD:
            acc = acc * x
        elif code == OpCode.MAX:
            acc = torch.maximum(acc, x)
        elif code == OpCode.MIN:
            acc = torch.minimum(acc, x)
        elif code == OpCode.BAND:
            acc = acc & x
        elif code == OpCode.BOR:
            acc = acc | x
        elif code == OpCode.BXOR:
            acc = acc ^ x
    return acc


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int32, torch.int64, torch.int16, torch.int8])
@pytest.mark.parametrize("code", [OpCode.SUM, OpCode.MAX, OpCode.MIN, OpCode.PROD])
@pytest.mark.parametrize("nin", [1, 2, 3, 8, 11])
def test_reduce_arith(dtype, code, nin):
    K = _native()
    n = 100_003  # odd: exercises the vector body and the scalar tail
    g = torch.Generator(device=DEV).manual_seed(nin * 31 + int(code))
    if dtype.is_floating_point:
        xs = [torch.randn(n, device=DEV, dtype=dtype, generator=g) for _ in range(nin)]
        if code == OpCode.PROD:
            xs = [x.clamp(-1.5, 1.5) for x in xs]
    else:
        xs = [torch.randint(-50, 50, (n,), device=DEV, dtype=dtype, generator=g) for _ in range(nin)]
    out = torch.empty_like(xs[0])
    K.reduce_(out, xs, int(code))
    if dtype.is_floating_point:
        ref = _ref_reduce([x.double() for x in xs], code, dtype).to(dtype)
        tol = 1e-5 if dtype == torch.float32 else 1e-12
        torch.testing.assert_close(out, ref, rtol=tol * nin, atol=tol * nin)
    else:
        # integer math wraps (two's complement) like the reference's Java operators
        ref = _ref_reduce([x.long() for x in xs], code, dtype)
        bits = torch.iinfo(dtype).bits
        ref = ((ref + (1 << (bits - 1))) % (1 << bits)) - (1 << (bits - 1)) if bits < 64 else ref
        assert torch.equal(out.long(), ref)


@pytest.mark.parametrize("dtype", [torch.int32, torch.int64, torch.int16, torch.int8])
@pytest.mark.parametrize("code", [OpCode.BAND, OpCode.BOR, OpCode.BXOR])
def test_reduce_bitwise(dtype, code):
    K = _native()
    n = 65_537
    xs = [torch.randint(-100, 100, (n,), device=DEV, dtype=dtype) for _ in range(4)]
    out = xs[0].clone()
    K.reduce_(out, [out] + xs[1:], int(code))
    assert torch.equal(out, _ref_reduce(xs, code, dtype))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_reduce_half_accumulates_in_f32(dtype):
    K = _native()
    n = 1 << 20
    xs = [torch.randn(n, device=DEV).to(dtype) for _ in range(8)]
    out = torch.empty_like(xs[0])
    K.reduce_(out, xs, int(OpCode.SUM))
    ref = sum(x.float() for x in xs).to(dtype)   # one rounding, like the kernel
    torch.testing.assert_close(out, ref, rtol=0, atol=0)


def test_reduce_loc_ops():
    K = _native()
    import numpy as np
    from mp4x.operators import Operators
    n = 10_001
    rng = np.random.default_rng(0)
    vals = [rng.integers(-5, 5, n).astype(np.float32) for _ in range(3)]   # many ties
    words = []
    for k, v in enumerate(vals):
        bits = (v.view(np.uint32).astype(np.uint64) << np.uint64(32)) | np.uint64(k)
        words.append(bits.view(np.float64))
    for op in (Operators.Double.FLOAT_MAX_LOC, Operators.Double.FLOAT_MIN_LOC):
        acc = words[0].copy()
        for w in words[1:]:
            op.reduce_into(acc, w)
        ts = [torch.from_numpy(w).to(DEV) for w in words]
        out = torch.empty_like(ts[0])
        K.reduce_(out, ts, int(op.code))
        assert np.array_equal(out.cpu().numpy().view(np.uint64), acc.view(np.uint64))
    ivals = [rng.integers(-5, 5, n).astype(np.int32) for _ in range(3)]
    iw = [((v.astype(np.int64) << 32) | k).astype(np.int64) for k, v in enumerate(ivals)]
    for op in (Operators.Long.INT_MAX_LOC, Operators.Long.INT_MIN_LOC):
        acc = iw[0].copy()
        for w in iw[1:]:
            op.reduce_into(acc, w)
        out = torch.empty(n, dtype=torch.int64, device=DEV)
        K.reduce_(out, [torch.from_numpy(w).to(DEV) for w in iw], int(op.code))
        assert np.array_equal(out.cpu().numpy(), acc)


def test_reduce_unaligned_views():
    K = _native()
    base = [torch.randn(5000, device=DEV) for _ in range(3)]
    xs = [b[1:4001] for b in base]            # 4-byte aligned, not 16-byte aligned
    out = torch.empty(4000, device=DEV)
    K.reduce_(out, xs, int(OpCode.SUM))
    torch.testing.assert_close(out, xs[0] + xs[1] + xs[2])


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("off", [0, 1])
def test_scale(dtype, off):
    """K1 scale: the 16-byte vector form (aligned, with a scalar tail) and the scalar form
    (misaligned view) against torch, in place too."""
    K = _native()
    x = torch.randn(12345 + off, device=DEV).to(dtype)[off:]
    y = torch.empty(12345 + off, device=DEV, dtype=dtype)[off:]
    K.scale_(y, x, 0.125)
    torch.testing.assert_close(y, (x.double() * 0.125).to(dtype), rtol=0, atol=0)
    z = x.clone()
    K.scale_(z, z, 0.125)
    assert torch.equal(z, y)


def test_segment_copy_and_gather_rows():
    K = _native()
    src = torch.arange(10_000, device=DEV, dtype=torch.float32)
    dst = torch.zeros(10_000, device=DEV)
    segs = [(0, 5000, 100), (100, 0, 3), (5000, 17, 4096), (9999, 1, 1)]
    K.segment_copy_(dst, src, segs)
    ref = torch.zeros(10_000, device=DEV)
    for d, s, l in segs:
        ref[d:d + l] = src[s:s + l]
    assert torch.equal(dst, ref)
    table = torch.randn(300, 40, device=DEV)
    idx = torch.randint(0, 300, (1000,), device=DEV)
    assert torch.equal(K.gather_rows(table, idx), table[idx])
    t3 = torch.randn(50, 7, device=DEV).to(torch.bfloat16)   # 14-byte rows: byte path
    i3 = torch.randint(0, 50, (77,), device=DEV)
    assert torch.equal(K.gather_rows(t3, i3), t3[i3])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fp8_codec_roundtrip_error(dtype):
    K = _native()
    n = 256 * 1000 + 4
    x = (torch.randn(n, device=DEV) * torch.linspace(0.01, 100, n, device=DEV)).to(dtype)
    q, s = K.quant_fp8(x)
    y = torch.empty(n, device=DEV, dtype=torch.float32)
    K.dequant_fp8(q, s, n, y)
    xf = x.float()
    # e4m3 has 3 mantissa bits: relative error <= 2^-4 of the block amax
    blk = torch.nn.functional.pad(xf.abs(), (0, (-n) % 256)).view(-1, 256).amax(1)
    bound = blk.repeat_interleave(256)[:n] * (2 ** -4) + 1e-30
    assert ((y - xf).abs() <= bound).all()


def test_fp8_dequant_reduce_requant():
    K = _native()
    n = 256 * 64
    xs = [torch.randn(n, device=DEV) for _ in range(5)]
    qs, ss = zip(*[K.quant_fp8(x) for x in xs])
    out = torch.empty(n, device=DEV)
    q2 = torch.empty(n, dtype=torch.uint8, device=DEV)
    s2 = torch.empty(n // 256, device=DEV)
    K.dequant_reduce_fp8(out, list(qs), list(ss), n, q_out=q2, s_out=s2)
    ref = sum(xs)
    assert (out - ref).abs().max() < 0.5   # 5 inputs x e4m3 error
    back = torch.empty(n, device=DEV)
    K.dequant_fp8(q2, s2, n, back)
    assert (back - out).abs().max() <= out.abs().max() * 2 ** -4 + 1e-6


@pytest.mark.parametrize("dim", [1, 8, 100])
def test_reduce_by_key_matches_torch(dim):
    K = _native()
    n = 20_000
    keys = torch.randint(0, 3000, (n,), device=DEV, dtype=torch.int64) * 7919
    vals = torch.randn(n, dim, device=DEV)
    uk, uv, cnt = K.reduce_by_key(keys, vals, int(OpCode.SUM))
    ref_k, inv = torch.unique(keys, sorted=True, return_inverse=True)
    ref_v = torch.zeros(ref_k.numel(), dim, device=DEV).index_add_(0, inv, vals)
    assert torch.equal(uk, ref_k)
    torch.testing.assert_close(uv, ref_v, rtol=1e-5, atol=1e-4)
    assert int(cnt.sum()) == n
    uk2, uv2, _ = K.reduce_by_key(keys, vals, int(OpCode.MAX))
    ref_m = torch.full((ref_k.numel(), dim), -float("inf"), device=DEV).scatter_reduce_(
        0, inv[:, None].expand(-1, dim), vals, "amax")
    torch.testing.assert_close(uv2, ref_m)


@pytest.mark.parametrize("bits", [12, 21])
def test_reduce_by_key_key_bits_matches_full_sort(bits):
    """Dense ids: sorting only the low ``bits`` bits gives the identical result."""
    K = _native()
    n = 50_000
    keys = torch.randint(0, 1 << bits, (n,), device=DEV, dtype=torch.int64)
    vals = torch.randn(n, 16, device=DEV)
    uk, uv, cnt = K.reduce_by_key(keys, vals, int(OpCode.SUM))
    uk2, uv2, cnt2 = K.reduce_by_key(keys, vals, int(OpCode.SUM), key_bits=bits)
    assert torch.equal(uk, uk2) and torch.equal(uv, uv2) and torch.equal(cnt, cnt2)


def test_key_owner_hist():
    K = _native()
    keys = torch.randint(0, 1 << 62, (50_000,), device=DEV, dtype=torch.int64)
    dest, hist = K.key_owner(keys, 7)
    assert torch.equal(dest.long(), keys % 7)
    assert torch.equal(hist.long(), torch.bincount(keys % 7, minlength=7))


def _owner_ref(keys, p):
    from mp4x.parallel.sparse import _owner
    return _owner(keys.cpu(), p).to(keys.device)


@pytest.mark.parametrize("p", [1, 3, 8, 1000])
@pytest.mark.parametrize("n", [0, 1, 255, 257, 70_001])
@pytest.mark.parametrize("dim,dtype", [(64, torch.float32), (3, torch.float32), (8, torch.bfloat16), (0, None)])
def test_partition_pack_is_stable_sort_by_owner(p, n, dim, dtype):
    """K4b fused LDS multisplit == stable argsort by (uint64)key % p (negative ids included)."""
    K = _native()
    g = torch.Generator(device="cpu").manual_seed(n * 31 + p)
    keys = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, dtype=torch.int64).to(DEV)
    vals = torch.randn(n, dim, generator=g).to(DEV, dtype) if dim else None
    sk, sv, counts, perm = K.partition_pack(keys, vals, p, want_perm=True)
    dest = _owner_ref(keys, p)
    ref = torch.argsort(dest, stable=True)
    assert torch.equal(perm, ref)
    assert torch.equal(sk, keys[ref])
    assert torch.equal(counts, torch.bincount(dest, minlength=p))
    if vals is not None:
        assert torch.equal(sv, vals[ref])
    else:
        assert sv is None


@pytest.mark.parametrize("n", [0, 1, 255, 257, 70_001])
def test_partition_pack_key_range(n):
    """want_range: counts[p:] = the smallest and largest key (0, 0 when empty), reduced inside
    the pack kernels (the count exchange carries it to size the reduce-by-key's sort)."""
    K = _native()
    g = torch.Generator(device="cpu").manual_seed(n + 5)
    for lo, hi in ((-(1 << 62), 1 << 62), (0, 1 << 24), (7, 8)):
        keys = torch.randint(lo, hi, (n,), generator=g, dtype=torch.int64).to(DEV)
        sk, _, counts, _ = K.partition_pack(keys, None, 8, want_range=True)
        assert counts.numel() == 10
        assert torch.equal(counts[:8], torch.bincount(_owner_ref(keys, 8), minlength=8))
        want = [int(keys.min()), int(keys.max())] if n else [0, 0]
        assert counts[8:].tolist() == want


def test_partition_pack_matches_sort_path():
    K = _native()
    keys = torch.randint(0, 1 << 62, (100_000,), device=DEV, dtype=torch.int64)
    vals = torch.randn(100_000, 16, device=DEV)
    dest, hist = K.key_owner(keys, 8)
    _, perm = K.sort_pairs(dest, end_bit=3)
    sk, sv, counts, _ = K.partition_pack(keys, vals, 8)
    assert torch.equal(sk, keys[perm]) and torch.equal(sv, vals[perm])
    assert torch.equal(counts, hist.long())


@pytest.mark.parametrize("dim,dtype", [(16, torch.float32), (5, torch.float32), (8, torch.int16), (3, torch.int8)])
def test_reduce_by_key_first_is_k8_dedupe(dim, dtype):
    """MP4X_FIRST: every key keeps the row of its first occurrence (K8 map merge)."""
    K = _native()
    n = 5000
    keys = torch.randint(0, 700, (n,), device=DEV, dtype=torch.int64)
    vals = torch.randint(-100, 100, (n, dim), device=DEV).to(dtype)
    uk, uv, cnt = K.reduce_by_key(keys, vals, 11)
    ref_k, inv = torch.unique(keys, sorted=True, return_inverse=True)
    first = torch.full((ref_k.numel(),), n, device=DEV, dtype=torch.int64)
    first.scatter_reduce_(0, inv, torch.arange(n, device=DEV), "amin")
    assert torch.equal(uk, ref_k) and torch.equal(uv, vals[first])
    assert int(cnt.sum()) == n


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16, torch.int8])
@pytest.mark.parametrize("density", [0.0, 0.03, 0.5, 1.0])
def test_zs_single_pass_encode_matches_three_kernel_form(dtype, density):
    """Single-pass encode (decoupled look-back) == mask + scan + compact, word for word, over
    several chunks (many tiles, so the look-back crosses 64-tile windows)."""
    K = _native()
    from mp4x.ops import native
    n = 3_000_000 + 77
    x = (torch.randn(n, device=DEV) * 10).to(dtype)
    x[torch.rand(n, device=DEV) >= density] = 0
    chunks = [(0, 1_000_003), (1_000_003, 999_000), (1_999_003, n - 1_999_003)]
    lib = native.hip()
    try:
        lib.mp4x_zs_set_twopass(1)
        ref = K.zs_encode(x, chunks)
        lib.mp4x_zs_set_twopass(0)
        got = K.zs_encode(x, chunks)
    finally:
        lib.mp4x_zs_set_twopass(1)       # back to the default
    for a, b in zip(ref[:3], got[:3]):
        assert torch.equal(a.view(torch.uint8) if a.dtype.is_floating_point else a,
                           b.view(torch.uint8) if b.dtype.is_floating_point else b)
    assert ref[3] == got[3] and ref[4] == got[4]
    out = torch.empty_like(x)
    K.zs_decode(got[0], got[1], got[2], chunks, out)
    assert torch.equal(out.view(torch.uint8), x.view(torch.uint8))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16, torch.int8])
def test_zs_codec_roundtrip_bits(dtype):
    """K6b: masks / counts / compacted words decode to the identical bit pattern (-0.0, NaN kept)."""
    K = _native()
    from mp4x.parallel import zs
    n = 10_000
    x = (torch.randn(n, device=DEV) * 10).to(dtype)
    x[torch.rand(n, device=DEV) < 0.8] = 0
    if dtype.is_floating_point:
        x[3] = -0.0
        x[4] = float("nan")
    chunks = [(0, 4000), (4000, 1), (4001, 0), (4001, n - 4001)]
    masks, counts, vals, nnz, bs = K.zs_encode(x, chunks)
    cm, cc, cv, cnnz, cbs = zs.encode(x.cpu(), chunks)            # CPU twin: identical format
    assert nnz == cnnz and bs == cbs
    assert torch.equal(masks.cpu(), cm) and torch.equal(counts.cpu(), cc)
    iv = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[x.element_size()]
    assert torch.equal(vals.cpu().view(iv), cv.view(iv))
    out = torch.full_like(x, 7)
    K.zs_decode(masks, counts, vals, chunks, out)
    assert torch.equal(out.view(iv), x.view(iv))


def test_device_map_pass_is_native_and_exact():
    """The device Map API's dict walk (csrc/pyext/map_ext.cpp) is loaded on the GPU box, finds
    the rows of a CUDA table, and the (ids, rows) it produces equal the per-key Python form."""
    import numpy as np
    from mp4x.ops import native
    from mp4x.parallel import sparse

    assert native.map_ext() is not None, "_mp4x_map not built/loaded"
    table = torch.randn(4096, 32, device=DEV)
    keys = [f"k{i}" for i in range(4096)]
    order = np.random.default_rng(0).permutation(4096)
    m = {keys[i]: table[i] for i in order}
    d = sparse.KeyDictionary()
    d.learn_round([keys[::2]])
    ids, nmiss, rows, base = sparse._pack_native(d, m)
    assert nmiss == 2048 and base is table
    assert np.array_equal(ids, d.lookup(list(m.keys())))
    got = base.reshape(-1, 32).index_select(0, torch.from_numpy(rows).to(DEV))
    assert torch.equal(got, torch.stack(list(m.values())))


def test_reduce_by_key_is_deterministic_in_input_order():
    """SURVEY §5.2 deterministic mode: the sort-based K5 reduce-by-key sums every key's rows in
    INPUT order (stable radix sort + sequential segment reduce), so repeated runs are bitwise
    equal and equal to a float64-free sequential reference in that order."""
    K = _native()
    n, dim = 50_000, 8
    g = torch.Generator(device=DEV).manual_seed(7)
    keys = torch.randint(0, 500, (n,), device=DEV, dtype=torch.int64, generator=g)
    vals = (torch.randn(n, dim, device=DEV, generator=g) * 1e3).float()
    runs = [K.reduce_by_key(keys, vals, int(OpCode.SUM)) for _ in range(3)]
    for uk, uv, _ in runs[1:]:
        assert torch.equal(uk, runs[0][0]) and torch.equal(uv, runs[0][1])
    # sequential f32 sums in input order for a few keys
    kc, vc = keys.cpu(), vals.cpu()
    for k in runs[0][0][:5].cpu().tolist():
        rows = vc[kc == k]
        acc = rows[0].clone()
        for r in rows[1:]:
            acc = acc + r
        j = int((runs[0][0].cpu() == k).nonzero()[0])
        assert torch.equal(runs[0][1][j].cpu(), acc), k


@pytest.mark.parametrize("n,bits", [(1, 8), (5000, 12), (300_000, 16), (600_000, 40), (200_000, 64)])
def test_sort_pairs_onesweep_matches_rocprim_dispatch(n, bits):
    """The forced-onesweep key sort (narrow keys, large counts) is the same stable sort as
    rocPRIM's own dispatch: identical keys and payload order, ties by input index."""
    K = _native()
    g = torch.Generator(device="cpu").manual_seed(n + bits)
    hi = (1 << bits) if bits < 63 else (1 << 62)
    keys = torch.randint(0, hi, (n,), generator=g, dtype=torch.int64).to(DEV)
    k0, i0 = K.sort_pairs(keys, end_bit=min(bits, 64), algo=0)
    k1, i1 = K.sort_pairs(keys, end_bit=min(bits, 64), algo=1)
    ref = torch.argsort(keys.cpu(), stable=True)
    assert torch.equal(i0.cpu(), ref) and torch.equal(i1.cpu(), ref)
    assert torch.equal(k0, k1)


@pytest.mark.parametrize("n,p,dim", [(0, 4, 16), (1, 3, 4), (70_001, 8, 64), (5000, 1000, 8)])
def test_partition_pack_halves_match_the_fused_pack(n, p, dim):
    """K4b split in two (count, then scatter anywhere — the sparse exchange scatters straight into
    its staging buffer): the same layout as partition_pack, keys at stride 1 or as the key half
    of 16-byte vectors, and the counts + key range of want_range."""
    K = _native()
    g = torch.Generator(device="cpu").manual_seed(n + p)
    keys = torch.randint(-(1 << 40), 1 << 40, (n,), generator=g, dtype=torch.int64).to(DEV)
    vals = torch.randn(n, dim, generator=g).to(DEV)
    sk, sv, counts, _ = K.partition_pack(keys, vals, p, want_range=True)
    pc = K.partition_count(keys, p)
    assert torch.equal(pc.info, counts)
    k1 = torch.empty_like(keys)
    v1 = torch.empty_like(vals)
    K.partition_scatter(pc, vals, v1.data_ptr(), k1.data_ptr())
    k2 = torch.zeros(n, 2, dtype=torch.int64, device=DEV)
    v2 = torch.empty_like(vals)
    K.partition_scatter(pc, vals, v2.data_ptr(), k2.data_ptr(), key_stride=2)
    torch.cuda.synchronize()
    assert torch.equal(k1, sk) and torch.equal(v1, sv)
    assert torch.equal(k2[:, 0], sk) and torch.equal(v2, sv) and not k2[:, 1].any()
