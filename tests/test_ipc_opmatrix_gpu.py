"""The whole operator table on the xGMI kernels (p processes sharing one GPU).

Every (dtype, op) pair of the reference's ``Operators`` (Operators.java:29-353: Double / Float /
Long / Int / Short / Byte, incl. PROD, BITS_AND / OR / XOR and the *_LOC packed words) plus the
16-bit floats, through the public ``allreduceArray`` on each IPC form — staged one-shot
(``ipc1``), staged two-shot (``ipc2``), zero-copy pull (``ipc2z``) and push (``ipc2w``) on a
registered tensor — and ``reduceScatterArray`` on the direct (staged) and zero-copy
reduce-scatter kernels.  Every result is compared bit for bit with a numpy fold in rank order
(``Operator.reduce_into``, the reference's argument order), and the engine's call counters show
that no call took the a2a detour (RCCL all-to-all + K1 + all-gather).  The default selection for
ops RCCL cannot reduce is checked too: small -> ``ipc1``, above the two-shot tier -> ``ipc2``
pieces (and ``reduce`` the same), never ``a2a``.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from spawn_ranks import run_spawn  # noqa: E402

pytestmark = pytest.mark.gpu

N = 16 * 6 * 217      # 20832: every rank's RS segment is a 16-byte multiple for p = 2, 3 and any dtype

# (Operators class, torch dtype, numpy dtype, op names) — the reference table + 16-bit floats
MATRIX = [
    ("Double", "float64", "float64", ("SUM", "MAX", "MIN", "PROD", "FLOAT_MAX_LOC", "FLOAT_MIN_LOC")),
    ("Float", "float32", "float32", ("SUM", "MAX", "MIN", "PROD")),
    ("Long", "int64", "int64", ("SUM", "MAX", "MIN", "BITS_AND", "BITS_OR", "BITS_XOR", "PROD", "INT_MAX_LOC",
                                "INT_MIN_LOC")),
    ("Int", "int32", "int32", ("SUM", "MAX", "MIN", "BITS_AND", "BITS_OR", "BITS_XOR", "PROD")),
    ("Short", "int16", "int16", ("SUM", "MAX", "MIN", "BITS_AND", "BITS_OR", "BITS_XOR", "PROD")),
    ("Byte", "int8", "int8", ("SUM", "MAX", "MIN", "BITS_AND", "BITS_OR", "BITS_XOR", "PROD")),
    ("BFloat16", "bfloat16", "float32", ("SUM", "MAX", "MIN", "PROD")),
    ("Half", "float16", "float32", ("SUM", "MAX", "MIN", "PROD")),
]


def _input(cls, op, np_dt, rank, n, salt):
    """This rank's exact-arithmetic input for (cls, op): small integers for floats (every sum /
    product exact in any order), the full range for integers (wrapping arithmetic is exact),
    packed (value, loc) words with frequent value ties for the *_LOC ops."""
    rng = np.random.default_rng(1000 * salt + rank)
    if op.endswith("_LOC"):
        vals = rng.integers(-2, 3, n)
        locs = rng.integers(0, 1 << 20, n).astype(np.uint64)
        if cls == "Double":
            hi = vals.astype(np.float32).view(np.uint32).astype(np.uint64)
        else:
            hi = vals.astype(np.int32).view(np.uint32).astype(np.uint64)
        return ((hi << np.uint64(32)) | locs).view(np.int64 if cls == "Long" else np.float64)
    if np_dt in ("float64", "float32"):
        if op == "PROD":
            return rng.choice(np.array([-2.0, -1.0, 0.5, 1.0, 2.0]), n).astype(np_dt)
        return rng.integers(-8, 9, n).astype(np_dt)
    info = np.iinfo(np_dt)
    return rng.integers(info.min, info.max, n, endpoint=True, dtype=np_dt)


def _expect(cls, op, np_dt, p, n, salt):
    from mp4x import Operators
    operator = getattr(getattr(Operators, cls), op)
    acc = _input(cls, op, np_dt, 0, n, salt).copy()
    with np.errstate(over="ignore", invalid="ignore"):
        for j in range(1, p):
            operator.reduce_into(acc, _input(cls, op, np_dt, j, n, salt))
    return acc


def _same(got, exp, dt_name):
    """Mismatch count, bitwise for integers / packed words, by value for floats."""
    g = got.cpu()
    if dt_name in ("bfloat16", "float16"):
        return int((g.float().numpy() != exp).sum())
    if dt_name in ("float64", "float32"):
        return int((g.numpy().view(np.uint8).reshape(len(exp), -1) !=
                    exp.view(np.uint8).reshape(len(exp), -1)).any(axis=1).sum())
    return int((g.numpy() != exp).sum())


def _opmatrix_fn(comm):
    from mp4x import CommUtils, Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    eng.ipc()
    assert eng.ipc_selftest and eng.ipc_selftest["ok"], eng.ipc_selftest
    reg = torch.zeros(N * 8, dtype=torch.uint8, device="cuda")
    assert comm.registerBuffer(reg)
    counts = [N // p] * p
    froms, tos = CommUtils.getFromsFromCount(0, counts, p), CommUtils.getTosFromCount(0, counts, p)
    bad, calls = {}, []
    salt = 0
    for cls, dt_name, np_dt, ops in MATRIX:
        dt = getattr(torch, dt_name)
        es = torch.empty((), dtype=dt).element_size()
        for op in ops:
            salt += 1
            operator = getattr(getattr(Operators, cls), op)
            x = torch.from_numpy(_input(cls, op, np_dt, r, N, salt)).to(dt).cuda()
            exp = _expect(cls, op, np_dt, p, N, salt)
            operand = Operands.DOUBLE_OPERAND()
            for algo in ("ipc1", "ipc2", "ipc2z", "ipc2w"):
                eng.algo = algo
                before = dict(eng.stats)
                v = reg[:N * es].view(dt) if algo in ("ipc2z", "ipc2w") else torch.empty(N, dtype=dt, device="cuda")
                v.copy_(x)
                comm.allreduceArray(v, operand, operator, 0, N)
                torch.cuda.synchronize()
                bad[f"{cls}.{op}.{algo}"] = _same(v, exp, dt_name)
                calls.append((f"{cls}.{op}.{algo}", {k: eng.stats.get(k, 0) - before.get(k, 0) for k in eng.stats
                                                     if eng.stats.get(k, 0) != before.get(k, 0)}))
            eng.algo = "auto"
            for zc in (False, True):
                before = dict(eng.stats)
                v = reg[:N * es].view(dt) if zc else torch.empty(N, dtype=dt, device="cuda")
                v.copy_(x)
                comm.reduceScatterArray(v, operand, operator, 0, counts)
                torch.cuda.synchronize()
                bad[f"{cls}.{op}.rs{'_zc' if zc else ''}"] = _same(v[froms[r]:tos[r]], exp[froms[r]:tos[r]], dt_name)
                calls.append((f"{cls}.{op}.rs{'_zc' if zc else ''}",
                              {k: eng.stats.get(k, 0) - before.get(k, 0) for k in eng.stats
                               if eng.stats.get(k, 0) != before.get(k, 0)}))
    comm.deregisterBuffer(reg)
    errw = [inst.error_word() for inst in eng._ipc_all()]
    return bad, calls, errw


@pytest.mark.parametrize("p", [2, 3])
def test_operator_matrix_on_every_ipc_form(p):
    out = run_spawn(p, _opmatrix_fn, timeout=240)
    for r, (bad, calls, errw) in out.items():
        wrong = {k: v for k, v in bad.items() if v}
        assert not wrong, (r, wrong)
        assert errw and not any(errw), errw
        for name, d in calls:
            kind = name.rsplit(".", 1)[1]
            assert not any("a2a" in k for k in d), (name, d)
            want = {"ipc1": "allreduce.ipc1", "ipc2": "allreduce.ipc2", "ipc2z": "allreduce.ipc2z",
                    "ipc2w": "allreduce.ipc2w", "rs": "reduce_scatter.ipc", "rs_zc": "reduce_scatter.ipc_zc"}[kind]
            assert d.get(want) == 1, (name, d)


def _default_select_fn(comm):
    """Ops RCCL cannot reduce, at the default (auto) selection: no a2a at any size."""
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    out = {}
    cases = [("Long", "BITS_OR", torch.int64, 4096), ("Short", "SUM", torch.int16, 4096),
             ("Int", "BITS_XOR", torch.int32, (24 << 20) // 4), ("Double", "FLOAT_MAX_LOC", torch.float64, 1 << 16),
             ("Byte", "BITS_AND", torch.int8, 24 << 20)]
    for cls, op, dt, n in cases:
        operator = getattr(getattr(Operators, cls), op)
        g = torch.Generator(device="cuda").manual_seed(7 + r)
        x = torch.randint(-100, 100, (n,), device="cuda", generator=g).to(dt)
        xs = [torch.randint(-100, 100, (n,), device="cuda", generator=torch.Generator(device="cuda").manual_seed(7 + j))
              .to(dt) for j in range(p)]
        exp = xs[0].cpu().numpy().copy()
        for j in range(1, p):
            with np.errstate(over="ignore"):
                operator.reduce_into(exp, xs[j].cpu().numpy())
        before = dict(eng.stats)
        y = x.clone()
        comm.allreduceArray(y, Operands.LONG_OPERAND(), operator, 0, n)
        z = x.clone()
        comm.reduceArray(z, Operands.LONG_OPERAND(), operator, 0, n, p - 1)
        torch.cuda.synchronize()
        d = {k: eng.stats.get(k, 0) - before.get(k, 0) for k in eng.stats if eng.stats.get(k, 0) != before.get(k, 0)}
        ok_ar = bool((y.cpu().numpy().view(np.uint8) == exp.view(np.uint8)).all())
        ok_red = r != p - 1 or bool((z.cpu().numpy().view(np.uint8) == exp.view(np.uint8)).all())
        out[f"{cls}.{op}.{n}"] = (ok_ar, ok_red, d)
    return out


def test_default_selection_never_takes_a2a_for_builtin_ops():
    out = run_spawn(2, _default_select_fn, timeout=240)
    for r, res in out.items():
        for name, (ok_ar, ok_red, d) in res.items():
            assert ok_ar and ok_red, (r, name, d)
            assert not any("a2a" in k for k in d), (r, name, d)
            assert any(k.startswith("allreduce.ipc") for k in d) and any(k.startswith("reduce.ipc") for k in d), \
                (r, name, d)
