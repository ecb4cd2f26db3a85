"""Real multi-GPU validation: rank r on cuda:r, RCCL (nccl backend) underneath — skipped on a box
with fewer GPUs than ranks, so the 1-GPU suite is unchanged and any multi-GPU lease validates
the cross-device paths with no edits:

* RCCL allreduce and reduce-scatter at p = 2 / 4 / 8 through the public API (exact pattern);
* the collective IPC self-test over real xGMI mappings;
* the zero-copy two-shot, pull AND push forms, twice in a row on the same registered tensor
  (the second call reads the first call's results on the peers: a stale L2 line from the cross-
  GPU coherence protocol would show here — the probe a shared GPU can never fail);
* the fused fp8 two-shot against the fp64 sum (e4m3 error bound);
* memAlloc above 2 GiB across GPUs, exact;
* the node-aware allreduce with simulated nodes of real GPUs (IPC sub-meshes + RCCL
  sub-communicators);
* the zero-copy reduce / broadcast / gather / scatter on memAlloc tensors across GPUs.

Dry run before first contact (``MP4X_TEST_MULTI_DRYRUN=1``, tests/spawn_ranks.py): the same tests
with every rank on cuda:0 and gloo standing in for RCCL.  Every exact-value check runs; skipped
are only the checks that need real RCCL or distinct device ordinals (the backend / ordinal
assertion, the dedicated-channel RCCL communicators, the RCCL abort).  Without the knob the module
skips on a box with fewer GPUs than ranks.
"""
import time

import pytest

torch = pytest.importorskip("torch")

from spawn_ranks import multi_dryrun, run_spawn  # noqa: E402

pytestmark = pytest.mark.gpu
DRY = multi_dryrun()       # (also true in the spawned ranks: they inherit the environment)
RCCL_ONLY = ("rccl_c64", "rccl_c112")     # dedicated-channel RCCL communicators: no gloo form


def _ngpu():
    try:
        return torch.cuda.device_count()
    except Exception:   # noqa: BLE001
        return 0


def _need(p):
    if DRY:
        return
    if _ngpu() < p:
        pytest.skip(f"needs {p} GPUs (box has {_ngpu()})")


def _pattern(n, r):
    return (torch.arange(n, device="cuda", dtype=torch.int32) % 13 + r).float()


def _expect(n, p):
    i = torch.arange(n, device="cuda", dtype=torch.int32) % 13
    return (i * p + p * (p - 1) // 2).float()


def _rccl_fn(comm):
    from mp4x import CommUtils, Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    assert DRY or (eng.backend == "nccl" and eng.device.index == r), (eng.backend, eng.device)
    n = (48 << 20) // 4
    x = _pattern(n, r)
    comm.allreduceArray(x, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, n)
    ok_ar = bool(torch.equal(x, _expect(n, p)))
    counts = [n // p] * p
    counts[-1] += n - sum(counts)
    y = _pattern(n, r)
    comm.reduceScatterArray(y, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, counts)
    f = CommUtils.getFromsFromCount(0, counts, p)
    t = CommUtils.getTosFromCount(0, counts, p)
    ok_rs = bool(torch.equal(y[f[r]:t[r]], _expect(n, p)[f[r]:t[r]]))
    torch.cuda.synchronize()
    return ok_ar, ok_rs, dict(eng.stats)


@pytest.mark.parametrize("p", [2, 4, 8])
def test_rccl_allreduce_reduce_scatter(p):
    _need(p)
    out = run_spawn(p, _rccl_fn, mode="multi", env={"MP4X_DEVICE_ALGO": "rccl"})
    for r, (ok_ar, ok_rs, stats) in out.items():
        assert ok_ar and ok_rs, (r, stats)
        assert stats.get("allreduce.rccl", 0) >= 1, stats


def _ipc_fn(comm):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    eng.ipc()
    st = eng.ipc_selftest
    res = {"selftest": st}
    n = (24 << 20) // 4
    buf = torch.empty(n, device="cuda")
    res["registered"] = comm.registerBuffer(buf)
    for algo in ("ipc2z", "ipc2w", "ipc1", "ipc2"):
        eng.algo = algo
        m = n if algo != "ipc1" else (64 << 10) // 4
        v = buf[:m]
        v.copy_(_pattern(m, r))
        bad = []
        for k in range(2):          # 2nd call reduces the 1st call's result: stale-line probe
            comm.allreduceArray(buf, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, m)
            torch.cuda.synchronize()
            bad.append(int((v != _expect(m, p) * (p ** k)).sum()))
        res[algo] = bad
    eng.algo = "auto"
    comm.deregisterBuffer(buf)
    res["stats"] = dict(eng.stats)
    return res


@pytest.mark.parametrize("p", [2, 4, 8])
def test_ipc_selftest_and_zero_copy_cross_gpu(p):
    _need(p)
    out = run_spawn(p, _ipc_fn, mode="multi")
    for r, res in out.items():
        assert res["selftest"] is not None and res["selftest"]["ok"], (r, res["selftest"])
        assert res["registered"], r
        for algo in ("ipc2z", "ipc2w", "ipc1", "ipc2"):
            assert res[algo] == [0, 0], (r, algo, res[algo])
        assert res["stats"].get("allreduce.ipc2z", 0) >= 2, res["stats"]


def _fp8_fn(comm):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    n = (16 << 20) // 4
    g = torch.Generator(device="cuda").manual_seed(100 + r)
    x = torch.randn(n, device="cuda", generator=g)
    ref = torch.zeros(n, dtype=torch.float64, device="cuda")
    mag = torch.zeros(n, dtype=torch.float64, device="cuda")
    for j in range(p):
        gj = torch.Generator(device="cuda").manual_seed(100 + j)
        xj = torch.randn(n, device="cuda", generator=gj).double()
        ref += xj
        mag += xj.abs()
    comm.allreduceArray(x, Operands.FLOAT_OPERAND(codec="fp8"), Operators.Float.SUM, 0, n)
    torch.cuda.synchronize()
    err = (x.double() - ref).abs()
    # two e4m3 roundings (3 mantissa bits: relative error <= 2^-4 each) of block-scaled values:
    # every input once, the reduced chunk once; 2x margin
    bound = (mag + ref.abs()) / 8 + 1e-3
    return int((err > bound).sum()), float(err.max()), dict(comm.device.stats)


@pytest.mark.parametrize("p", [2, 8])
def test_fp8_twoshot_cross_gpu(p):
    _need(p)
    out = run_spawn(p, _fp8_fn, mode="multi")
    for r, (nbad, emax, stats) in out.items():
        assert nbad == 0, (r, nbad, emax)
        assert stats.get("allreduce.fp8", 0) >= 1, stats


def _memalloc_fn(comm, n):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    t = comm.memAlloc(n, torch.float32)
    t.copy_(_pattern(n, r))
    bad = []
    for k in range(2):
        comm.allreduceArray(t, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, n)
        torch.cuda.synchronize()
        bad.append(int((t != _expect(n, p) * (p ** k)).sum()))
    comm.memFree(t)
    return bad, dict(comm.device.stats)


@pytest.mark.parametrize("p", [2, 8])
def test_memalloc_above_2gib_cross_gpu(p):
    _need(p)
    n = (2 << 30) // 4 + (1 << 20)
    out = run_spawn(p, _memalloc_fn, args=(n,), mode="multi", timeout=300)
    for r, (bad, stats) in out.items():
        assert bad == [0, 0], (r, bad)


def _hier_fn(comm):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    h = eng.hier()
    n = (24 << 20) // 4 + 1024
    x = _pattern(n, r)
    comm.allreduceArray(x, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, n)
    torch.cuda.synchronize()
    return bool(torch.equal(x, _expect(n, p))), h is not None and h.ipc is not None, h.selftest, \
        eng.stats.get("allreduce.hier", 0)


@pytest.mark.parametrize("p,node", [(4, 2), (8, 4)])
def test_hier_allreduce_cross_gpu(p, node):
    """Node-aware allreduce with simulated nodes of real GPUs: IPC sub-meshes over xGMI inside
    each "node", RCCL sub-communicators across them, 8 MiB pipelined pieces."""
    _need(p)
    res = run_spawn(p, _hier_fn, timeout=240, mode="multi",
                    env={"MP4X_SIM_NODE_SIZE": str(node), "MP4X_HIER_PIECE_BYTES": str(8 << 20), "MP4X_HIER": "1"})
    for r, (ok, has_ipc, st, calls) in res.items():
        assert ok and has_ipc and st["ok"] and calls == 1, (r, ok, has_ipc, st, calls)


def _zc_rooted_cross_fn(comm):
    from mp4x import CommUtils, Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    F = Operands.FLOAT_OPERAND()
    n = (96 << 20) // 4
    x = comm.memAlloc(n, torch.float32)
    root = p - 1
    x.copy_(_pattern(n, r))
    comm.reduceArray(x, F, Operators.Float.SUM, 0, n, root)
    ok = [r != root or bool(torch.equal(x, _expect(n, p)))]
    base = torch.arange(n, device="cuda", dtype=torch.int32).remainder_(11).float()
    x.copy_(base if r == root else torch.zeros_like(base))
    comm.broadcastArray(x, F, 0, n, root)
    ok.append(bool(torch.equal(x, base)))
    counts = [n // p] * p
    counts[-1] += n - sum(counts)
    fr, to = CommUtils.getFromsFromCount(0, counts, p), CommUtils.getTosFromCount(0, counts, p)
    x.fill_(-1.0)
    x[fr[r]:to[r]] = r + 1.0
    comm.gatherArray(x, F, fr, to, root)
    ok.append(r != root or all(bool((x[fr[j]:to[j]] == j + 1).all()) for j in range(p)))
    x.fill_(-1.0)
    if r == root:
        for j in range(p):
            x[fr[j]:to[j]] = 10.0 + j
    comm.scatterArray(x, F, fr, to, root)
    ok.append(bool((x[fr[r]:to[r]] == 10.0 + r).all()))
    torch.cuda.synchronize()
    st = {k: v for k, v in comm.device.stats.items() if k.endswith("ipc_zc")}
    comm.memFree(x)
    return ok, st


@pytest.mark.parametrize("p", [2, 8])
def test_zero_copy_rooted_cross_gpu(p):
    """reduce / broadcast / gather / scatter on a memAlloc tensor across real GPUs: one zero-copy
    kernel each, pulling over xGMI from the peers' tensors."""
    _need(p)
    res = run_spawn(p, _zc_rooted_cross_fn, timeout=240, mode="multi")
    for r, (ok, st) in res.items():
        assert all(ok), (r, ok)
        assert all(st.get(f"{k}.ipc_zc") == 1 for k in ("reduce", "broadcast", "gather", "scatter")), st


# ====================================================================== every schedule, RCCL underneath
# The engine's schedule names (allreduce_candidates, _CAPTURABLE, the rooted / RS / AG tuners' and
# the codec schedules) each ran by at least one test below, one GPU per rank, RCCL for real.
# tests/test_multigpu_coverage.py checks on CPU that this table names every schedule the engine has.
COVERS = {
    "test_forced_allreduce_schedules_cross_gpu": [
        "allreduce:rccl", "allreduce:rccl_c64", "allreduce:rccl_c112", "allreduce:ipc1", "allreduce:ipc2",
        "allreduce:ipc2p", "allreduce:ipc2z", "allreduce:ipc2w", "allreduce:ipc2z_b64", "allreduce:ipc2z_b128",
        "allreduce:a2a", "allreduce:rhd", "allreduce:zs", "allreduce:fp8", "allreduce:bf16"],
    "test_autotuners_with_rccl_candidates_cross_gpu": [
        "reduce_scatter:rccl", "reduce_scatter:a2a", "reduce_scatter:ipc", "allgather:rccl", "allgather:p2p",
        "allgather:ipc", "reduce:rccl", "reduce:a2a", "reduce:ipc", "broadcast:rccl", "broadcast:composite",
        "broadcast:ipc", "gather:p2p", "gather:ipc", "scatter:p2p", "scatter:ipc"],
    "test_hier_allreduce_cross_gpu": ["allreduce:hier"],
}


def _forced_fn(comm):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    n = (80 << 20) // 4                  # above the 32 MiB large buffer below: ipc2p runs pieces
    buf = torch.empty(n, device="cuda")
    assert comm.registerBuffer(buf)
    plain = torch.empty(n, device="cuda")
    F, SUM = Operands.FLOAT_OPERAND(), Operators.Float.SUM
    res = {}
    for algo in COVERS["test_forced_allreduce_schedules_cross_gpu"]:
        name = algo.split(":")[1]
        if DRY and name in RCCL_ONLY:
            continue
        operand, forced, m = F, name, n
        if name in ("zs", "fp8", "bf16"):
            operand = Operands.FLOAT_OPERAND(compress=True) if name == "zs" else Operands.FLOAT_OPERAND(codec=name)
            forced = "auto"
        if name == "ipc1":
            m = (256 << 10) // 4
        eng.algo = forced
        v = (buf if name.startswith("ipc2z") or name == "ipc2w" else plain)[:m]
        before = dict(eng.stats)
        bad = []
        for k in range(2):           # the second call reduces the first call's result
            if k == 0:
                v.copy_(_pattern(m, r))
            comm.allreduceArray(v, operand, SUM, 0, m)
            torch.cuda.synchronize()
            exp = _expect(m, p) * (p ** k)
            if name == "fp8":        # lossy codec: two e4m3 roundings, 2^-4 relative each
                bad.append(int(((v - exp).abs() > exp.abs() / 8 + 1e-3).sum()))
            else:
                bad.append(int((v != exp).sum()))
            if name == "fp8":
                v.copy_(exp)
        used = {x: c - before.get(x, 0) for x, c in eng.stats.items() if c != before.get(x, 0)}
        res[name] = (bad, used)
    eng.algo = "auto"
    comm.deregisterBuffer(buf)
    return res


@pytest.mark.parametrize("p", [2, 8])
def test_forced_allreduce_schedules_cross_gpu(p):
    """Every allreduce schedule forced in turn on real GPUs, exact twice in a row (fp8 within its
    codec bound): RCCL and its 64 / 112-channel communicators, the staged / pipelined / zero-copy
    pull / push / fixed-grid IPC forms, a2a and rhd over RCCL, and the zs / fp8 / bf16 codecs."""
    _need(p)
    out = run_spawn(p, _forced_fn, mode="multi", timeout=300, env={"MP4X_IPC_LARGE_BYTES": str(32 << 20)})
    for r, res in out.items():
        for name, (bad, used) in res.items():
            assert bad == [0, 0], (r, name, bad, used)
            key = "allreduce.fp8" if name == "fp8" else f"allreduce.{name}"
            assert used.get(key, 0) == 2, (r, name, used)


def _tuners_fn(comm):
    from mp4x import Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    out = {}
    for nb in (1 << 20, 64 << 20):
        like = torch.empty(nb // 4, device="cuda")
        out[f"allreduce:{nb}"] = eng.autotune_allreduce(like, Operators.Float.SUM, iters=2)
        out[f"reduce_scatter:{nb}"] = eng.autotune_reduce_scatter(like, Operators.Float.SUM, iters=2)
        out[f"allgather:{nb}"] = eng.autotune_allgather(like, iters=2)
        out[f"reduce:{nb}"] = eng.autotune_reduce(like, Operators.Float.SUM, root=p - 1, iters=2)
        out[f"broadcast:{nb}"] = eng.autotune_broadcast(like, root=p - 1, iters=2)
        out[f"gather:{nb}"] = eng.autotune_gather(like, root=p - 1, iters=2)
        out[f"scatter:{nb}"] = eng.autotune_scatter(like, root=p - 1, iters=2)
    return out, eng.ipc_selftest


@pytest.mark.parametrize("p", [2, 8])
def test_autotuners_with_rccl_candidates_cross_gpu(p):
    """Every tuner on real GPUs with RCCL among the candidates: each candidate's warm-up call is an
    exact probe, run twice (the second on the first's result), so a finite time means that
    schedule was exact on every rank; inf would mean wrong / failed / timed out somewhere.  The
    opt-in schedules join (MP4X_AUTOTUNE_EXTRA=1: RCCL with pinned channel counts, the composite
    broadcast, ...) so every schedule the tuners know is probed here."""
    _need(p)
    # (dry run: gloo stands in for RCCL, and the tuners keep its candidates only when asked)
    env = {"MP4X_AUTOTUNE_EXTRA": "1", **({"MP4X_AUTOTUNE_GLOO": "1"} if DRY else {})}
    out = run_spawn(p, _tuners_fn, mode="multi", timeout=600, env=env)
    want = {k.split(":")[0]: set() for ks in COVERS.values() for k in ks}
    for ks in COVERS["test_autotuners_with_rccl_candidates_cross_gpu"]:
        kind, algo = ks.split(":")
        want[kind].add(algo)
    for r, (res, st) in out.items():
        assert st is not None and st["ok"], (r, st)
        for key, times in res.items():
            kind = key.split(":")[0]
            assert all(t != float("inf") for t in times.values()), (r, key, times)
            if kind != "allreduce":
                assert want[kind] <= set(times), (key, sorted(times))
        big = res[f"allreduce:{64 << 20}"]
        want_big = {"rccl", "ipc2z", "ipc2w", "a2a"} | (set() if DRY else set(RCCL_ONLY))
        assert want_big <= set(big), sorted(big)


def _train_fn(comm):
    from mp4x.models.mlp import train_dp, train_single
    from mp4x.models.zero import train_single_adamw, train_zero
    dp = train_dp(comm, steps=6, global_batch=64, device="cuda", bucket_mb=0.01)
    z = train_zero(comm, steps=6, global_batch=64, device="cuda")
    ref_dp = train_single(steps=6, global_batch=64, device="cuda")
    ref_z = train_single_adamw(steps=6, global_batch=64, device="cuda")
    st = {k: v for k, v in comm.device.stats.items()}
    return dp, ref_dp, z, ref_z, st


@pytest.mark.parametrize("p", [2, 8])
def test_ddp_and_zero_match_single_gpu_training(p):
    """SURVEY §7.4 acceptance across real GPUs: data-parallel SGD (bucketed gradient allreduce on
    a memAlloc arena) and ZeRO-2 AdamW (reduce-scatter + all-gather) follow the single-GPU loss
    trajectory on the full batch."""
    import numpy as np
    _need(p)
    out = run_spawn(p, _train_fn, mode="multi", timeout=300)
    for r, (dp, ref_dp, z, ref_z, st) in out.items():
        np.testing.assert_allclose(dp, ref_dp, rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(z, ref_z, rtol=1e-3, atol=1e-5)
        assert st.get("reduce_scatter.ipc_zc", 0) >= 6 and st.get("allgather.ipc_zc", 0) >= 6, st


def _graph_fn(comm):
    from mp4x import Operands, Operators
    from mp4x.ops.device_ops import scale_
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    small = torch.zeros(16 << 10, device="cuda")
    mid = torch.zeros(2 << 20, device="cuda")
    reg = torch.zeros(4 << 20, device="cuda")
    assert comm.registerBuffer(reg)
    F = Operands.FLOAT_OPERAND()

    def step():
        eng.allreduce(small, 0, small.numel(), Operators.Float.SUM)            # ipc1
        eng.allreduce(mid, 0, mid.numel(), Operators.Float.SUM)                # ipc2
        eng.allreduce(reg, 0, reg.numel(), Operators.Float.SUM)                # ipc2z (registered)
        scale_(mid, mid, 0.5)

    g = eng.capture(step)
    bad = 0
    for i in range(4):
        for t in (small, mid, reg):
            t.copy_(_pattern(t.numel(), r) + i)
        g.replay()
        torch.cuda.synchronize()
        bad += int((small != _expect(small.numel(), p) + i * p).sum())
        bad += int((mid != (_expect(mid.numel(), p) + i * p) * 0.5).sum())
        bad += int((reg != _expect(reg.numel(), p) + i * p).sum())
    eager = _pattern(small.numel(), r)                  # eager calls interleave with the replays
    comm.allreduceArray(eager, F, Operators.Float.SUM, 0, eager.numel())
    torch.cuda.synchronize()
    bad += int((eager != _expect(eager.numel(), p)).sum())
    comm.deregisterBuffer(reg)
    return bad, dict(eng.stats)


@pytest.mark.parametrize("p", [2, 8])
def test_hipgraph_capture_with_device_epochs_cross_gpu(p):
    _need(p)
    out = run_spawn(p, _graph_fn, mode="multi", timeout=240)
    for r, (bad, st) in out.items():
        assert bad == 0, (r, st)
        assert st.get("allreduce.ipc2z", 0) >= 1 and st.get("allreduce.ipc1", 0) >= 1, st


def _thread_fn(comm):
    import threading
    from mp4x import Operands, Operators
    r, p, T = comm.getRank(), comm.getSlaveNum(), comm.getThreadNum()
    n = (8 << 20) // 4 + 4
    res = [None] * T
    errs = []

    def body(t):
        try:
            torch.cuda.set_device(0 if DRY else r)       # (the dry run puts every rank on cuda:0)
            comm.setThreadId(t)
            x = _pattern(n, r * T + t)
            comm.allreduceArray(x, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, n)
            torch.cuda.synchronize()
            res[t] = int((x != _expect(n, p * T)).sum())
        except BaseException:   # noqa: BLE001
            import traceback
            errs.append(traceback.format_exc())

    ths = [threading.Thread(target=body, args=(t,)) for t in range(T)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return res, errs


@pytest.mark.parametrize("p,T", [(2, 2), (8, 2)])
def test_thread_comm_per_rank_gpu(p, T):
    """ThreadCommSlave with T host threads per rank, each rank on its own GPU: K1 thread phase +
    the device engine's process phase over RCCL / xGMI."""
    _need(p)
    out = run_spawn(p, _thread_fn, mode="multi", threads=T, timeout=240)
    for r, (res, errs) in out.items():
        assert not errs, errs[0]
        assert res == [0] * T, (r, res)


def _rsag_zc_fn(comm):
    from mp4x import CommUtils, Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    n = (256 << 20) // 2
    x = comm.memAlloc(n, torch.bfloat16)
    counts = [n // p] * p
    counts[-1] += n - sum(counts)
    fr, to = CommUtils.getFromsFromCount(0, counts, p), CommUtils.getTosFromCount(0, counts, p)
    ok = []
    for rep in range(2):
        x.copy_(_pattern(n, r).to(torch.bfloat16))
        comm.reduceScatterArray(x, Operands.FLOAT_OPERAND(), Operators.BFloat16.SUM, 0, counts)
        exp = _expect(n, p).to(torch.bfloat16)
        torch.cuda.synchronize()
        ok.append(bool(torch.equal(x[fr[r]:to[r]], exp[fr[r]:to[r]])))
        comm.allgatherArray(x, Operands.FLOAT_OPERAND(), fr, to)
        torch.cuda.synchronize()
        ok.append(bool(torch.equal(x, exp)))
    st = dict(comm.device.stats)
    comm.memFree(x)
    return ok, st


@pytest.mark.parametrize("p", [2, 8])
def test_zero_copy_rs_ag_halves_on_memalloc_cross_gpu(p):
    """BASELINE config 3's shape (bf16 RS + AG, ZeRO partition) on a memAlloc tensor across GPUs:
    the zero-copy reduce-scatter and all-gather kernels, twice on the same memory."""
    _need(p)
    out = run_spawn(p, _rsag_zc_fn, mode="multi", timeout=240)
    for r, (ok, st) in out.items():
        assert all(ok), (r, ok)
        assert st.get("reduce_scatter.ipc_zc") == 2 and st.get("allgather.ipc_zc") == 2, st


def _map_fn(comm):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    dim = 64
    g = torch.Generator().manual_seed(300 + r)
    keys = [f"f{int(k)}" for k in torch.randperm(30000, generator=g)[:20000]]
    rows = torch.randint(-8, 8, (len(keys), dim), generator=g).float().cuda()
    mp = {k: rows[i] for i, k in enumerate(keys)}
    before = dict(comm.device.stats)
    res = comm.allreduceMap(mp, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
    torch.cuda.synchronize()
    used = {x: c - before.get(x, 0) for x, c in comm.device.stats.items() if c != before.get(x, 0)}
    out = {k: v.cpu().numpy() for k, v in res.items()}
    return out, used


@pytest.mark.parametrize("p", [2, 8])
def test_sparse_map_allreduce_over_ipc_cross_gpu(p):
    """BASELINE config 4's shape (Map<String, float[64]> allreduceMap) across GPUs: the ragged
    key/row exchanges run as IPC copy plans over xGMI; exact against the host sum."""
    import numpy as np
    _need(p)
    out = run_spawn(p, _map_fn, mode="multi", timeout=300)
    ref = {}
    for j in range(p):
        g = torch.Generator().manual_seed(300 + j)
        keys = [f"f{int(k)}" for k in torch.randperm(30000, generator=g)[:20000]]
        rows = torch.randint(-8, 8, (len(keys), 64), generator=g).float().numpy()
        for i, k in enumerate(keys):
            ref[k] = ref[k] + rows[i] if k in ref else rows[i].copy()
    for r, (res, used) in out.items():
        assert set(res) == set(ref), r
        assert all(np.array_equal(res[k], ref[k]) for k in ref), r
        assert used.get("sparse.a2a.ipc", 0) >= 1, used


def _abort_fn(comm):
    from mp4x import Operands, Operators
    from mp4x.exceptions import Mp4jException
    r = comm.getRank()
    eng = comm.device
    assert eng.watchdog is not None and eng.watchdog.action == "abort"
    x = torch.ones(16 << 20, device="cuda")
    if r == 0:
        comm.allreduceArray(x, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, x.numel())   # rank 1 never joins
        t0 = time.time()
        while eng.watchdog.failure is None and time.time() - t0 < 30:
            time.sleep(0.2)
        err = None
        try:
            comm.allreduceArray(x, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, x.numel())
        except Mp4jException as e:
            err = str(e)
        return eng.watchdog.failure, err
    time.sleep(12)
    return None, None


def test_watchdog_abort_action_with_rccl():
    """MP4X_WATCHDOG_ACTION=abort on real GPUs: a rank whose RCCL allreduce never completes (its
    peer never joins) is detected on the device (pending event), the communicators are aborted
    (ncclCommAbort) and the next collective raises instead of hanging."""
    if DRY:
        pytest.skip("needs a real RCCL communicator to abort (dry run: gloo)")
    _need(2)
    env = {"MP4X_WATCHDOG": "1", "MP4X_WATCHDOG_ACTION": "abort", "MP4X_WATCHDOG_TIMEOUT": "3",
           "MP4X_WATCHDOG_PERIOD": "0.2", "MP4X_DEVICE_ALGO": "rccl"}
    out = run_spawn(2, _abort_fn, mode="multi", timeout=120, env=env)
    failure, err = out[0]
    assert failure and "not complete on the device" in failure, failure
    assert err and "watchdog" in err, err
