"""The allreduceArray latency fast path (VERDICT r4 Next #5): a repeated small device allreduce
goes from the public API's first lines to ONE native call (mp4x_ipc_fast_allreduce: error words,
capture check, epoch, launch) — exact every call, counted like the full path, invalidated when
anything that decided it changes, and failing loudly when an earlier collective timed out.
Two ranks share GPU 0 (the IPC kernels run for real)."""
import pytest

torch = pytest.importorskip("torch")

from spawn_ranks import run_spawn  # noqa: E402

pytestmark = pytest.mark.gpu


def _pat(n, r, k):
    return ((torch.arange(n, device="cuda", dtype=torch.int32) + k) % 13 + r).float()


def _exp(n, p, k):
    i = (torch.arange(n, device="cuda", dtype=torch.int32) + k) % 13
    return (i * p + p * (p - 1) // 2).float()


def _fast_fn(comm):
    import ctypes
    from mp4x import Operands, Operators
    from mp4x.exceptions import Mp4jException
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    eng.ipc()
    F, SUM = Operands.FLOAT_OPERAND(), Operators.Float.SUM
    out = {}
    for n, tag in ((1024, "4KiB"), ((1 << 20) // 4, "1MiB")):
        x = torch.empty(n, device="cuda")
        bad = 0
        for k in range(40):
            x.copy_(_pat(n, r, k))
            comm.allreduceArray(x, Operands.FLOAT_OPERAND(), SUM, 0, n)   # a fresh operand object each call
            torch.cuda.synchronize()
            bad += int((x != _exp(n, p, k)).sum())
        out[tag] = {"bad": bad, "memo": len(eng._fast_ar)}
        # fused scale through the fast path (the DP average)
        x.copy_(_pat(n, r, 3))
        for _ in range(3):
            comm.allreduceArray(x, F, SUM, 0, n, scale=1.0 / p)
        torch.cuda.synchronize()
        out[tag]["scale_bad"] = int((x != _exp(n, p, 3) / p).sum())
    calls = comm.stats["calls"].get("allreduceArray", 0)
    eng_calls = sum(v for k, v in eng.stats.items() if k in ("allreduce.ipc1", "allreduce.ipc2"))
    # one memo entry serves every tensor of the shape (nothing registered): fresh buffers at other
    # addresses launch natively; an unaligned one is refused natively before its epoch moves and
    # the full path runs it (exact)
    launched = []
    orig = comm._fast_lx

    def spy(*a):
        rc = orig(*a)
        launched.append(rc)
        return rc
    comm._fast_lx = spy
    n = 1024
    pool = [torch.empty(n, device="cuda") for _ in range(3)]
    big = torch.empty(n + 1, device="cuda")
    fresh_bad = 0
    for k in range(12):
        x = big[1:] if k % 4 == 3 else pool[k % 3]
        x.copy_(_pat(n, r, k))
        comm.allreduceArray(x, F, SUM, 0, n)
        torch.cuda.synchronize()
        fresh_bad += int((x != _exp(n, p, k)).sum())
    fresh = {"bad": fresh_bad, "launched": launched.count(0), "refused": len(launched) - launched.count(0),
             "addrs": len({t.data_ptr() for t in pool}), "by_ptr": eng._fast_ar.by_ptr}
    # with a registered tensor the memo keys on the address: the registered one runs zero-copy
    y = torch.empty(1 << 21, device="cuda")      # 8 MiB: the two-shot tier, zero-copy when registered
    comm.registerBuffer(y)
    keyed = eng._fast_ar.by_ptr
    zc_before = sum(v for k, v in eng.stats.items() if k.endswith("ipc2z") or k.endswith("ipc_zc"))
    reg_bad = 0
    for k in range(4):
        for t in (y, pool[0]):
            t.copy_(_pat(t.numel(), r, k))
            comm.allreduceArray(t, F, SUM, 0, t.numel())
            torch.cuda.synchronize()
            reg_bad += int((t != _exp(t.numel(), p, k)).sum())
    zc = sum(v for k, v in eng.stats.items() if k.endswith("ipc2z") or k.endswith("ipc_zc")) - zc_before
    comm.deregisterBuffer(y)
    fresh.update(reg_bad=reg_bad, keyed=keyed, zc_calls=zc, unkeyed_after=not eng._fast_ar.by_ptr)
    # reduceArray's latency tier is the same staged allreduce: memoised, then one native call
    launched.clear()
    z = torch.empty(1024, device="cuda")
    red_bad = 0
    for k in range(6):
        z.copy_(_pat(1024, r, k))
        comm.reduceArray(z, F, SUM, 0, 1024, 0)
        torch.cuda.synchronize()
        if r == 0:
            red_bad += int((z != _exp(1024, p, k)).sum())
    fresh.update(reduce_bad=red_bad, reduce_launched=launched.count(0),
                 reduce_calls=comm.stats["calls"].get("reduceArray", 0),
                 reduce_eng=sum(v for k, v in eng.stats.items() if k.startswith("reduce.ipc")))
    comm._fast_lx = orig
    # broadcast / gather / scatter / all-gather: one memoised copy plan, then one native call each
    from mp4x import CommUtils
    plan_rc = []
    orig_pl = comm._fast_pl

    def spy_pl(*a):
        rc = orig_pl(*a)
        plan_rc.append(rc)
        return rc
    comm._fast_pl = spy_pl
    n = 1024
    fr, to = CommUtils.createProcessArrayFroms(n, p), CommUtils.createProcessArrayTos(n, p)
    root = p - 1
    plan_bad = dict.fromkeys(("broadcast", "gather", "scatter", "allgather"), 0)
    for k in range(6):
        w = torch.full((n,), -1.0, device="cuda")
        if r == root:
            w.copy_(_pat(n, 7, k))
        comm.broadcastArray(w, F, 0, n, root)
        torch.cuda.synchronize()
        plan_bad["broadcast"] = plan_bad.get("broadcast", 0) + int((w != _pat(n, 7, k)).sum())
        w = torch.full((n,), -1.0, device="cuda")
        w[fr[r]:to[r]] = float(r + k)
        comm.gatherArray(w, F, list(fr), list(to), root)
        torch.cuda.synchronize()
        if r == root:
            plan_bad["gather"] = plan_bad.get("gather", 0) + sum(
                int((w[fr[j]:to[j]] != float(j + k)).sum()) for j in range(p))
        w = torch.full((n,), -1.0, device="cuda")
        if r == root:
            for j in range(p):
                w[fr[j]:to[j]] = float(10 * j + k)
        comm.scatterArray(w, F, list(fr), list(to), root)
        torch.cuda.synchronize()
        plan_bad["scatter"] = plan_bad.get("scatter", 0) + int((w[fr[r]:to[r]] != float(10 * r + k)).sum())
        w = torch.full((n,), -1.0, device="cuda")
        w[fr[r]:to[r]] = float(r - k)
        comm.allgatherArray(w, F, list(fr), list(to))
        torch.cuda.synchronize()
        plan_bad["allgather"] = plan_bad.get("allgather", 0) + sum(
            int((w[fr[j]:to[j]] != float(j - k)).sum()) for j in range(p))
    comm._fast_pl = orig_pl
    rs_rc = []
    orig_rs = comm._fast_rs

    def spy_rs(*a):
        rc = orig_rs(*a)
        rs_rc.append(rc)
        return rc
    comm._fast_rs = spy_rs
    counts = [t - f for f, t in zip(fr, to)]
    rs_bad = 0
    for k in range(6):
        w = _pat(n, r, k)
        comm.reduceScatterArray(w, F, SUM, 0, counts)
        torch.cuda.synchronize()
        rs_bad += int((w[fr[r]:to[r]] != _exp(n, p, k)[fr[r]:to[r]]).sum())
    comm._fast_rs = orig_rs
    fresh.update(rs_bad=rs_bad, rs_launched=rs_rc.count(0), rs_calls=comm.stats["calls"].get("reduceScatterArray", 0),
                 rs_eng=eng.stats.get("reduce_scatter.ipc", 0))
    api_calls = comm.stats["calls"]
    fresh.update(plan_bad=plan_bad, plan_launched=plan_rc.count(0), plan_refused=len(plan_rc) - plan_rc.count(0),
                 plan_calls={k: api_calls.get(k + "Array", 0) for k in ("broadcast", "gather", "scatter", "allgather")},
                 plan_eng={k: eng.stats.get(k + ".ipc", 0) for k in ("broadcast", "gather", "scatter", "allgather")})
    # an earlier collective that timed out fails the next call (no launch), then the job goes on
    x = torch.empty(1024, device="cuda")
    comm.barrier()
    ctypes.c_uint32.from_address(eng._ipc_obj._herr.value).value = 1
    raised = None
    try:
        comm.allreduceArray(x, F, SUM, 0, 1024)
    except Mp4jException as e:
        raised = str(e)
    comm.barrier()
    x.copy_(_pat(1024, r, 5))
    comm.allreduceArray(x, F, SUM, 0, 1024)
    torch.cuda.synchronize()
    after_fail_bad = int((x != _exp(1024, p, 5)).sum())
    # a registration (an input of the decision) clears the memo
    before = len(eng._fast_ar)
    y = torch.empty(1 << 20, device="cuda")
    comm.registerBuffer(y)
    cleared = len(eng._fast_ar) == 0 and before > 0
    comm.deregisterBuffer(y)
    return {"sizes": out, "calls": calls, "eng_calls": eng_calls, "raised": raised, "fresh": fresh,
            "after_fail_bad": after_fail_bad, "cleared": cleared}


def test_fast_path_is_exact_counted_invalidated_and_fail_stop():
    out = run_spawn(2, _fast_fn, timeout=240)
    for r, o in out.items():
        for tag, v in o["sizes"].items():
            assert v["bad"] == 0 and v["scale_bad"] == 0, (r, tag, v)
            assert v["memo"] >= 1, (r, tag, v)          # the shape was memoised
        assert o["calls"] == 2 * 43, o                   # every API call counted, fast or not
        assert o["eng_calls"] == 2 * 43, o
        assert o["raised"] and "timed out" in o["raised"], o
        assert o["after_fail_bad"] == 0 and o["cleared"], o
        f = o["fresh"]
        assert f["bad"] == 0 and f["reg_bad"] == 0, f
        assert f["addrs"] == 3 and f["by_ptr"] is False, f
        assert f["launched"] >= 8 and f["refused"] == 3, f    # 9 aligned calls (1st may miss), 3 unaligned
        assert f["keyed"] and f["zc_calls"] == 4 and f["unkeyed_after"], f
        assert f["reduce_bad"] == 0 and f["reduce_launched"] >= 5, f     # the first call memoises
        assert f["reduce_calls"] == 6 and f["reduce_eng"] == 6, f          # counted like the full path
        assert all(v == 0 for v in f["plan_bad"].values()) and len(f["plan_bad"]) == 4, f
        assert f["plan_launched"] >= 20 and f["plan_refused"] == 0, f      # 4 ops x 6 calls, first ones memoise
        assert all(v == 6 for v in f["plan_calls"].values()), f
        assert all(v == 6 for v in f["plan_eng"].values()), f
        assert f["rs_bad"] == 0 and f["rs_launched"] >= 5 and f["rs_calls"] == 6 and f["rs_eng"] == 6, f
