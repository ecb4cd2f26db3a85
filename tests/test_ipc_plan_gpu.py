"""IPC copy-plan collectives (csrc/runtime/ipc.hip k_ipc_copy_plan): broadcast / scatter / gather in
one kernel per call, p processes sharing ONE GPU, every root, ragged 16-byte segments; misaligned
ranges decline (False) identically on every rank so the engine falls back to RCCL."""
import multiprocessing as mp
import tempfile
import traceback

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _worker(port, q):
    try:
        import torch
        from mp4x import CommUtils, ProcessCommSlave
        from mp4x.parallel.ipc import IpcAllreduce
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("t", "127.0.0.1", port, heartbeat=False)
        r, p = comm.getRank(), comm.getSlaveNum()
        ipc = IpcAllreduce(comm, nbytes=1 << 20)
        res = []
        counts = [4 * (1000 + 300 * j) for j in range(p)]           # ragged, whole 16-byte vectors (f32)
        froms = CommUtils.getFromsFromCount(8, counts, p)
        tos = CommUtils.getTosFromCount(8, counts, p)
        n = tos[-1] + 12
        for root in range(p):
            # broadcast of [4, n - 8)
            x = torch.full((n,), -1.0, device="cuda")
            if r == root:
                x[4:n - 8] = torch.arange(n - 12, device="cuda", dtype=torch.float32) + root
            ok = ipc.broadcast(x, 4, n - 8, root)
            torch.cuda.synchronize()
            good = bool(torch.equal(x[4:n - 8], torch.arange(n - 12, device="cuda", dtype=torch.float32) + root))
            good &= bool(torch.all(x[:4] == (-1 if r != root else -1))) and bool(torch.all(x[n - 8:] == -1))
            res.append(("bcast", root, ok, good))
            # scatter: root holds segment j = j * 10 + root, rank r ends with its own
            x = torch.full((n,), -1.0, device="cuda")
            if r == root:
                for j in range(p):
                    x[froms[j]:tos[j]] = j * 10 + root
            ok = ipc.scatter(x, froms, tos, root)
            torch.cuda.synchronize()
            good = bool(torch.all(x[froms[r]:tos[r]] == r * 10 + root))
            res.append(("scatter", root, ok, good))
            # gather: rank j contributes segment j = j + 100 * root
            x = torch.full((n,), -1.0, device="cuda")
            x[froms[r]:tos[r]] = r + 100 * root
            ok = ipc.gather(x, froms, tos, root)
            torch.cuda.synchronize()
            if r == root:
                good = all(bool(torch.all(x[froms[j]:tos[j]] == j + 100 * root)) for j in range(p))
            else:
                good = bool(torch.all(x[froms[r]:tos[r]] == r + 100 * root))
            res.append(("gather", root, ok, good))
        # a misaligned range declines on every rank (nothing launched)
        x = torch.zeros(n, device="cuda")
        res.append(("misaligned", 0, not ipc.broadcast(x, 1, n - 8, 0), True))
        res.append(("error_word", 0, ipc.error_word() == 0, True))
        comm.barrier()
        ipc.close()
        comm.close(0)
        q.put((r, "ok", res))
    except BaseException:
        q.put((-1, "err", traceback.format_exc()))


@pytest.mark.parametrize("p", [2, 4])
def test_ipc_copy_plans(p):
    from mp4x import CommMaster
    m = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(m.port, q)) for _ in range(p)]
    for pr in procs:
        pr.start()
    res = {}
    try:
        for _ in range(p):
            r, st, val = q.get(timeout=240)
            assert st == "ok", val
            res[r] = val
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
        m.stop(timeout=5)
    for r, rows in res.items():
        for kind, root, ok, good in rows:
            assert ok and good, (r, kind, root)


def _engine_worker(port, q):
    try:
        import os
        os.environ["MP4X_DEVICE_BACKEND"] = "gloo"       # RCCL refuses 2 ranks on one GPU; IPC is real
        os.environ["MP4X_DEVICE_INDEX"] = "0"
        import torch
        from mp4x import CommUtils, Operands, ProcessCommSlave
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("t", "127.0.0.1", port, heartbeat=False)
        r, p = comm.getRank(), comm.getSlaveNum()
        F = Operands.FLOAT_OPERAND()
        n = 4096 * p
        froms = CommUtils.createProcessArrayFroms(n, p)
        tos = CommUtils.createProcessArrayTos(n, p)
        x = torch.full((n,), float(r), device="cuda")
        comm.broadcastArray(x, F, 0, n, p - 1)
        ok = bool(torch.all(x == p - 1))
        y = torch.full((n,), -1.0, device="cuda")
        if r == 0:
            for j in range(p):
                y[froms[j]:tos[j]] = j
        comm.scatterArray(y, F, froms, tos, 0)
        ok &= bool(torch.all(y[froms[r]:tos[r]] == r))
        z = torch.full((n,), -1.0, device="cuda")
        z[froms[r]:tos[r]] = r * 2
        comm.gatherArray(z, F, froms, tos, p - 1)
        if r == p - 1:
            ok &= all(bool(torch.all(z[froms[j]:tos[j]] == j * 2)) for j in range(p))
        from mp4x import Operators
        w = torch.full((n,), float(r + 1), device="cuda")
        comm.reduceArray(w, F, Operators.Float.SUM, 0, n, 0)
        if r == 0:
            ok &= bool(torch.all(w == p * (p + 1) / 2))
        st = dict(comm.device.stats)
        comm.close(0)
        q.put((r, "ok", (ok, st)))
    except BaseException:
        q.put((-1, "err", traceback.format_exc()))


def test_engine_routes_small_bcast_scatter_gather_reduce_through_ipc():
    from mp4x import CommMaster
    p = 2
    m = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_engine_worker, args=(m.port, q)) for _ in range(p)]
    for pr in procs:
        pr.start()
    res = {}
    try:
        for _ in range(p):
            r, st, val = q.get(timeout=240)
            assert st == "ok", val
            res[r] = val
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
        m.stop(timeout=5)
    for r, (ok, stats) in res.items():
        assert ok, r
        for k in ("broadcast.ipc", "scatter.ipc", "gather.ipc", "reduce.ipc1"):
            assert stats.get(k) == 1, (r, stats)


def _misaligned_worker(port, q):
    """Rank 0 passes tensors that start 4 bytes past a 16-byte boundary, rank 1 aligned ones:
    every IPC collective must still run the SAME protocol on both ranks (aligned temporaries on
    rank 0) — a rank-dependent decline would leave the peer spinning in a barrier."""
    try:
        import torch
        from mp4x import CommUtils, Operators, ProcessCommSlave
        from mp4x.parallel.ipc import IpcAllreduce, TWOSHOT
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("t", "127.0.0.1", port, heartbeat=False)
        r, p = comm.getRank(), comm.getSlaveNum()
        ipc = IpcAllreduce(comm, nbytes=1 << 20)
        n = 4096
        shift = 1 if r == 0 else 0

        def mk(fill):
            big = torch.empty(n + 4, device="cuda")
            v = big[shift:shift + n]
            v.copy_(fill)
            return v
        res = []
        base = torch.arange(n, device="cuda", dtype=torch.float32)
        x = mk(base + r)
        ipc.allreduce(x, Operators.Float.SUM, algo=TWOSHOT)
        res.append(("allreduce", bool(torch.equal(x, base * p + sum(range(p))))))
        froms, tos, _ = CommUtils.even_split(0, n, p)
        x = mk(base + r)
        ok = ipc.reduce_scatter(x, froms, tos, Operators.Float.SUM)
        res.append(("rs", ok and bool(torch.equal(x[froms[r]:tos[r]], (base * p + sum(range(p)))[froms[r]:tos[r]]))))
        x = mk(torch.full((n,), -1.0, device="cuda"))
        x[froms[r]:tos[r]] = r
        ok = ipc.allgather(x, froms, tos)
        res.append(("ag", ok and all(bool(torch.all(x[froms[j]:tos[j]] == j)) for j in range(p))))
        x = mk(base if r == 1 else torch.zeros(n, device="cuda"))
        ok = ipc.broadcast(x, 0, n, 1)
        res.append(("bcast", ok and bool(torch.equal(x, base))))
        x = mk(torch.full((n,), float(r), device="cuda"))
        ok = ipc.gather(x, froms, tos, 1)
        res.append(("gather", ok and (r != 1 or all(bool(torch.all(x[froms[j]:tos[j]] == j)) for j in range(p)))))
        x = mk(torch.full((n,), 0.0, device="cuda"))
        if r == 0:
            for j in range(p):
                x[froms[j]:tos[j]] = j + 10
        ok = ipc.scatter(x, froms, tos, 0)
        res.append(("scatter", ok and bool(torch.all(x[froms[r]:tos[r]] == r + 10))))
        x = mk(torch.ones(n, device="cuda"))
        ipc.allreduce_fp8(x)
        res.append(("fp8", bool(torch.allclose(x, torch.full_like(x, float(p)), rtol=2 ** -3))))
        torch.cuda.synchronize()
        res.append(("error_word", ipc.error_word() == 0))
        comm.barrier()
        ipc.close()
        comm.close(0)
        q.put((r, "ok", res))
    except BaseException:
        q.put((-1, "err", traceback.format_exc()))


def test_misaligned_tensor_on_one_rank_keeps_protocols_in_step():
    from mp4x import CommMaster
    m = CommMaster(2, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_misaligned_worker, args=(m.port, q)) for _ in range(2)]
    for pr in procs:
        pr.start()
    res = {}
    try:
        for _ in range(2):
            r, st, val = q.get(timeout=240)
            assert st == "ok", val
            res[r] = val
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
        m.stop(timeout=5)
    for r, rows in res.items():
        for name, good in rows:
            assert good, (r, name)
