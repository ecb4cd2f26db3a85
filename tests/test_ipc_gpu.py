"""Custom IPC allreduce (csrc/runtime/ipc.hip): p processes sharing ONE GPU.

On a single-GPU box the peers' buffers are IPC mappings of memory on the same device, which
exercises the whole protocol (handle exchange, epoch flags, per-block barriers, one-shot and
two-shot schedules, piecewise large messages) except the xGMI hop itself.
"""
import multiprocessing as mp
import os
import tempfile
import traceback

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _ipc_worker(port, q, sizes, dtype_name, algos, nbytes_buf):
    try:
        import torch
        from mp4x import ProcessCommSlave, Operators
        from mp4x.parallel.ipc import IpcAllreduce, ONESHOT, TWOSHOT
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("t", "127.0.0.1", port, heartbeat=False)
        r, p = comm.getRank(), comm.getSlaveNum()
        dt = getattr(torch, dtype_name)
        ipc = IpcAllreduce(comm, nbytes=nbytes_buf)
        res = []
        for n in sizes:
            for algo in algos:
                for op in ("SUM", "MAX"):
                    g = torch.Generator(device="cuda").manual_seed(1000 + r)
                    x = torch.randn(n, device="cuda", generator=g).to(dt)
                    out = torch.empty_like(x)
                    operator = getattr(Operators.Float, op)
                    ipc.allreduce(x, operator, algo=algo, out=out)
                    torch.cuda.synchronize()
                    # reference: regenerate every rank's input locally
                    xs = [torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1000 + j)).to(dt)
                          for j in range(p)]
                    if op == "SUM":
                        ref = xs[0].double()
                        for j in range(1, p):
                            ref = ref + xs[j].double()
                    else:
                        ref = xs[0].double()
                        for j in range(1, p):
                            ref = torch.maximum(ref, xs[j].double())
                    err = (out.double() - ref).abs().max().item() if n else 0.0
                    res.append((n, algo, op, err, ipc.error_word()))
        comm.barrier()
        ipc.close()
        comm.close(0)
        q.put((r, "ok", res))
    except BaseException:
        q.put((-1, "err", traceback.format_exc()))


def _run(p, sizes, dtype_name="float32", algos=(0, 1), nbytes_buf=1 << 20):
    from mp4x import CommMaster
    m = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ipc_worker, args=(m.port, q, sizes, dtype_name, algos, nbytes_buf)) for _ in range(p)]
    for pr in procs:
        pr.start()
    out = {}
    try:
        for _ in range(p):
            r, st, val = q.get(timeout=240)
            assert st == "ok", val
            out[r] = val
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
        m.stop(timeout=5)
    return out


@pytest.mark.parametrize("p", [2, 4])
def test_ipc_allreduce_f32(p):
    # 64 elems (one vector per thread at most), ragged sizes, and > buffer (piecewise)
    out = _run(p, [64, 4 * 1000, 3 * (1 << 18) + 4096])
    for r, res in out.items():
        for n, algo, op, err, ew in res:
            assert ew == 0, f"rank {r}: barrier timeout flag {ew}"
            assert err < 1e-4 * p, (r, n, algo, op, err)


@pytest.mark.parametrize("overlap", ["1", "0"])
def test_ipc_allreduce_large_pipelined(overlap, monkeypatch):
    """10 MiB messages through a 1 MiB buffer: half-buffer pieces with the input copy of the
    next piece overlapped on a side stream (MP4X_IPC_OVERLAP=1) or serial pieces (0)."""
    monkeypatch.setenv("MP4X_IPC_OVERLAP", overlap)
    out = _run(2, [(10 << 20) // 4 + 64], algos=(1,))
    for r, res in out.items():
        for n, algo, op, err, ew in res:
            assert ew == 0 and err < 1e-4 * 2, (r, n, algo, op, err)


def test_ipc_allreduce_bf16():
    out = _run(2, [8 * 4096], dtype_name="bfloat16")
    for r, res in out.items():
        for n, algo, op, err, ew in res:
            assert ew == 0 and err < 0.05, (n, algo, op, err)


def _graph_worker(port, q, n, replays):
    try:
        import torch
        from mp4x import ProcessCommSlave, Operators
        from mp4x.parallel.ipc import IpcAllreduce, ONESHOT, TWOSHOT
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("t", "127.0.0.1", port, heartbeat=False)
        r, p = comm.getRank(), comm.getSlaveNum()
        ipc = IpcAllreduce(comm, nbytes=1 << 20).prepare_graph()
        x = torch.zeros(n, device="cuda")
        y = torch.zeros(n, device="cuda")
        ipc.allreduce(x, Operators.Float.SUM, algo=ONESHOT, out=y)      # eager call in graph mode
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            ipc.allreduce(x, Operators.Float.SUM, algo=TWOSHOT, out=y)
        torch.cuda.synchronize()
        bad = 0
        for i in range(replays):
            x.fill_(float(r + 1 + i))
            g.replay()
            torch.cuda.synchronize()
            expect = sum(j + 1 + i for j in range(p))
            bad += int((y != expect).sum().item())
            if i % 5 == 0:   # interleave eager calls with replays
                ipc.allreduce(x, Operators.Float.SUM, algo=ONESHOT, out=y)
                torch.cuda.synchronize()
                bad += int((y != expect).sum().item())
        comm.barrier()
        ew = ipc.error_word()
        ipc.close()
        comm.close(0)
        q.put((r, "ok", (bad, ew)))
    except BaseException:
        q.put((-1, "err", traceback.format_exc()))


def test_ipc_allreduce_hipgraph_replay():
    from mp4x import CommMaster
    p = 3
    m = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_graph_worker, args=(m.port, q, 4096 * 3, 20)) for _ in range(p)]
    for pr in procs:
        pr.start()
    try:
        for _ in range(p):
            r, st, val = q.get(timeout=240)
            assert st == "ok", val
            assert val == (0, 0), (r, val)
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
        m.stop(timeout=5)


def _rsag_worker(port, q):
    try:
        import torch
        from mp4x import Operators, ProcessCommSlave
        from mp4x.parallel.ipc import IpcAllreduce
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("t", "127.0.0.1", port, heartbeat=False)
        r, p = comm.getRank(), comm.getSlaveNum()
        ipc = IpcAllreduce(comm, nbytes=1 << 20)
        errs = []
        for dt, opname in ((torch.float32, "SUM"), (torch.bfloat16, "MAX"), (torch.int64, "SUM")):
            es = torch.empty(0, dtype=dt).element_size()
            q16 = 16 // es                                     # elements per 16 bytes
            counts = [q16 * (3 + 5 * j) for j in range(p)]      # ragged, 16-byte multiples
            base = 2 * q16
            froms = [base + sum(counts[:j]) for j in range(p)]
            tos = [f + c for f, c in zip(froms, counts)]
            n = tos[-1] + 7
            x = ((torch.arange(n, device="cuda") % 11) + r).to(dt)
            ops = {torch.float32: Operators.Float, torch.bfloat16: Operators.BFloat16, torch.int64: Operators.Long}[dt]
            y = x.clone()
            assert ipc.reduce_scatter(y, froms, tos, getattr(ops, opname))
            xs = [((torch.arange(n, device="cuda") % 11) + j).to(torch.float64) for j in range(p)]
            ref = sum(xs) if opname == "SUM" else torch.stack(xs).max(0).values
            if not torch.equal(y[froms[r]:tos[r]].double(), ref[froms[r]:tos[r]]):
                errs.append(("rs", str(dt)))
            if not torch.equal(y[:froms[0]], x[:froms[0]]) or not torch.equal(y[tos[-1]:], x[tos[-1]:]):
                errs.append(("rs-outside", str(dt)))
            z = torch.full((n,), -1, device="cuda").to(dt)
            z[froms[r]:tos[r]] = r
            assert ipc.allgather(z, froms, tos)
            for j in range(p):
                if not bool((z[froms[j]:tos[j]] == j).all()):
                    errs.append(("ag", str(dt), j))
            # a range whose byte offset is not a 16-byte multiple does not qualify (same on every rank)
            assert not ipc.allgather(z, [froms[0] + 1] + froms[1:], tos)
        torch.cuda.synchronize()
        comm.barrier()
        ew = ipc.error_word()
        ipc.close()
        comm.close(0)
        q.put((r, "ok", (errs, ew)))
    except BaseException:
        q.put((-1, "err", traceback.format_exc()))


@pytest.mark.parametrize("p", [2, 3])
def test_ipc_direct_reduce_scatter_allgather_ragged(p):
    from mp4x import CommMaster
    m = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rsag_worker, args=(m.port, q)) for _ in range(p)]
    for pr in procs:
        pr.start()
    try:
        for _ in range(p):
            r, st, val = q.get(timeout=240)
            assert st == "ok", val
            errs, ew = val
            assert ew == 0 and not errs, (r, errs, ew)
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
        m.stop(timeout=5)
