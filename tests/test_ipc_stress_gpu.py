"""Randomised soak of the IPC allreduce protocol (race detection).

p processes share GPU 0 and run the SAME seeded random sequence of calls: sizes from 16 B to
3 MiB through a 1 MiB buffer (so some calls are piecewise, pipelined or serial), one-shot /
two-shot, SUM / MAX, f32 / bf16 / f64 / i32, in place and out of place, back to back with no
host synchronisation in between, each rank pausing at random points of its own (so ranks run
ahead of each other, the case the one-shot's double-buffered slots and its start-barrier rule
exist for).  Every result is checked exactly (integers, small-integer floats) against a local
recomputation; the barrier error word must stay 0.
"""
import multiprocessing as mp
import os
import tempfile
import traceback

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ITERS = int(os.environ.get("MP4X_TEST_SOAK_ITERS", 120))      # a longer soak on demand
SEEDS = [int(x) for x in os.environ.get("MP4X_TEST_SOAK_SEEDS", "1,2").split(",")]


def _worker(port, q, seed):
    try:
        import random

        import torch
        from mp4x import Operators, ProcessCommSlave
        from mp4x.parallel.ipc import ONESHOT, TWOSHOT, IpcAllreduce
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("s", "127.0.0.1", port, heartbeat=False)
        r, p = comm.getRank(), comm.getSlaveNum()
        ipc = IpcAllreduce(comm, nbytes=4 << 20)    # 1-4 MiB single pieces take the slots
        rng = random.Random(seed)
        jitter = random.Random(seed * 31 + r)     # rank-dependent: ranks drift apart in time
        pending = []
        bad = []
        for it in range(ITERS):
            if jitter.random() < 0.15:
                # a late rank: the others run ahead — after a double-buffered one-shot (no end
                # barrier) a peer may store the NEXT call's start flag before this rank saw the
                # current one (csrc/runtime/ipc_common.hpp block_barrier)
                import time
                time.sleep(jitter.choice([0.0005, 0.002, 0.005]))
            dt = rng.choice([torch.float32, torch.bfloat16, torch.float64, torch.int32])
            es = torch.empty(0, dtype=dt).element_size()
            nbytes = rng.choice([16, 256, 4096, 65536, 300_000 // 16 * 16, (1 << 20) + 4096, 3 << 20, 4 << 20,
                                 (4 << 20) + 4096])
            n = nbytes // es
            algo = rng.choice([ONESHOT, TWOSHOT])
            opname = "SUM" if dt in (torch.int32, torch.float64) else rng.choice(["SUM", "MAX"])
            overlap = rng.choice([True, False])
            inplace = rng.choice([True, False])
            # rank-dependent small integers: exact in every dtype, sums stay exact
            base = torch.arange(n, device="cuda", dtype=torch.int64) % 13
            x = ((base + r * 3 + it) % 17).to(dt)
            out = x if inplace else torch.empty_like(x)
            ops = {torch.float32: Operators.Float, torch.bfloat16: Operators.BFloat16,
                   torch.float64: Operators.Double, torch.int32: Operators.Int}[dt]
            ipc.allreduce(x, getattr(ops, opname), algo=algo, out=out, overlap=overlap)
            pending.append((it, dt, n, opname, out))
            if len(pending) >= 8 or it == ITERS - 1:   # check lazily: several calls in flight
                torch.cuda.synchronize()
                for it2, dt2, n2, op2, o in pending:
                    b = torch.arange(n2, device="cuda", dtype=torch.int64) % 13
                    xs = [((b + j * 3 + it2) % 17) for j in range(p)]
                    ref = sum(xs) if op2 == "SUM" else torch.stack(xs).max(0).values
                    if not torch.equal(o.to(torch.int64), ref):
                        bad.append((it2, str(dt2), n2, op2))
                pending = []
        comm.barrier()
        ew = ipc.error_word()
        ipc.close()
        comm.close(0)
        q.put((r, "ok", (bad, ew)))
    except BaseException:
        q.put((-1, "err", traceback.format_exc()))


@pytest.mark.parametrize("p,seed", [(4, SEEDS[0]), (8, SEEDS[-1])])
def test_ipc_protocol_random_soak(p, seed):
    from mp4x import CommMaster
    m = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(m.port, q, seed)) for _ in range(p)]
    for pr in procs:
        pr.start()
    try:
        for _ in range(p):
            r, st, val = q.get(timeout=420)
            assert st == "ok", val
            bad, ew = val
            assert ew == 0, f"rank {r}: barrier timeout flag {ew}"
            assert not bad, (r, bad[:5])
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
        m.stop(timeout=5)


def _zc_soak_fn(comm, seed, iters):
    import random

    import torch
    from mp4x import CommUtils, Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    F = Operands.FLOAT_OPERAND()
    n = (48 << 20) // 4
    x = comm.memAlloc(n, torch.float32)
    rng = random.Random(seed)
    bad = []
    for it in range(iters):
        op = rng.choice(["allreduce", "reduce", "broadcast", "gather", "scatter", "reduce_scatter", "allgather"])
        root = rng.randrange(p)
        a = rng.randrange(0, n // 2) // 4 * 4                      # 16-byte grid
        b = min(n, a + rng.choice([1 << 16, 1 << 20, 3 << 20, 10 << 20]) // 4 * 4)
        idx = torch.arange(a, b, device="cuda", dtype=torch.int64)
        base = ((idx % 13) + it).float()
        if op in ("allreduce", "reduce"):
            x[a:b] = base + r
            (comm.allreduceArray(x, F, Operators.Float.SUM, a, b) if op == "allreduce"
             else comm.reduceArray(x, F, Operators.Float.SUM, a, b, root))
            exp = base * p + p * (p - 1) // 2
            ok = (op == "reduce" and r != root) or bool(torch.equal(x[a:b], exp))
        elif op == "broadcast":
            x[a:b] = base if r == root else -1.0
            comm.broadcastArray(x, F, a, b, root)
            ok = bool(torch.equal(x[a:b], base))
        else:
            m = b - a
            counts = [(m // p) // 4 * 4] * p
            counts[-1] = m - sum(counts[:-1])
            fr, to = CommUtils.getFromsFromCount(a, counts, p), CommUtils.getTosFromCount(a, counts, p)
            if op == "reduce_scatter":
                x[a:b] = base + r
                comm.reduceScatterArray(x, F, Operators.Float.SUM, a, counts)
                exp = base * p + p * (p - 1) // 2
                ok = bool(torch.equal(x[fr[r]:to[r]], exp[fr[r] - a:to[r] - a]))
            else:
                x[a:b] = -1.0
                if op == "scatter":
                    if r == root:
                        x[a:b] = base
                    comm.scatterArray(x, F, fr, to, root)
                    ok = bool(torch.equal(x[fr[r]:to[r]], base[fr[r] - a:to[r] - a]))
                else:
                    x[fr[r]:to[r]] = base[fr[r] - a:to[r] - a]
                    (comm.gatherArray(x, F, fr, to, root) if op == "gather" else comm.allgatherArray(x, F, fr, to))
                    ok = (op == "gather" and r != root) or bool(torch.equal(x[a:b], base))
        if not ok:
            bad.append((it, op, root, a, b))
    torch.cuda.synchronize()
    zc = sum(v for k, v in comm.device.stats.items() if k.endswith("ipc_zc") or k.endswith("ipc2z"))
    comm.memFree(x)
    return bad, zc


@pytest.mark.parametrize("p,seed", [(3, 5), (4, 6)])
def test_zero_copy_random_soak(p, seed):
    """The zero-copy forms of all 7 collectives on one memAlloc arena, a seeded random sequence of
    ops, roots and 16-byte-grid ranges (overlapping from call to call), every result exact."""
    from spawn_ranks import run_spawn
    iters = int(os.environ.get("MP4X_TEST_ZC_SOAK_ITERS", 60))
    out = run_spawn(p, _zc_soak_fn, args=(seed, iters), timeout=300)
    for r, (bad, zc) in out.items():
        assert not bad, (r, bad[:5])
        assert zc >= iters // 2, zc
