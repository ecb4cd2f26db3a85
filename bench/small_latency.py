#!/usr/bin/env python3
"""Public-API latency of small device allreduces (the latency tier: IPC one-shot), p processes
sharing GPU 0: wall time per ``comm.allreduceArray`` call incl. every host-side layer (tracer,
collective watchdog, schedule selection, ctypes launches).  Rehearsal numbers: protocol and host
overhead, not xGMI latency.  One JSON line per size.

    python bench/small_latency.py --procs 2 --iters 2000 [--sizes 4096,65536]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(port, q, sizes, iters, profile=None, ops=False):
    import torch
    from mp4x import Operands, Operators, ProcessCommSlave
    torch.cuda.set_device(0)
    os.environ.setdefault("MP4X_DEVICE_INDEX", "0")
    comm = ProcessCommSlave("b", "127.0.0.1", port, heartbeat=False)
    eng = comm.device            # gloo stands in for RCCL on a shared GPU; the IPC tier is real
    out = []
    if ops:
        from mp4x import CommUtils
        p, r = comm.getSlaveNum(), comm.getRank()
        for nb in sizes:
            n = nb // 8                                  # double[] like the reference's table
            x = torch.randn(n, device="cuda", dtype=torch.float64)
            D, SUM = Operands.DOUBLE_OPERAND(), Operators.Double.SUM
            fr, to = CommUtils.createProcessArrayFroms(n, p), CommUtils.createProcessArrayTos(n, p)
            calls = {"gather": lambda: comm.gatherArray(x, D, fr, to, 0),
                     "scatter": lambda: comm.scatterArray(x, D, fr, to, 0),
                     "allgather": lambda: comm.allgatherArray(x, D, fr, to),
                     "reduce_scatter": lambda: comm.reduceScatterArray(x, D, SUM, 0, [t - f for f, t in zip(fr, to)]),
                     "broadcast": lambda: comm.broadcastArray(x, D, 0, n, 0),
                     "reduce": lambda: comm.reduceArray(x, D, SUM, 0, n, 0),
                     "allreduce": lambda: comm.allreduceArray(x, D, SUM, 0, n)}
            for name, fn in calls.items():
                for _ in range(20):
                    fn()
                torch.cuda.synchronize()
                eng.barrier()
                prof = None
                if profile and comm.getRank() == 0:
                    import cProfile
                    prof = cProfile.Profile()
                    prof.enable()
                t0 = time.perf_counter()
                for _ in range(iters):
                    fn()
                torch.cuda.synchronize()
                out.append({"op": name, "bytes": n * 8, "us_per_call": (time.perf_counter() - t0) / iters * 1e6})
                if prof is not None:
                    prof.disable()
                    import io
                    import pstats
                    buf = io.StringIO()
                    pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(30)
                    with open(f"{profile}.{name}.{n * 8}.txt", "w") as f:
                        f.write(buf.getvalue())
                eng.barrier()
        comm.close(0)
        q.put((comm.getRank(), out))
        return
    for nb in sizes:
        x = torch.randn(nb // 4, device="cuda")
        opnd, op = Operands.FLOAT_OPERAND(), Operators.Float.SUM
        for _ in range(50):
            comm.allreduceArray(x, opnd, op, 0, x.numel())
        torch.cuda.synchronize()
        eng.barrier()
        prof = None
        if profile and comm.getRank() == 0:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        for _ in range(iters):
            comm.allreduceArray(x, opnd, op, 0, x.numel())
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        if prof is not None:
            prof.disable()
            import io
            import pstats
            buf = io.StringIO()
            pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(25)
            with open(f"{profile}.{nb}.txt", "w") as f:
                f.write(buf.getvalue())
        out.append({"bytes": nb, "us_per_call": dt * 1e6, "algo": eng.select("allreduce", nb, op, x.dtype, opnd)})
        eng.barrier()
    comm.close(0)
    q.put((comm.getRank(), out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--sizes", default="4096,65536")
    ap.add_argument("--profile", default=None, help="cProfile rank 0's timed loop into <prefix>.<bytes>.txt")
    ap.add_argument("--all-ops", action="store_true",
                    help="every collective of the reference's table on double[] (sizes in bytes)")
    a = ap.parse_args()
    os.environ.setdefault("MP4X_DEVICE_BACKEND", "gloo")
    from mp4x import CommMaster
    m = CommMaster(a.procs, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    sizes = [int(x) for x in a.sizes.split(",")]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(m.port, q, sizes, a.iters, a.profile, a.all_ops)) for _ in range(a.procs)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=600) for _ in range(a.procs))
    [p.join(timeout=30) for p in ps]
    m.stop(timeout=5)
    for i, row in enumerate(res[0]):
        worst = max(res[r][i]["us_per_call"] for r in res)
        if a.all_ops:
            print(json.dumps({"procs_on_one_gpu": a.procs, **row, "us_per_call_max_rank": worst}))
            continue
        print(json.dumps({"procs_on_one_gpu": a.procs, "watchdog": os.environ.get("MP4X_WATCHDOG", "1"),
                          **row, "us_per_call_max_rank": worst}))


if __name__ == "__main__":
    main()
