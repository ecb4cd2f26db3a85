#!/usr/bin/env python3
"""Host TCP allreduce schedules: ring (reference) vs recursive halving/doubling, p = 4/8/6.

    python bench/host_allreduce_algos.py   # -> one JSON line per (p, elements); p50 over iterations
"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from harness import run_ranks

def job(comm, n, iters):
    import numpy as np
    from mp4x import Operands, Operators
    a = np.ones(n)
    for _ in range(3):
        comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, n)
    comm.peer_barrier()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, n)
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]

for p in (4, 8, 6):
    for n in (16, 1024, 32768, 1000000):
        row = {"procs": p, "elements": n}
        for algo in ("ring", "rhd"):
            res, _, _ = run_ranks(p, job, (n, 30 if n < 100000 else 8), env={"MP4X_SHM": "0", "MP4X_HOST_ALGO": algo}, timeout=300)
            row[algo + "_p50_us"] = round(max(res.values()) * 1e6, 1)
        print(json.dumps(row), flush=True)
