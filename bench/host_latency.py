#!/usr/bin/env python3
"""Host-path latency: ``allreduceArray`` of a small numpy double[] between p processes on one
host (the /dev/shm engine), wall time per call, p50 of the per-rank means (max over ranks).

    python bench/host_latency.py --procs 2,4 --n 16 --iters 3000
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def job(comm, n, iters):
    import numpy as np
    from mp4x import Operands, Operators
    a = np.ones(n)
    D, S = Operands.DOUBLE_OPERAND(), Operators.Double.SUM
    for _ in range(50):
        comm.allreduceArray(a, D, S, 0, n)
    comm.peer_barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        comm.allreduceArray(a, D, S, 0, n)
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="2,4")
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--iters", type=int, default=3000)
    a = ap.parse_args()
    from harness import run_ranks
    for p in (int(x) for x in a.procs.split(",")):
        res, _, _ = run_ranks(p, job, (a.n, a.iters), timeout=300)
        print(json.dumps({"procs": p, "elements": a.n, "engine": "shm",
                          "us_per_call_max_rank": round(max(res.values()) * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
