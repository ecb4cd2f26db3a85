#!/usr/bin/env python3
"""Host-path allreduce (numpy double[]) on one machine: TCP ring vs the C++ /dev/shm engine.

Same payloads as the reference's published table (1 GbE cluster there).
    python bench/host_allreduce.py --procs 4
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
    for _ in range(2):   # warm up: engine setup + first-touch page faults of the shm slots
        comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, n)
    comm.peer_barrier()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, n)
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from harness import run_ranks
    ref = {2: {100000: 12, 1000000: 110, 10000000: 955, 100000000: 9547},
           4: {100000: 23, 1000000: 130, 10000000: 1230, 100000000: 13283},
           8: {100000: 28, 1000000: 183, 10000000: 1641, 100000000: 16332}}
    for n in (100000, 1000000, 10000000, 100000000):
        for mode in ("tcp", "shm"):
            env = {"MP4X_SHM": "0" if mode == "tcp" else "1"}
            res, _, _ = run_ranks(a.procs, job, (n, a.iters), env=env, timeout=600)
            t = max(res.values())
            p = a.procs
            print(json.dumps({"procs": p, "elements": n, "engine": mode, "p50_ms": round(t * 1e3, 2),
                              "busbw_GBps": round(n * 8 / t / 1e9 * 2 * (p - 1) / p, 3),
                              "ref_ms_1GbE": ref.get(p, {}).get(n)}), flush=True)


if __name__ == "__main__":
    main()
