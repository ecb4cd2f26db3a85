#!/usr/bin/env python3
"""BASELINE config 1: 2-thread in-process float[1024] allreduceArray on CPU (ThreadCommSlave
plumbing, no GPU).  One process, T threads, embedded master; p50 / p99 latency per call.

    python bench/thread_cpu.py [--threads 2] [--n 1024] [--iters 2000] [--procs 1]
"""
import argparse
import json
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(port, T, n, iters, out):
    import numpy as np
    from mp4x import Operands, Operators, ThreadCommSlave
    tc = ThreadCommSlave("bench", T, "127.0.0.1", port, heartbeat=False)
    lat = [[] for _ in range(T)]
    wall = [0.0] * T

    def body(t):
        tc.setThreadId(t)
        a = np.ones(n, dtype=np.float32)
        op, opnd = Operators.Float.SUM, Operands.FLOAT_OPERAND()
        for _ in range(50):
            tc.allreduceArray(a, opnd, op, 0, n)
        tc.threadBarrier()
        w0 = time.perf_counter()
        for _ in range(iters):
            t0 = time.perf_counter()
            tc.allreduceArray(a, opnd, op, 0, n)
            lat[t].append(time.perf_counter() - t0)
        wall[t] = time.perf_counter() - w0
        a[:] = t + 1                                 # one checked call after the timed ones
        tc.allreduceArray(a, opnd, op, 0, n)
        assert (a == T * (T + 1) // 2).all()

    ths = [threading.Thread(target=body, args=(t,)) for t in range(T)]
    [x.start() for x in ths]
    [x.join() for x in ths]
    tc.close(0)
    per_call = sorted(max(lat[t][i] for t in range(T)) for i in range(iters))
    out.append((per_call, max(wall) / iters))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=2000)
    a = ap.parse_args()
    from mp4x import CommMaster
    m = CommMaster(1, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    out = []
    worker(m.port, a.threads, a.n, a.iters, out)
    m.stop(timeout=5)
    lat, period = out[0]
    env = {k: os.environ[k] for k in ("MP4X_TEAM_EXT", "MP4X_TEAM_HANDOFF_US", "MP4X_THREAD_TEAM") if k in os.environ}
    print(json.dumps({"config": f"{a.threads}-thread in-process float[{a.n}] allreduceArray (CPU, ThreadCommSlave)",
                      "p50_us": round(lat[len(lat) // 2] * 1e6, 2),
                      "p99_us": round(lat[int(0.99 * len(lat))] * 1e6, 2),
                      "period_us": round(period * 1e6, 2),          # wall time per call, back to back
                      "calls_per_s": round(1 / period, 1), "env": env}))


if __name__ == "__main__":
    main()
