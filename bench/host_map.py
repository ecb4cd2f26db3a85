#!/usr/bin/env python3
"""Host ``allreduceMap`` (values on the CPU) across p real processes over the TCP data plane:
``Dict[str, float32[dim]]`` with half the keys shared by every rank, half private.

Reference: ProcessCommSlave.allreduceMap (J/comm/ProcessCommSlave.java:2053-2088): Java-hash
owner partition -> ring reduce-scatter of per-owner maps -> ring allgather -> merge.
Prints one JSON line: median / max-over-ranks ms per call.

  python bench/host_map.py [--p 2] [--keys 50000] [--dim 16] [--iters 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def body(comm, nkeys, dim, iters):
    import numpy as np
    from mp4x import Operands, Operators
    r = comm.getRank()
    rng = np.random.default_rng(r)
    m = {f"f{i}": rng.standard_normal(dim).astype(np.float32) for i in range(nkeys // 2)}
    m.update({f"r{r}_{i}": rng.standard_normal(dim).astype(np.float32) for i in range(nkeys - nkeys // 2)})
    ts, tl = [], []
    out = None
    for _ in range(iters + 1):
        comm.barrier()
        t0 = time.perf_counter()
        out = comm.allreduceMap(m, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
        t1 = time.perf_counter()
        _ = out["f0"]                   # first lookup: builds a RowMap's key index
        ts.append(t1 - t0)
        tl.append(time.perf_counter() - t0)
    mid = len(ts[1:]) // 2
    return len(out), sorted(ts[1:])[mid], sorted(tl[1:])[mid], type(out).__name__


def main():
    from harness import run_ranks
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, default=2)
    ap.add_argument("--keys", type=int, default=50_000)
    ap.add_argument("--dim", type=int, default=16)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    res, _, _ = run_ranks(a.p, body, args=(a.keys, a.dim, a.iters), timeout=600)
    n = {v[0] for v in res.values()}
    assert n == {a.keys // 2 + a.p * (a.keys - a.keys // 2)}, n
    print(json.dumps({"config": f"host allreduceMap Dict[str, float32[{a.dim}]] {a.keys} keys/rank (50% shared)",
                      "procs": a.p, "result_keys": n.pop(),
                      "map_algo": os.environ.get("MP4X_HOST_MAP_ALGO", "auto"),
                      "native_ext": os.environ.get("MP4X_MAP_EXT", "1") != "0",
                      "p50_ms_max_rank": round(max(v[1] for v in res.values()) * 1e3, 2),
                      "p50_ms_incl_first_lookup": round(max(v[2] for v in res.values()) * 1e3, 2),
                      "result_type": res[0][3]}))


if __name__ == "__main__":
    main()
