#!/usr/bin/env python3
"""Phase breakdown of the device sparse allreduce (BASELINE config 4 shape: 200k int64 ids x 64
float rows per rank, half the ids shared), p processes sharing GPU 0 (gloo stands in for RCCL,
the IPC copy plans are real).  Each phase of ``mp4x.parallel.sparse.allreduce_sparse`` is timed
with a device sync before and after it (diagnostic: the syncs add their own cost), then the
whole call without syncs.  One JSON line: per-phase ms (max over ranks) and the end-to-end p50.

    python bench/sparse_phases.py --procs 2 --iters 20 [--keys 200000 --dim 64]
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


def worker(port, q, nkeys, dim, iters):
    import torch
    from mp4x import Operators, ProcessCommSlave
    from mp4x.operators import dtype_of_torch, for_dtype
    from mp4x.ops import device_ops as K
    from mp4x.parallel import sparse as sp
    torch.cuda.set_device(0)
    os.environ.setdefault("MP4X_DEVICE_INDEX", "0")
    comm = ProcessCommSlave("b", "127.0.0.1", port, heartbeat=False)
    eng = comm.device
    r = comm.getRank()
    shared = nkeys // 2
    ids = torch.cat([torch.arange(shared), 10_000_000 + r * nkeys + torch.arange(nkeys - shared)]).cuda()
    vals = (torch.arange(nkeys * dim, device="cuda") % 7 + r).float().view(nkeys, dim)
    op = for_dtype(Operators.Float.SUM, dtype_of_torch(vals.dtype))
    for _ in range(3):
        comm.allreduceSparse(ids, vals, Operators.Float.SUM)
    torch.cuda.synchronize()

    phases = {}

    def tick(name, t0):
        torch.cuda.synchronize()
        t = time.perf_counter()
        phases.setdefault(name, []).append((t - t0) * 1e3)
        return t
    for _ in range(iters):
        eng.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        pc = K.partition_count(ids, eng.p)                     # K4b first half: counts + key range
        t = tick("pack_count", t)
        mat, bits, rng = sp._split_info(sp._count_matrix(eng, pc.info), eng.p, with_range=True)
        t = tick("count_matrix", t)
        rk, rv = sp._ipc_alltoallv(eng, ids, vals, mat,         # scatter into staging + the plan
                                   stage=lambda a, b: K.partition_scatter(pc, vals, a, b, 2))
        t = tick("ipc_alltoallv", t)
        uk, uv, _ = sp._reduce_by_key(rk, rv, op, bits, sp._dense_plan(rng, eng.p, rk))
        t = tick("reduce_by_key", t)
        sizes = sp._row_counts(eng, uk.shape[0], uk.device)
        t = tick("row_counts", t)
        sp._ipc_allgatherv(eng, uk, uv, sizes)
        tick("ipc_allgatherv", t)
    whole = []
    for _ in range(iters):
        eng.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        comm.allreduceSparse(ids, vals, Operators.Float.SUM)
        torch.cuda.synchronize()
        whole.append((time.perf_counter() - t0) * 1e3)
    comm.close(0)
    med = {k: sorted(v)[len(v) // 2] for k, v in phases.items()}
    q.put((r, med, sorted(whole)[len(whole) // 2]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--keys", type=int, default=200_000)
    ap.add_argument("--dim", type=int, default=64)
    a = ap.parse_args()
    os.environ.setdefault("MP4X_DEVICE_BACKEND", "gloo")
    from mp4x import CommMaster
    m = CommMaster(a.procs, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(m.port, q, a.keys, a.dim, a.iters)) for _ in range(a.procs)]
    [p.start() for p in ps]
    res = [q.get(timeout=600) for _ in range(a.procs)]
    [p.join(timeout=30) for p in ps]
    m.stop(timeout=5)
    names = list(res[0][1])
    print(json.dumps({"procs_on_one_gpu": a.procs, "keys_per_rank": a.keys, "dim": a.dim,
                      "phase_ms_p50_max_rank": {k: round(max(x[1][k] for x in res), 3) for k in names},
                      "whole_ms_p50_max_rank": round(max(x[2] for x in res), 3)}), flush=True)


if __name__ == "__main__":
    main()
