#!/usr/bin/env python3
"""BASELINE config 4 through the public Map API: ``allreduceMap`` of a ``Dict[str, Tensor]``
with 200k keys x float[64] per rank (half the keys shared by every rank, half private), p
virtual ranks on ONE GPU (LoopbackColl: the exchange is an in-process copy, the K4b / K5
kernels are real).  Reference: ProcessCommSlave.allreduceMap (ProcessCommSlave.java:2053-2088).

Reports, per call (median, max over virtual ranks): the whole call, and its split into
``to_tensors`` (dict -> id / row tensors: dictionary lookup + one stack), ``kernels`` (the
sparse allreduce: partition + exchange + sort + reduce-by-key + all-gather) and
``to_dict`` (id / row tensors -> dict of row views).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from loopback_cases import run_virtual
    from mp4x import Operators
    from mp4x.parallel import sparse

    # p virtual ranks are p threads of ONE process: with the default 5 ms GIL switch interval
    # every rendezvous between them can wait out switch intervals, a cost one-process-per-GPU
    # ranks never pay.  MAP_SWITCH_S sets a shorter one (A/B of the harness artifact).
    if os.environ.get("MAP_SWITCH_S"):
        sys.setswitchinterval(float(os.environ["MAP_SWITCH_S"]))
    DEV = os.environ.get("MAP_DEVICE", "cuda:0")
    p = int(os.environ.get("MAP_P", 8))
    nkeys = int(os.environ.get("MAP_KEYS", 200_000))
    dim = int(os.environ.get("MAP_DIM", 64))
    iters = int(os.environ.get("MAP_ITERS", 5))
    op = Operators.Float.SUM

    def sync():
        if DEV != "cpu":
            torch.cuda.synchronize()

    def body(eng, r, p):
        shared = nkeys // 2
        base = torch.randn(nkeys, dim, device=DEV)
        keys = [f"f{i}" for i in range(shared)] + [f"r{r}_{i}" for i in range(nkeys - shared)]
        m = dict(zip(keys, base.unbind(0)))
        ts = {"total": [], "to_tensors": [], "kernels": [], "to_dict": []}
        for it in range(iters + 1):
            sync()
            eng.barrier()
            t0 = time.perf_counter()
            out = eng.allreduce_map(m, op)
            sync()
            t1 = time.perf_counter()
            # the same call in its three phases
            eng.barrier()
            a = time.perf_counter()
            k, v, shape = sparse._map_tensors(eng, m)
            sync()
            b = time.perf_counter()
            rk, rv = sparse.allreduce_sparse(eng, k, v, op, sparse._dictionary(eng).bits)
            sync()
            c = time.perf_counter()
            out2 = sparse._tensors_map(eng, rk, rv, shape)
            d = time.perf_counter()
            if r == 0:
                print(f"iter {it}: total {t1 - t0:.3f}s to_tensors {b - a:.3f}s kernels {c - b:.3f}s "
                      f"to_dict {d - c:.3f}s", file=sys.stderr, flush=True)
            if it:
                ts["total"].append(t1 - t0)
                ts["to_tensors"].append(b - a)
                ts["kernels"].append(c - b)
                ts["to_dict"].append(d - c)
        assert len(out) == len(out2) == shared + p * (nkeys - shared)
        assert torch.allclose(out["f0"], out2["f0"])
        return {k: sorted(v)[len(v) // 2] for k, v in ts.items()}

    res = run_virtual(p, body, device=DEV)
    rec = {"config": "allreduceMap Dict[str, float[%d]] %d keys/rank (50%% shared)" % (dim, nkeys),
           "virtual_ranks": p, "result_keys": nkeys // 2 + p * (nkeys - nkeys // 2),
           "dict_per_call": "same dict every call (walk cached by PEP 509 version tag; "
                            "one_rank_host_pass_native_ms is the uncached walk)"}
    for k in ("total", "to_tensors", "kernels", "to_dict"):
        rec[f"{k}_ms"] = round(max(r[k] for r in res) * 1e3, 2)
    rec.update(one_rank_host_pass(DEV, nkeys, dim, iters, sync))
    print(json.dumps(rec), flush=True)


def one_rank_host_pass(dev, nkeys, dim, iters, sync):
    """What ONE process (one rank per GPU) pays on the host to turn its dict into (ids, rows):
    the virtual-rank numbers above serialise p ranks' Python on one GIL.  Native walk
    (csrc/pyext/map_ext.cpp) vs the Python form of the same pass."""
    import numpy as np
    import torch
    from mp4x.parallel import sparse
    keys = [f"f{i}" for i in range(nkeys)]
    d = sparse.KeyDictionary()
    d.learn_round([keys])
    base = torch.randn(nkeys, dim, device=dev)
    m = dict(zip(keys, base.unbind(0)))

    def native():
        ids, _, rows, b = sparse._pack_native(d, m)
        v = sparse._take_rows(b.reshape(-1, dim), rows)
        return torch.from_numpy(ids).to(dev), v

    def python():
        ids = d.lookup(list(m.keys()))
        v = sparse._stack_rows(list(m.values()))
        return torch.from_numpy(ids).to(dev), v

    def native_cached():
        return native()

    out = {}
    for name, fn in (("native", native), ("python", python), ("native_same_dict_cached", native_cached)):
        # "native": the full walk every call (walk cache off); "..._cached": the same dict passed
        # again unmodified, which skips the walk (PEP 509 version tag, sparse._pack_native)
        sparse._WALK_CACHE = name == "native_same_dict_cached"
        d._walk_cache = None
        ts = []
        for _ in range(iters + 1):
            sync()
            t0 = time.perf_counter()
            fn()
            sync()
            ts.append(time.perf_counter() - t0)
        out[f"one_rank_host_pass_{name}_ms"] = round(sorted(ts[1:])[len(ts[1:]) // 2] * 1e3, 2)
    sparse._WALK_CACHE = True
    a, b = native(), python()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    return out


if __name__ == "__main__":
    main()
