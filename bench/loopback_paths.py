#!/usr/bin/env python3
"""Device-engine schedules with p virtual ranks on ONE GPU (LoopbackColl), for rocprofv3.

No xGMI here (the "collective" is an in-process copy); what this measures is the local
kernel work of each schedule with the real HIP kernels: K1 rank-ordered reduce (a2a two-shot),
K6 fp8 quant / fused dequant-reduce-requant, K6b zero suppression, K4b partition + K5
reduce-by-key (sparse map).  Prints one JSON line per schedule (median wall ms per call,
max over virtual ranks).

    rocprofv3 --kernel-trace --stats -d gpurun_out/lb -- python3 bench/loopback_paths.py
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
    from mp4x.operands import Operands
    from mp4x.parallel.sparse import allreduce_sparse

    p = int(os.environ.get("LB_P", 8))
    iters = int(os.environ.get("LB_ITERS", 5))
    n = 16 << 20          # 64 MiB f32 per rank

    def timed(fn):
        def body(eng, r, p):
            ts = []
            for i in range(iters + 1):
                torch.cuda.synchronize()
                eng.barrier()
                t0 = time.perf_counter()
                fn(eng, r, p)
                torch.cuda.synchronize()
                if i:
                    ts.append(time.perf_counter() - t0)
            return sorted(ts)[len(ts) // 2]
        return body

    def dense(algo, operand=None):
        def f(eng, r, p):
            eng.algo = algo
            x = f.buf.setdefault(r, torch.randn(n, device="cuda:0"))
            eng.allreduce(x, 0, n, Operators.Float.SUM, operand)
        f.buf = {}
        return f

    def sparse_density(eng, r, p, cache={}):
        x = cache.get(r)
        if x is None:
            x = cache[r] = torch.randn(n, device="cuda:0") * (torch.rand(n, device="cuda:0") < 0.05)
        eng.algo = "auto"
        eng.allreduce(x.clone(), 0, n, Operators.Float.SUM, Operands.FLOAT_OPERAND(compress=True))

    def sparse_map(eng, r, p, cache={}):
        kv = cache.get(r)
        if kv is None:
            g = torch.Generator(device="cuda:0").manual_seed(r)
            keys = torch.randint(0, 1 << 40, (200_000,), device="cuda:0", generator=g).unique()
            kv = cache[r] = (keys, torch.randn(keys.numel(), 64, device="cuda:0"))
        allreduce_sparse(eng, kv[0], kv[1], Operators.Float.SUM)

    cases = [("a2a_allreduce_64MiB", timed(dense("a2a"))),
             ("fp8_allreduce_64MiB", timed(dense("auto", Operands.FLOAT_OPERAND(codec="fp8")))),
             ("zs_allreduce_64MiB_5pct", timed(sparse_density)),
             ("sparse_map_200kx64", timed(sparse_map))]
    for name, fn in cases:
        t = max(run_virtual(p, fn, device="cuda:0"))
        print(json.dumps({"virtual_ranks": p, "schedule": name, "ms_per_call": round(t * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
