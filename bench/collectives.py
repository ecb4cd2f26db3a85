#!/usr/bin/env python3
"""nccl-tests-style sweep of every mp4x collective on MI355X + the BASELINE.json configs.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/collectives.py --sweep ref
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/collectives.py --config zero_bf16
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/collectives.py --config sparse_map
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/collectives.py --config fp8_8gb

``--sweep ref`` runs the reference's published table shape: double[] of
1e5 ... 1e9 elements for gather / scatter / allgather / reduce-scatter / broadcast / reduce /
allreduce, reporting algbw, busbw (nccl-tests factors) and p50/p99 per size,
plus the reference's own time at that (p, size) for comparison.  One JSON line per row.
``--check`` adds one exact-value verification call per (op, size) after the timed calls
(small-integer patterns, exact in double; the row gets ``"exact": true/false``); the configs
check their results too (exact for the bf16 ZeRO pair, error-bounded against the fp64 sum for
the fp8-compressed allreduce).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# README.md:341-352 of the reference (8 slaves, 1 GbE, ms) and :302-339 for 2/4/6
REF_MS = {
    2: {100000: [6, 6, 6, 7, 12, 12, 12], 1000000: [48, 43, 45, 38, 95, 105, 110],
        10000000: [397, 355, 445, 447, 850, 840, 955], 100000000: [3526, 3555, 4667, 4611, 8002, 8061, 9547],
        1000000000: [34228, 34464, 47179, 47361, 80846, 78442, 93624]},
    4: {100000: [12, 8, 10, 11, 19, 20, 23], 1000000: [57, 56, 63, 65, 118, 121, 130],
        10000000: [538, 534, 630, 618, 1149, 1237, 1230], 100000000: [5223, 5266, 6601, 7322, 11973, 11894, 13283],
        1000000000: [51396, 52517, 65308, 62918, 117354, 118999, 129174]},
    6: {100000: [13, 13, 14, 14, 24, 24, 24], 1000000: [62, 62, 75, 84, 155, 146, 159],
        10000000: [602, 762, 681, 731, 1533, 1561, 1529], 100000000: [5770, 6934, 7584, 7408, 14734, 15791, 15226],
        1000000000: [56946, 57042, 74376, 69005, 140572, 126827, 143813]},
    8: {100000: [16, 11, 15, 14, 24, 25, 28], 1000000: [69, 67, 92, 85, 152, 155, 183],
        10000000: [645, 648, 741, 749, 1449, 1431, 1641], 100000000: [6050, 6143, 8716, 8931, 14800, 14561, 16332],
        1000000000: [59974, 61426, 75464, 74495, 136574, 134260, 154090]},
}
OPS = ["gather", "scatter", "allgather", "reduce_scatter", "broadcast", "reduce", "allreduce"]


def busfactor(op, p):
    if op in ("gather", "scatter", "allgather", "reduce_scatter"):
        return (p - 1) / p
    if op in ("broadcast", "reduce"):
        return 1.0
    return 2.0 * (p - 1) / p


def timed(fn, iters, warmup, sync):
    import torch
    for _ in range(warmup):
        fn()
    sync()
    s = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
    for i in range(iters):
        s[i].record()
        fn()
        e[i].record()
    sync()
    ts = sorted(a.elapsed_time(b) for a, b in zip(s, e))
    return ts[len(ts) // 2], ts[min(len(ts) - 1, int(0.99 * len(ts)))]


def check_op(op, buf, comm, D, froms, tos, counts, p, r, sync):
    """One exact-value call of ``op`` on small-integer patterns (exact in double).  Patterns are
    built and compared in chunks, so a 1e9-double row needs no full-size temporaries."""
    import torch
    from mp4x import Operators
    n = buf.numel()
    CH = 1 << 26
    root = 0

    def base(s, e):
        return torch.remainder(torch.arange(s, e, device=buf.device, dtype=torch.float64), 97)

    def fill(fn, lo=0, hi=n):
        for s in range(lo, hi, CH):
            buf[s:min(hi, s + CH)] = fn(s, min(hi, s + CH))

    def same(fn, lo=0, hi=n):
        return all(bool(torch.equal(buf[s:min(hi, s + CH)], fn(s, min(hi, s + CH)))) for s in range(lo, hi, CH))

    if op in ("gather", "allgather"):
        buf.fill_(-1)
        buf[froms[r]:tos[r]] = r + 1
        (comm.gatherArray(buf, D, froms, tos, root) if op == "gather" else comm.allgatherArray(buf, D, froms, tos))
        sync()
        if op == "gather" and r != root:
            return True
        return all(bool((buf[froms[j]:tos[j]] == j + 1).all()) for j in range(p))
    if op == "scatter":
        buf.fill_(-1)
        if r == root:
            for j in range(p):
                buf[froms[j]:tos[j]] = j + 1
        comm.scatterArray(buf, D, froms, tos, root)
        sync()
        return bool((buf[froms[r]:tos[r]] == r + 1).all())
    if op == "broadcast":
        if r == root:
            fill(base)
        else:
            buf.fill_(-1)
        comm.broadcastArray(buf, D, 0, n, root)
        sync()
        return same(base)
    fill(lambda s, e: base(s, e) + r)

    def exp(s, e):
        return base(s, e) * p + p * (p - 1) // 2
    if op == "reduce_scatter":
        comm.reduceScatterArray(buf, D, Operators.Double.SUM, 0, counts)
        sync()
        return same(exp, froms[r], tos[r])
    if op == "reduce":
        comm.reduceArray(buf, D, Operators.Double.SUM, 0, n, root)
        sync()
        return r != root or same(exp)
    comm.allreduceArray(buf, D, Operators.Double.SUM, 0, n)
    sync()
    return same(exp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", choices=["ref", "none"], default="none")
    ap.add_argument("--config", choices=["none", "zero_bf16", "sparse_map", "fp8_8gb", "allreduce_1gb"],
                    default="none")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--max-elems", type=float, default=1e9)
    ap.add_argument("--check", action="store_true", help="exact-value check of every row / config")
    ap.add_argument("--ops", default=",".join(OPS), help="--sweep ref: comma list of collectives to run")
    ap.add_argument("--alloc", choices=("memalloc", "plain"), default="memalloc",
                    help="configs: the big tensor from comm.memAlloc (zero-copy at any size) or torch.empty")
    ap.add_argument("--sizes", default=None, help="--sweep ref: comma list of element counts (default: ref sizes)")
    ap.add_argument("--sweep-alloc", choices=("plain", "memalloc"), default="plain",
                    help="--sweep ref: the swept array from torch (staged kernels above the registration limit) "
                         "or comm.memAlloc (mapped into every peer: zero-copy kernels at any size, e.g. 1e9 doubles)")
    ap.add_argument("--codecs", default="none,fp8", help="fp8_8gb config: wire codecs to run")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from mp4x import CommUtils, Operands, Operators
    from mp4x.launch import init_from_env
    local = int(os.environ.get("MP4X_DEVICE_INDEX", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    comm = init_from_env(heartbeat=False)
    p, r = comm.getSlaveNum(), comm.getRank()
    eng = comm.device if p > 1 else None

    def sync():
        torch.cuda.synchronize()
        if eng is not None:
            eng.barrier()
            torch.cuda.synchronize()

    def emit(rec):
        if r == 0:
            print(json.dumps(rec), flush=True)

    if a.sweep == "ref":
        D = Operands.DOUBLE_OPERAND()
        sizes = [int(float(x)) for x in a.sizes.split(",")] if a.sizes else \
            [100000, 1000000, 10000000, 100000000, 1000000000]
        want = set(a.ops.split(","))
        for n in sizes:
            if n > a.max_elems:
                break
            if p > 1 and a.sweep_alloc == "memalloc":
                buf = comm.memAlloc(n, torch.float64)
                for s0 in range(0, n, 1 << 27):
                    buf[s0:s0 + (1 << 27)].normal_()
            else:
                buf = torch.randn(n, device="cuda", dtype=torch.float64)
            froms = CommUtils.createProcessArrayFroms(n, p)
            tos = CommUtils.createProcessArrayTos(n, p)
            counts = [t - f for f, t in zip(froms, tos)]
            fns = {
                "gather": lambda: comm.gatherArray(buf, D, froms, tos, 0),
                "scatter": lambda: comm.scatterArray(buf, D, froms, tos, 0),
                "allgather": lambda: comm.allgatherArray(buf, D, froms, tos),
                "reduce_scatter": lambda: comm.reduceScatterArray(buf, D, Operators.Double.SUM, 0, counts),
                "broadcast": lambda: comm.broadcastArray(buf, D, 0, n, 0),
                "reduce": lambda: comm.reduceArray(buf, D, Operators.Double.SUM, 0, n, 0),
                "allreduce": lambda: comm.allreduceArray(buf, D, Operators.Double.SUM, 0, n),
            }
            for k, op in enumerate(OPS):
                if op not in want:
                    continue
                st0 = dict(eng.stats) if eng is not None else {}
                p50, p99 = timed(fns[op], a.iters, a.warmup, sync)
                nb = n * 8
                algbw = nb / (p50 * 1e-3) / 1e9
                ref = REF_MS.get(p, {}).get(n)
                rec = {"op": op, "p": p, "elements": n, "bytes": nb, "p50_ms": round(p50, 4), "p99_ms": round(p99, 4),
                       "algbw_GBps": round(algbw, 3), "busbw_GBps": round(algbw * busfactor(op, p), 3),
                       "ref_ms_1GbE": ref[k] if ref else None,
                       "speedup_vs_ref": round(ref[k] / p50, 1) if ref else None}
                if eng is not None:
                    rec["path"] = sorted(x for x, v in eng.stats.items() if v != st0.get(x, 0))
                if a.check:
                    rec["exact"] = check_op(op, buf, comm, D, froms, tos, counts, p, r, sync)
                if p > 1 and a.sweep_alloc == "memalloc":
                    rec["alloc"] = "memalloc"
                emit(rec)
            if p > 1 and a.sweep_alloc == "memalloc":
                comm.memFree(buf)
            del buf
    if a.config == "zero_bf16":   # BASELINE config 3: RS + AG of a 4 GB bf16 tensor
        n = 2_000_000_000 // p * p
        # memAlloc (default for p > 1): mapped into every peer at any size, so RS and AG run the
        # zero-copy kernels on it (a 4 GB caching-allocator tensor cannot be mapped: staged pieces)
        x = comm.memAlloc(n, torch.bfloat16) if (p > 1 and a.alloc == "memalloc") else \
            torch.empty(n, device="cuda", dtype=torch.bfloat16)
        CH0 = 1 << 28
        for s0 in range(0, n, CH0):
            x[s0:s0 + CH0] = torch.randn(min(CH0, n - s0), device="cuda").to(torch.bfloat16)
        B = Operands.BF16_OPERAND()
        counts = [n // p] * p
        froms = CommUtils.getFromsFromCount(0, counts, p)
        tos = CommUtils.getTosFromCount(0, counts, p)

        def step():
            comm.reduceScatterArray(x, B, Operators.BFloat16.SUM, 0, counts)
            comm.allgatherArray(x, B, froms, tos)
        tuned = None
        if p > 1 and a.alloc != "memalloc":
            # untimed: RCCL vs piecewise IPC vs a2a / p2p, pinned per size class (MAX over ranks);
            # a memAlloc tensor always takes the zero-copy kernels, so nothing to pin there
            tuned = {"reduce_scatter": eng.autotune_reduce_scatter(x, Operators.BFloat16.SUM, iters=2),
                     "allgather": eng.autotune_allgather(x, iters=2)}
            tuned = {k: {c: round(t * 1e3, 3) for c, t in v.items()} for k, v in tuned.items()}
        p50, p99 = timed(step, a.iters, a.warmup, sync)
        nb = n * 2
        rec = {"config": "reduceScatter + allgather of 4 GB bf16 (ZeRO)", "p": p, "p50_ms": p50, "p99_ms": p99,
               "alloc": a.alloc if p > 1 else "plain", "path": sorted(k for k in eng.stats) if eng is not None else None,
               "busbw_GBps": round(nb / (p50 * 1e-3) / 1e9 * 2 * (p - 1) / p, 3) if p > 1 else None,
               "autotune_ms": tuned}
        if a.check:     # (i % 13 + rank) per rank: the RS + AG result is exact in bf16
            CH = 1 << 28
            for s0 in range(0, n, CH):
                i = torch.arange(s0, min(n, s0 + CH), device="cuda")
                x[s0:s0 + CH] = (i % 13 + r).to(torch.bfloat16)
            step()
            sync()
            ok = True
            for s0 in range(0, n, CH):
                i = torch.arange(s0, min(n, s0 + CH), device="cuda")
                ok &= bool(torch.equal(x[s0:s0 + CH], (p * (i % 13) + p * (p - 1) // 2).to(torch.bfloat16)))
            rec["exact"] = bool(ok)
        emit(rec)
    if a.config == "sparse_map":  # BASELINE config 4: sparse Map<String, float[]> allreduce
        dim, nkeys = 64, 200_000
        shared = nkeys // 2
        ids = torch.cat([torch.arange(shared), 10_000_000 + r * nkeys + torch.arange(nkeys - shared)]).cuda()
        vals = torch.randn(nkeys, dim, device="cuda")
        fn = (lambda: comm.allreduceSparse(ids, vals, Operators.Float.SUM)) if p > 1 else (lambda: None)
        p50, p99 = timed(fn, a.iters, a.warmup, sync)
        m = {f"feat{i}": vals[i] for i in range(2000)}
        t0 = time.perf_counter()
        if p > 1:
            comm.allreduceMap(m, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
        t_map = time.perf_counter() - t0
        emit({"config": "sparse allreduce, 200k keys x float[64] per rank (50% shared)", "p": p,
              "p50_ms": p50, "p99_ms": p99, "map_api_2000_keys_ms": t_map * 1e3})
    if a.config in ("fp8_8gb", "allreduce_1gb"):   # BASELINE configs 5 / 2
        nbytes = 8_000_000_000 if a.config == "fp8_8gb" else 1_000_000_000
        n = nbytes // 4
        CH = 1 << 27

        def fill(dst, rank):      # chunk c of rank j from seed (j, c): any rank can regenerate it
            for c, s0 in enumerate(range(0, n, CH)):
                g = torch.Generator(device="cuda").manual_seed(rank * 100003 + c)
                dst[s0:s0 + CH] = torch.randn(min(CH, n - s0), device="cuda", generator=g)
        x = torch.empty(n, device="cuda")
        fill(x, r)
        codecs = [None if c == "none" else c for c in a.codecs.split(",")] if a.config == "fp8_8gb" else [None]
        for codec in codecs:
            F = Operands.FLOAT_OPERAND(codec=codec)
            p50, p99 = timed(lambda: comm.allreduceArray(x, F, Operators.Float.SUM, 0, n), a.iters, a.warmup, sync)
            rec = {"config": f"allreduce {nbytes/1e9:.0f} GB f32", "codec": codec or "none", "p": p,
                   "p50_ms": p50, "p99_ms": p99,
                   "busbw_GBps": round(nbytes / (p50 * 1e-3) / 1e9 * 2 * (p - 1) / p, 3) if p > 1 else None}
            if a.check:       # one call on fresh data against the fp64 sum of every rank's input
                fill(x, r)
                comm.allreduceArray(x, F, Operators.Float.SUM, 0, n)
                sync()
                num = den = 0.0
                worst = 0.0
                for c, s0 in enumerate(range(0, n, CH)):
                    m = min(CH, n - s0)
                    ref = torch.zeros(m, dtype=torch.float64, device="cuda")
                    for j in range(p):
                        g = torch.Generator(device="cuda").manual_seed(j * 100003 + c)
                        ref += torch.randn(m, device="cuda", generator=g).double()
                    d = x[s0:s0 + m].double() - ref
                    num += float((d * d).sum())
                    den += float((ref * ref).sum())
                    worst = max(worst, float(d.abs().max()))
                rel = (num / max(den, 1e-300)) ** 0.5
                rec["rel_l2_error_vs_fp64"] = rel
                rec["max_abs_error"] = worst
                rec["exact"] = rel < (0.1 if codec == "fp8" else 1e-6)
            emit(rec)
    if eng is not None and r == 0:
        # the IPC instances' co-residency grid caps (shared GPU: derived per kernel from occupancy)
        caps = {name: inst.grid_caps_summary() for name, inst in
                (("default", eng._ipc_obj), ("large", eng._ipc_large), ("fp8", eng._ipc_fp8_big)) if inst is not None}
        emit({"ipc_grid_caps": caps, "share": getattr(eng._ipc_obj, "share", None)})
    comm.close(0)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
