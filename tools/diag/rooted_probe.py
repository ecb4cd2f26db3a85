#!/usr/bin/env python3
"""Diagnose the rooted autotune probe at 1 MiB (broadcast / gather / scatter 'ipc' ruled out in
the 4-rank bench rehearsal): p ranks on one GPU, the agreement values of every probe recorded per
rank.  python tools/diag/rooted_probe.py [p]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def fn(comm, sizes, pre=""):
    import torch
    from mp4x import Operands, Operators
    eng = comm.device
    eng.ipc()
    op = Operators.Float.SUM
    if "head" in pre:            # bench.py's sequence before its rooted sweep
        n = 250_000_000
        buf = torch.randn(n, device="cuda")
        comm.registerBuffer(buf)
        if "tune1g" in pre:
            eng.autotune_allreduce(buf, op, iters=5)
        for _ in range(5):
            comm.allreduceArray(buf, Operands.FLOAT_OPERAND(), op, 0, n, scale=0.25)
        torch.cuda.synchronize()
    if "tiers" in pre:
        for nb in (65536, 4194304):
            eng.autotune_allreduce(torch.empty(nb // 4, device="cuda"), op, iters=3)
    log = []
    orig = eng._agree

    def agree(flags):
        out = orig(flags)
        log.append((list(flags), out))
        return out
    eng._agree = agree
    res = {}
    for nb in sizes:
        like = torch.empty(nb // 4, device="cuda")
        for kind in ("reduce", "broadcast", "gather", "scatter"):
            mark = len(log)
            from mp4x import Operators
            root = int(os.environ.get("DIAG_ROOT", comm.getSlaveNum() - 1))     # bench.py uses p - 1
            r = getattr(eng, "autotune_" + kind)(like, Operators.Float.SUM, root=root) if kind == "reduce" else \
                getattr(eng, "autotune_" + kind)(like, root=root)
            res[f"{nb}:{kind}"] = {"times": r, "agree": log[mark:]}
    return res


if __name__ == "__main__":
    from spawn_ranks import run_spawn
    p = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    pre = sys.argv[2] if len(sys.argv) > 2 else ""
    out = run_spawn(p, fn, args=([1 << 20, 16 << 20], pre), timeout=300)
    for r in sorted(out):
        print(json.dumps({"rank": r, "res": out[r]}, default=str))
