#!/usr/bin/env python3
"""Diagnose memAlloc -> memFree -> memAlloc (p ranks on one GPU): per rank, the VAs of every
allocation (own + imported peers), the tensor's content right before the allreduce, the result,
and the same after a system-scope release on every XCD (mp4x_release_all) — to tell a stale
mapping of a reused VA from unflushed cache lines.  Prints one line per rank and step.

  MP4X_VMM_CHUNK=8388608 python tools/vmm_realloc_probe.py [--p 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def body(comm, sizes):
    import torch
    from mp4x import Operands, Operators
    from mp4x.ops import native
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    lines = []
    for step, n in enumerate(sizes):
        t = comm.memAlloc(n, torch.float32)
        reg = eng._ipc_obj._find(t)[0]
        vas = [hex(v.va) for v in reg.vmm]
        handles = [hex(v._handles[0]) for v in reg.vmm[:2]]
        i = torch.arange(n, device="cuda", dtype=torch.int32) % 11
        exp = (i * p + p * (p - 1) // 2).float()
        for mode in ("plain", "release"):
            t.copy_(i + r)
            torch.cuda.synchronize()
            pre_ok = bool(torch.equal(t, (i + r).float()))
            if mode == "release":
                native.check(native.hip().mp4x_release_all(native.stream_ptr()), "release_all")
                torch.cuda.synchronize()
            comm.barrier()
            comm.allreduceArray(t, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, n)
            torch.cuda.synchronize()
            nbad = int((t != exp).sum())
            sample = t[:4].tolist()
            lines.append(f"r{r} step{step} n={n} {mode}: own handles={handles} vas={vas} pre_ok={pre_ok} wrong={nbad} head={sample} "
                         f"exp_head={exp[:4].tolist()} err={eng._ipc_obj.host_error()}")
        comm.memFree(t)
    return lines


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, default=3)
    ap.add_argument("--sizes", default="10485776,1048576,1048576")
    a = ap.parse_args()
    from spawn_ranks import run_spawn
    sizes = [int(x) for x in a.sizes.split(",")]
    out = run_spawn(a.p, body, args=(sizes,), timeout=180)
    for r in sorted(out):
        for ln in out[r]:
            print(ln, flush=True)


if __name__ == "__main__":
    main()
