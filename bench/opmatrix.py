#!/usr/bin/env python3
"""Per-call latency of the whole operator table on the xGMI kernels.

    torchrun --nproc-per-node P --master-addr 127.0.0.1 bench/opmatrix.py [--sizes ...]

For every (dtype, op) pair of the reference's ``Operators`` table (+ bf16 / f16) and each size,
``allreduceArray`` at the default selection (no forcing): W warm-up calls, then K calls with a
hipEvent pair around each (p50 / p99, MAX over ranks), one exact check, and the schedule the
engine took (call counters).  The hot pairs (SUM, float MAX / MIN) run compile-time-op kernels,
every other pair the runtime-op kernel of its dtype — same bytes moved, so the two should time
alike at equal size.  With ``MP4X_DEVICE_BACKEND=gloo`` several ranks can share one GPU (the
IPC kernels run for real, no RCCL)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PAIRS = [("Float", "float32", "SUM"), ("Float", "float32", "PROD"), ("Float", "float32", "MAX"),
         ("Double", "float64", "SUM"), ("Double", "float64", "MAX"), ("Double", "float64", "FLOAT_MAX_LOC"),
         ("Long", "int64", "SUM"), ("Long", "int64", "BITS_OR"), ("Long", "int64", "INT_MIN_LOC"),
         ("Int", "int32", "SUM"), ("Int", "int32", "BITS_XOR"), ("Short", "int16", "SUM"), ("Short", "int16", "MAX"),
         ("Byte", "int8", "SUM"), ("Byte", "int8", "BITS_AND"), ("BFloat16", "bfloat16", "SUM"),
         ("BFloat16", "bfloat16", "PROD")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="65536,4194304,67108864")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", default="", help="comma list of Class.OP to keep (default: all)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    from mp4x import Operands, Operators
    from mp4x.launch import init_from_env
    local = int(os.environ.get("MP4X_DEVICE_INDEX", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    comm = init_from_env(heartbeat=False)
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    keep = {x.strip() for x in a.pairs.split(",") if x.strip()}
    agree_dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    for cls, dtn, opn in PAIRS:
        if keep and f"{cls}.{opn}" not in keep:
            continue
        dt = getattr(torch, dtn)
        op = getattr(getattr(Operators, cls), opn)
        es = torch.empty((), dtype=dt).element_size()
        for nb in [int(x) for x in a.sizes.split(",")]:
            n = nb // es
            g = torch.Generator(device="cuda").manual_seed(11 + r)
            if dt.is_floating_point:
                x = torch.randint(-4, 5, (n,), device="cuda", generator=g).to(dt)
            else:
                x = torch.randint(-100, 100, (n,), device="cuda", generator=g).to(dt)
            before = dict(eng.stats)
            for _ in range(a.warmup):
                comm.allreduceArray(x.clone(), Operands.DOUBLE_OPERAND(), op, 0, n)
            buf = x.clone()
            st = [torch.cuda.Event(enable_timing=True) for _ in range(a.iters)]
            en = [torch.cuda.Event(enable_timing=True) for _ in range(a.iters)]
            torch.cuda.synchronize()
            comm.barrier()
            for i in range(a.iters):
                st[i].record()
                comm.allreduceArray(buf, Operands.DOUBLE_OPERAND(), op, 0, n)
                en[i].record()
            torch.cuda.synchronize()
            lat = sorted(s.elapsed_time(e) for s, e in zip(st, en))
            # exact check of one call against the host fold in rank order
            y = x.clone()
            comm.allreduceArray(y, Operands.DOUBLE_OPERAND(), op, 0, n)
            torch.cuda.synchronize()
            exp = None
            for j in range(p):
                gj = torch.Generator(device="cuda").manual_seed(11 + j)
                xj = (torch.randint(-4, 5, (n,), device="cuda", generator=gj).to(dt) if dt.is_floating_point else
                      torch.randint(-100, 100, (n,), device="cuda", generator=gj).to(dt))
                xj = xj.float().cpu().numpy() if dt == torch.bfloat16 else xj.cpu().numpy()
                if exp is None:
                    exp = xj.copy()
                else:
                    with np.errstate(over="ignore", invalid="ignore"):
                        op.reduce_into(exp, xj)
            got = y.float().cpu().numpy() if dt == torch.bfloat16 else y.cpu().numpy()
            exact = bool(np.array_equal(got.view(np.uint8), exp.view(np.uint8))) if dt != torch.bfloat16 \
                else bool(np.array_equal(got, exp))
            used = {k: c - before.get(k, 0) for k, c in eng.stats.items() if c != before.get(k, 0)}
            t = torch.tensor([lat[len(lat) // 2], lat[min(len(lat) - 1, int(0.99 * len(lat)))], 0.0 if exact else 1.0],
                             dtype=torch.float64, device=agree_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if r == 0:
                p50, p99, wrong = t.tolist()
                busbw = nb / (p50 * 1e-3) / 1e9 * 2 * (p - 1) / p
                print(json.dumps({"pair": f"{cls}.{opn}", "dtype": dtn, "bytes": nb, "p": p, "p50_ms": round(p50, 4),
                                  "p99_ms": round(p99, 4), "busbw_gbps": round(busbw, 2), "exact": wrong == 0,
                                  "calls": used}), flush=True)
    comm.close(0)


if __name__ == "__main__":
    main()
