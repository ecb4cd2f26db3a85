#!/usr/bin/env python3
"""K4b (csrc/kernels/sparse.hip) halves against the copy roofline: partition_count (histogram +
scan + counts) and partition_scatter (owner-sorted rows + keys), for config 4's rows per rank
(200 k x float[64]) and 8x that, at p = 2 and 8; ``clone`` = a plain device copy of the same
rows (the bandwidth ceiling for a pass that reads and writes every row once).  One JSON line per
case: p50 ms of device time (hipEvents).

    python bench/pack_ab.py [--iters 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--ns", default="200000,1600000")
    ap.add_argument("--ps", default="2,8")
    a = ap.parse_args()
    import torch
    from mp4x.ops import device_ops as K

    def t(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return round(sorted(ts)[len(ts) // 2], 4)

    g = torch.Generator(device="cuda").manual_seed(3)
    for n in [int(x) for x in a.ns.split(",")]:
        keys = torch.randint(0, 1 << 40, (n,), device="cuda", generator=g, dtype=torch.int64)
        vals = torch.randn(n, 64, device="cuda", generator=g)
        ok = torch.empty_like(keys)
        ov = torch.empty_like(vals)
        for p in [int(x) for x in a.ps.split(",")]:
            pc = K.partition_count(keys, p)
            rec = {"n": n, "p": p, "row_bytes": 256,
                   "count_ms": t(lambda: K.partition_count(keys, p)),
                   "scatter_ms": t(lambda: K.partition_scatter(pc, vals, ov.data_ptr(), ok.data_ptr())),
                   "fused_ms": t(lambda: K.partition_pack(keys, vals, p)),
                   "clone_ms": t(lambda: ov.copy_(vals))}
            moved = vals.numel() * 4 * 2 + keys.numel() * 8 * 2          # rows + keys, read + written
            rec["scatter_TBps"] = round(moved / (rec["scatter_ms"] * 1e-3) / 1e12, 2)
            rec["clone_TBps"] = round(vals.numel() * 8 / (rec["clone_ms"] * 1e-3) / 1e12, 2)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
