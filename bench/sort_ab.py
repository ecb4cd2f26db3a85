#!/usr/bin/env python3
"""A/B of the reduce-by-key's key sort (csrc/kernels/sparse.hip): rocPRIM's own dispatch (block
sort + merge passes below 1 M items) vs forced onesweep (one pass per 8 key bits), int64 keys
with an int64 index payload, by item count and key width.  One JSON line per case (p50 ms of
device time over --iters calls, hipEvent-timed).

    python bench/sort_ab.py [--ns 200000,1000000] [--bits 16,24,32,40,64] [--iters 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="200000,1000000")
    ap.add_argument("--bits", default="16,24,32,40,64")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import torch
    from mp4x.ops import device_ops as K
    g = torch.Generator(device="cuda").manual_seed(1)
    for n in [int(x) for x in a.ns.split(",")]:
        for b in [int(x) for x in a.bits.split(",")]:
            hi = (1 << b) if b < 63 else (1 << 62)
            keys = torch.randint(0, hi, (n,), device="cuda", generator=g, dtype=torch.int64)
            res = {}
            outs = {}
            for algo in (0, 1):
                for _ in range(3):
                    outs[algo] = K.sort_pairs(keys, end_bit=min(b, 64), algo=algo)
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.iters):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    K.sort_pairs(keys, end_bit=min(b, 64), algo=algo)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                res["rocprim_ms" if algo == 0 else "onesweep_ms"] = round(sorted(ts)[len(ts) // 2], 4)
            same = all(torch.equal(x, y) for x, y in zip(outs[0], outs[1]))
            print(json.dumps({"n": n, "bits": b, **res, "identical": same}), flush=True)


if __name__ == "__main__":
    main()
