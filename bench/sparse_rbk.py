#!/usr/bin/env python3
"""A/B of the sparse reduce-by-key (K5): the deterministic sort path (rocPRIM radix sort + run
starts + segmented reduce, csrc/kernels/sparse.hip) vs the hash path (K5h, open addressing +
row lists, csrc/kernels/sparse_hash.hip) and the dense path (K5d, direct addressing) on BASELINE
config 4's shape: the rows one owner receives at p ranks (200k keys x float[64] per rank, half
shared).  ``--dense-ids``: the keys are dictionary ids (the map API's numbering: the shared keys
0..99999, then every rank's own keys), so the sort runs over their bit width and K5d applies.  One JSON line per (p, path):
p50 ms over --iters calls (hipEvents around each), exactness against the other path.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ps", default="2,8")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--paths", default="sort,hash", help="sort, hash, dense (with --dense-ids)")
    ap.add_argument("--dense-ids", action="store_true")
    args = ap.parse_args()
    import torch
    from mp4x.ops.device_ops import dense_reduce_by_key, hash_reduce_by_key, reduce_by_key
    for p in [int(x) for x in args.ps.split(",")]:
        nkeys, shared = 200_000, 100_000
        ks, vs = [], []
        for r in range(p):
            own0 = shared + r * (nkeys - shared) if args.dense_ids else 10_000_000 + r * nkeys
            ids = torch.cat([torch.arange(shared), own0 + torch.arange(nkeys - shared)])
            ids = ids[ids % p == 0]
            ks.append(ids)
            vs.append(((ids.view(-1, 1) * 7 + torch.arange(args.dim) + r) % 23 - 11).float())
        keys, rows = torch.cat(ks).cuda(), torch.cat(vs).cuda()
        res = {}
        for path in args.paths.split(","):
            bits = int(keys.max()).bit_length() if args.dense_ids else None
            base, T = int(keys.min()) // p, int(keys.max()) // p - int(keys.min()) // p + 1
            fn = {"sort": lambda: reduce_by_key(keys, rows, 0, key_bits=bits),
                  "hash": lambda: hash_reduce_by_key(keys, rows, 0),
                  "dense": lambda: dense_reduce_by_key(keys, rows, 0, base, p, T)}[path]
            for _ in range(5):
                out = fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.iters):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                out = fn()
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b))
            ts.sort()
            k, v, c = out
            o = torch.argsort(k)
            res[path] = (k[o], v[o], c[o])
            print(json.dumps({"p": p, "path": path, "rows": keys.numel(), "unique": int(k.numel()), "dim": args.dim,
                              "p50_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4),
                              "row_bytes_in": keys.numel() * args.dim * 4}), flush=True)
        if len(res) >= 2:
            (k1, v1, c1), *rest = res.values()
            print(json.dumps({"p": p, "exact": all(bool(torch.equal(k1, k2) and torch.equal(v1, v2) and
                                                        torch.equal(c1, c2)) for k2, v2, c2 in rest)}), flush=True)


if __name__ == "__main__":
    main()
