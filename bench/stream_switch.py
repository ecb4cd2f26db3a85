#!/usr/bin/env python3
"""What a cross-stream dependency costs on this GPU, without mp4x: one process, a tiny kernel
(``x.add_(1)``) issued (a) on one stream, (b) alternating between two streams with the join the
stream-order guard makes (event on the previous stream, the next stream waits for it), (c)
alternating with no join, then (a) again — µs per op, host clock around K ops + one sync.

    python bench/stream_switch.py [--iters 2000]
"""
import argparse
import json
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    a = ap.parse_args()
    import torch
    x = torch.zeros(1024, device="cuda")
    s = [torch.cuda.Stream(), torch.cuda.Stream()]
    ev = torch.cuda.Event()

    def run(name, step):
        for i in range(50):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.iters):
            step(i)
        torch.cuda.synchronize()
        return name, round((time.perf_counter() - t0) / a.iters * 1e6, 2)

    def same(i):
        x.add_(1)

    def joined(i):
        cur, prev = s[i & 1], s[(i + 1) & 1]
        ev.record(prev)
        cur.wait_event(ev)
        with torch.cuda.stream(cur):
            x.add_(1)

    def unjoined(i):
        with torch.cuda.stream(s[i & 1]):
            x.add_(1)

    def ctx_same(i):
        with torch.cuda.stream(s[0]):
            x.add_(1)
    out = dict([run("default_stream", same), run("stream_ctx_same", ctx_same), run("alternating_joined", joined),
                run("alternating_unjoined", unjoined), run("default_stream_after", same)])
    print(json.dumps({"us_per_op": out, "join_cost_us": round(out["alternating_joined"] - out["stream_ctx_same"], 2)}))


if __name__ == "__main__":
    main()
