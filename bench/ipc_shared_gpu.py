#!/usr/bin/env python3
"""Latency / throughput of the custom IPC allreduce protocol with p processes sharing GPU 0.

This is the single-GPU rehearsal of csrc/runtime/ipc.hip: every peer buffer is an IPC
mapping of memory on the same MI355X, so the numbers measure the protocol (epoch flags,
per-block barriers, kernel launch, uncached buffer traffic) — not xGMI bandwidth.
Prints one JSON line per (size, algo).
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(port, q, sizes, iters, buf_bytes=64 << 20, algos=(0, 1)):
    import torch
    from mp4x import ProcessCommSlave, Operators
    from mp4x.parallel.ipc import IpcAllreduce
    torch.cuda.set_device(0)
    comm = ProcessCommSlave("b", "127.0.0.1", port, heartbeat=False)
    ipc = IpcAllreduce(comm, nbytes=buf_bytes).prepare_graph()
    out = []
    for nbytes in sizes:
        x = torch.randn(nbytes // 4, device="cuda")
        for algo in algos:
            def call():
                if algo == 2:
                    ipc.allreduce_fp8(x)      # fused fp8 two-shot (K6 codec on the links)
                else:
                    ipc.allreduce(x, Operators.Float.SUM, algo=algo)
            for _ in range(5):
                call()
            torch.cuda.synchronize()
            comm.barrier()
            s = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
            e = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
            for i in range(iters):
                s[i].record()
                call()
                e[i].record()
            torch.cuda.synchronize()
            ts = sorted(a.elapsed_time(b) for a, b in zip(s, e))
            # same call captured in a hipGraph (launch overhead removed)
            gs = torch.cuda.Stream()
            gs.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=gs):
                call()
            torch.cuda.synchronize()
            comm.barrier()
            for i in range(iters):
                s[i].record()
                g.replay()
                e[i].record()
            torch.cuda.synchronize()
            tg = sorted(a.elapsed_time(b) for a, b in zip(s, e))
            out.append({"bytes": nbytes, "algo": ["oneshot", "twoshot", "fp8_twoshot"][algo], "p50_us": ts[len(ts) // 2] * 1e3,
                        "p99_us": ts[min(len(ts) - 1, int(0.99 * len(ts)))] * 1e3,
                        "graph_p50_us": tg[len(tg) // 2] * 1e3, "err": ipc.error_word()})
            comm.barrier()
    ipc.close()
    comm.close(0)
    q.put((comm.getRank(), out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--sizes", default="4096,65536,262144,1048576,8388608,33554432", help="message bytes, comma list")
    ap.add_argument("--buf-mib", type=int, default=64, help="IPC buffer size (larger messages go in pieces)")
    ap.add_argument("--algos", default="0,1", help="0 = one-shot, 1 = two-shot, 2 = fused fp8 two-shot")
    a = ap.parse_args()
    from mp4x import CommMaster
    m = CommMaster(a.procs, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    sizes = [int(x) for x in a.sizes.split(",")]
    algos = tuple(int(x) for x in a.algos.split(","))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(m.port, q, sizes, a.iters, a.buf_mib << 20, algos)) for _ in range(a.procs)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=600) for _ in range(a.procs))
    [p.join(timeout=30) for p in ps]
    m.stop(timeout=5)
    for row0 in res[0]:
        worst = max(r for r in (next(x for x in res[k] if x["bytes"] == row0["bytes"] and x["algo"] == row0["algo"])
                                for k in res) for r in [r["p50_us"]])
        print(json.dumps({"procs_on_one_gpu": a.procs, **row0, "p50_us_max_rank": worst}))


if __name__ == "__main__":
    main()
