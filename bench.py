#!/usr/bin/env python3
"""Headline benchmark: allreduce bus bandwidth + p50 latency, 1 GB float[] (BASELINE.json).

``python bench.py --gpus N --steps K --warmup W`` — for N>1 the driver launches one rank
per GPU with ``torch.distributed.run``.  Every step is ONE public-API call

    comm.allreduceArray(buf, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, n)

on a 1e9-byte float32 array (250,000,000 elements, synthetic random data) resident on the
rank's MI355X, i.e. the reference's ``ProcessCommSlave.allreduceArray`` on the BASELINE
config.  For N>1 the warm-up first autotunes the schedule (RCCL, IPC two-shot over xGMI,
a2a two-shot; MAX time over ranks, on a scratch tensor).  Timing: W untimed warmup calls,
barrier + device sync, K timed calls with a hipEvent pair around each (p50 / p99),
barrier + sync; MAX over ranks.

busbw follows the nccl-tests convention used in BASELINE.md: algbw = bytes / t,
busbw = algbw * 2(p-1)/p, and ``value`` IS that busbw (per rank, the BASELINE metric; the
whole-job sum ``N * busbw`` is reported separately as ``aggregate_busbw_gbps``).
With one rank nothing crosses a link (factor 2(p-1)/p = 0) and the in-place call is a
no-op by the reference's contract, so N=1 times the OUT-OF-PLACE form of the same call
(``out=``; a 1 GB device copy through the K1 kernel) and reports algbw for it — HBM
evidence, not an allreduce number.

For N>1 the buffer is registered with the communicator (``registerBuffer``, collective), so
the zero-copy two-shot can run straight on the peers' tensors; the autotune times it next to
RCCL and the staged kernels (bounded per candidate, ``MP4X_AUTOTUNE_CAP_S``) and only ever
pins a schedule that was exact on every rank; if every custom schedule fails, RCCL stays.
Before any IPC tier is used, a collective self-test of the IPC mesh runs (``ipc_selftest``).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# reference busbw (MB/s) for ~1 GB allreduce, BASELINE.md section D (mean of 1e8 and 5e8 rows)
REF_BUSBW_MBPS = {2: 85.2, 4: 92.1, 6: 86.8, 8: 88.0}
METRIC = "allreduce bus bandwidth (GB/s) + p50 latency, 1 GB float[], 1/2/4/8 MI355X"


class _CpuEvent:
    """time.perf_counter stand-in for torch.cuda.Event in the --cpu dry run."""

    def __init__(self, enable_timing=True):
        self.t = 0.0

    def record(self, *a):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bytes", type=int, default=1_000_000_000)
    ap.add_argument("--algo", default=None, help="force device algorithm: rccl | a2a")
    ap.add_argument("--codec", default=None, help="wire codec for the fp8-compressed config: fp8")
    ap.add_argument("--cpu", action="store_true", help="dry run of the launch/rendezvous path on CPU (gloo)")
    ap.add_argument("--no-autotune", action="store_true",
                    help="skip the warm-up schedule autotune (RCCL vs IPC two-shot vs a2a) for N>1")
    ap.add_argument("--no-register", action="store_true",
                    help="do not register the buffer for the zero-copy IPC two-shot")
    ap.add_argument("--no-tier-sweep", action="store_true",
                    help="N>1: skip the untimed per-size schedule sweep (4 KiB .. 64 MiB) run after the timed steps")
    args = ap.parse_args()
    if args.algo:
        os.environ["MP4X_DEVICE_ALGO"] = args.algo

    import torch
    import torch.distributed as dist
    from mp4x import Operands, Operators
    from mp4x.launch import init_from_env

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("MP4X_DEVICE_INDEX", os.environ.get("LOCAL_RANK", "0")))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if args.cpu:
        dev = torch.device("cpu")
        torch.cuda.synchronize = lambda *a, **k: None
        torch.cuda.Event = _CpuEvent
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)

    comm = init_from_env(heartbeat=False)
    p = comm.getSlaveNum()
    n = args.bytes // 4
    operand = Operands.FLOAT_OPERAND(codec=args.codec)
    op = Operators.Float.SUM

    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    buf = torch.randn(n, device=dev, dtype=torch.float32, generator=g)
    out = torch.empty_like(buf) if p == 1 else None

    def step():
        if p == 1:
            comm.allreduceArray(buf, operand, op, 0, n, out=out)
        else:
            comm.allreduceArray(buf, operand, op, 0, n)

    def sync_all():
        torch.cuda.synchronize()
        if p > 1:
            comm.peer_barrier() if args.cpu else comm.device.barrier()
            torch.cuda.synchronize()

    tuned = None
    registered = False
    if p > 1 and not args.cpu:
        comm.device  # bring up the RCCL communicator before timing
        if not args.no_register:
            registered = comm.registerBuffer(buf)   # collective; False on every rank alike
        if not (args.no_autotune or args.algo or args.codec):
            # untimed: measure every applicable schedule on a scratch tensor of this shape and
            # pin the fastest (all ranks agree: MAX over ranks); the timed steps run it in full
            tuned = {k: round(v * 1e3, 3) for k, v in
                     comm.device.autotune_allreduce(buf, op, iters=2).items()}
    for _ in range(args.warmup):
        step()
    sync_all()

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record()
        step()
        ends[i].record()
    sync_all()
    wall = time.perf_counter() - t0
    lat = sorted(s.elapsed_time(e) for s, e in zip(starts, ends))   # ms

    # MAX over ranks
    vals = torch.tensor([wall, lat[len(lat) // 2], lat[min(len(lat) - 1, int(0.99 * len(lat)))]],
                        dtype=torch.float64, device=dev)
    if p > 1:
        if args.cpu:
            vals = torch.from_numpy(comm.allreduceArray(vals.numpy(), Operands.DOUBLE_OPERAND(),
                                                        Operators.Double.MAX, 0, 3))
        else:
            dist.all_reduce(vals, op=dist.ReduceOp.MAX)
    wall, p50, p99 = vals.tolist()

    # after the timed steps (never inside them): measure every schedule at the size classes
    # the IPC tiers are chosen for, so a multi-GPU run records the tier boundaries on real links
    tiers = None
    if p > 1 and not args.cpu and not args.no_tier_sweep and not (args.algo or args.codec):
        tiers = {}
        for nb in (4 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
            failed = 0.0
            try:
                res = comm.device.autotune_allreduce(torch.empty(nb // 4, device=dev), op, iters=3)
                tiers[str(nb)] = {k: (round(v * 1e3, 4) if v != float("inf") else None) for k, v in res.items()}
            except Exception as e:   # noqa: BLE001 — evidence only; the headline is already measured
                tiers[str(nb)] = {"error": str(e)[:200]}
                failed = 1.0
            # every rank stops together (a rank-local failure must not leave the others waiting
            # in the next size's collectives)
            flag = torch.tensor([failed], dtype=torch.float64, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            if flag.item() > 0:
                break

    ms_per_step = wall * 1e3 / args.steps
    nbytes = n * 4
    algbw = nbytes / (ms_per_step * 1e-3) / 1e9
    factor = 2.0 * (p - 1) / p if p > 1 else 1.0
    busbw = algbw * factor
    ref = REF_BUSBW_MBPS.get(p)
    algo = "k1_copy (out-of-place, 1 rank)" if p == 1 else ("host-tcp" if args.cpu else
                                  comm.device.select("allreduce", nbytes, Operators.Float.SUM, torch.float32, operand))
    if algo == "ipc2" and registered and not args.cpu and not comm.device._select_tuned:
        algo = "ipc2z"
    selftest = None if (p == 1 or args.cpu) else comm.device.ipc_selftest
    stats = None if (p == 1 or args.cpu) else {k: v for k, v in comm.device.stats.items() if k.startswith("allreduce")}
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(busbw, 3),
            "unit": "GB/s",
            "n_gpus": p,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(busbw / (ref / 1e3), 2) if ref else None,
            "dtype": "fp32",
            "data": "synthetic (torch.randn per rank)",
            "config": {"model": f"allreduceArray float[{n}] ({nbytes / 1e9:g} GB), Operators.Float.SUM",
                       "global_batch": p, "seq_len": n, "parallelism": f"dp{p}",
                       "payload_bytes": nbytes, "algo": algo, "registered": registered,
                       "in_place": p > 1, "autotune_ms": tuned, "ipc_selftest": selftest,
                       "calls": stats, "tier_sweep_ms": tiers},
            "busbw_gbps_per_rank": round(busbw, 3),
            "aggregate_busbw_gbps": round(busbw * p, 3),
            "algbw_gbps": round(algbw, 3),
            "p50_ms": round(p50, 4),
            "p99_ms": round(p99, 4),
            "busbw_factor": factor,
            "note": ("p=1: nothing crosses a link (nccl-tests busbw factor 2(p-1)/p = 0), so this is "
                     "busbw := algbw of the out-of-place single-rank allreduce, a 1 GB HBM copy through K1; "
                     "N>=2 values are xGMI-link-bound and not comparable to N=1 as a scaling base"
                     if p == 1 else "value = busbw = algbw * 2(p-1)/p (nccl-tests convention, per rank); "
                                    "aggregate_busbw_gbps = p * busbw"),
        }
        print(json.dumps(rec), flush=True)
    comm.close(0)
    if p > 1 and dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
