#!/usr/bin/env python3
"""Where the host time of a small device allreduce goes: p processes on GPU 0, the same 4 KiB
f32 SUM issued through each layer in turn (public API with its native latency fast path ->
the public API's full Python path -> DeviceEngine -> IpcAllreduce -> the bare ctypes launch),
wall time per call (MAX over ranks).  Also the public call inside a stream context, on one
stream or alternating between two: the difference is the cost of the communicator's
stream-order join (an event on the previous stream, a wait on the new one).  Rehearsal numbers: protocol
and host overhead, not xGMI latency.

    python bench/latency_layers.py --procs 2 --iters 3000 [--bytes 4096]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(port, q, nbytes, iters):
    import torch
    from mp4x import Operands, Operators, ProcessCommSlave
    from mp4x.operators import DType, for_dtype
    torch.cuda.set_device(0)
    os.environ.setdefault("MP4X_DEVICE_INDEX", "0")
    comm = ProcessCommSlave("b", "127.0.0.1", port, heartbeat=False)
    eng = comm.device
    x = torch.randn(nbytes // 4, device="cuda")
    n = x.numel()
    opnd, op = Operands.FLOAT_OPERAND(), Operators.Float.SUM
    fop = for_dtype(op, DType.F32)
    inst = eng.ipc()
    from mp4x.parallel import ipc as ipcm
    lib = inst.lib
    st = ipcm.stream_ptr()
    dt = int(ipcm.dtype_of_torch(x.dtype))

    def raw():
        inst.epoch = (inst.epoch + 1) & 0x3FFFFFFF or 1
        lib.mp4x_ipc_allreduce_ex(ipcm.ONESHOT, dt, int(fop.code), inst._pp_data[0], inst._pp_sig[0], inst.rank,
                                  inst.p, nbytes, x.data_ptr(), x.data_ptr(), inst.epoch, 8 if inst.shared_gpu else 0,
                                  None, 1.0, st)
    fast_memo = comm._fast_ar

    def api_full():            # the public call with the latency fast path disarmed
        comm._fast_ar = None
        try:
            comm.allreduceArray(x, opnd, op, 0, n)
        finally:
            comm._fast_ar = fast_memo
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    flip = [0]

    def api_stream(alternate):
        # the public call inside a stream context: the same stream every call, or alternating
        # between two (every call then joins the other stream: the stream-order guard's switch)
        def fn():
            i = flip[0] = flip[0] + 1 if alternate else 0
            with torch.cuda.stream(streams[i & 1]):
                comm.allreduceArray(x, opnd, op, 0, n)
        return fn
    layers = {"api": lambda: comm.allreduceArray(x, opnd, op, 0, n),
              "api_full_path": api_full,
              "engine": lambda: eng.allreduce(x, 0, n, op, opnd),
              "ipc": lambda: inst.allreduce(x, fop, algo=ipcm.ONESHOT),
              "raw_launch": raw,
              # last: work on two more streams changes how this process's launches are scheduled
              # from then on (bench/stream_switch.py)
              "api_stream_ctx_same": api_stream(False),
              "api_stream_ctx_alternating": api_stream(True),
              "api_after_streams": lambda: comm.allreduceArray(x, opnd, op, 0, n)}
    out = {}
    for name, fn in layers.items():
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        eng.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) / iters * 1e6
        eng.barrier()
    comm.close(0)
    q.put((comm.getRank(), out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--iters", type=int, default=3000)
    ap.add_argument("--bytes", type=int, default=4096)
    a = ap.parse_args()
    os.environ.setdefault("MP4X_DEVICE_BACKEND", "gloo")
    from mp4x import CommMaster
    m = CommMaster(a.procs, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(m.port, q, a.bytes, a.iters)) for _ in range(a.procs)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=600) for _ in range(a.procs))
    [p.join(timeout=30) for p in ps]
    m.stop(timeout=5)
    us = {k: round(max(res[r][k] for r in res), 2) for k in res[0]}
    print(json.dumps({"procs_on_one_gpu": a.procs, "bytes": a.bytes, "watchdog": os.environ.get("MP4X_WATCHDOG", "1"),
                      "us_per_call_max_rank": us, "api_minus_raw_launch_us": round(us["api"] - us["raw_launch"], 2),
                      "stream_switch_us": round(us["api_stream_ctx_alternating"] - us["api_stream_ctx_same"], 2)}))


if __name__ == "__main__":
    main()
