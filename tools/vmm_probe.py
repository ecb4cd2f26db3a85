#!/usr/bin/env python3
"""Step-by-step probe of the memAlloc primitives (csrc/runtime/vmm.hip, mp4x/parallel/vmm.py)
with 2 processes on one GPU: create -> tensor view -> fill -> fd exchange -> import -> peer
read -> free, for growing sizes.  Every step is logged with a timestamp (stdout, flushed) so a
hang names its step; each rank dumps its Python stack after ``--stuck`` seconds.

  python tools/vmm_probe.py [--sizes 64M:1,8M:4,512M:5] [--stuck 60]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _sz(s):
    m = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(s[:-1]) * m[s[-1]] if s[-1] in m else int(s)


def rank_main(port, plan, stuck):
    import faulthandler
    faulthandler.dump_traceback_later(stuck, exit=True)
    t0 = time.perf_counter()
    from mp4x import ProcessCommSlave
    comm = ProcessCommSlave("probe", "127.0.0.1", port, heartbeat=False)
    r, p = comm.getRank(), comm.getSlaveNum()

    def log(msg):
        print(f"[r{r} {time.perf_counter() - t0:8.3f}s] {msg}", flush=True)

    import ctypes
    import torch
    torch.cuda.set_device(0)
    from mp4x.ops import native
    from mp4x.parallel import vmm
    lib = native.hip()
    g = ctypes.c_size_t()
    native.check(lib.mp4x_vmm_granularity(ctypes.byref(g)), "granularity")
    log(f"granularity {g.value}")
    for chunk, n in plan:
        log(f"--- chunk {chunk} x {n}")
        own = vmm.VmmRegion.create(lib, chunk, n)
        log(f"created va=0x{own.va:x} fds={own.fds}")
        t = vmm.tensor_at(own.va, chunk * n, torch.float32, torch.device("cuda", 0))
        t.fill_(float(r + 1))
        torch.cuda.synchronize()
        log(f"filled ({t.numel()} floats), local sum ok={bool((t[:1024] == r + 1).all())}")
        got = vmm.exchange_fds(comm.server, r, p, own.fds, timeout=30)
        log("fds exchanged: " + ", ".join(f"rank {j}: {len(f)} fds" for j, f in got.items()))
        own.close_fds()
        peers = []
        for j, fds in got.items():
            pr = vmm.VmmRegion.import_fds(lib, fds, chunk)
            for fd in fds:
                os.close(fd)
            log(f"imported rank {j} at va=0x{pr.va:x}")
            peers.append((j, pr))
        comm.server.call("barrier", r)

        def read(tag):
            for j, pr in peers:
                pt = vmm.tensor_at(pr.va, chunk * n, torch.float32, torch.device("cuda", 0))
                head = float(pt[:1 << 16].sum())
                tail = float(pt[-(1 << 16):].sum())
                whole = float((pt == j + 1).sum()) / pt.numel()
                torch.cuda.synchronize()
                log(f"{tag} peer {j}: head {head} tail {tail} (expect {(j + 1) * (1 << 16)}), "
                    f"fraction right {whole:.6f}")
        read("plain")
        comm.server.call("barrier", r)
        native.check(lib.mp4x_release_all(native.stream_ptr()), "release_all")
        torch.cuda.synchronize()
        comm.server.call("barrier", r)
        read("after writer's system release")
        comm.server.call("barrier", r)
        del t
        for j, pr in peers:
            pr.free()
        comm.server.call("barrier", r)
        own.free()
        log("freed")
    comm.close(0)
    log("done")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64M:1,8M:4,512M:5")
    ap.add_argument("--stuck", type=float, default=60)
    a = ap.parse_args()
    plan = [(_sz(x.split(":")[0]), int(x.split(":")[1])) for x in a.sizes.split(",")]
    import multiprocessing as mp
    import tempfile
    from mp4x import CommMaster
    m = CommMaster(2, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=rank_main, args=(m.port, plan, a.stuck)) for _ in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join()
    m.stop(timeout=5)
    codes = [pr.exitcode for pr in procs]
    print("exit codes", codes, flush=True)
    sys.exit(0 if all(c == 0 for c in codes) else 1)


if __name__ == "__main__":
    main()
