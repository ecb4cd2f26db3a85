"""Spawned multi-rank harness for GPU tests: a CommMaster + p fresh (spawned) rank processes
sharing cuda:0.  ``fn(comm, *args)`` must be a module-level function (it is pickled by name);
its return value comes back per rank.  ``threads`` > 0 gives each rank a ThreadCommSlave.

Device collectives other than the IPC kernels go through gloo (``MP4X_DEVICE_BACKEND=gloo``):
RCCL refuses two ranks on one GPU, the IPC kernels run for real.
"""
import multiprocessing as mp
import os
import tempfile
import traceback


def _worker(fn, port, args, env, threads, q, dump_after):
    try:
        import faulthandler
        import sys
        faulthandler.dump_traceback_later(dump_after, exit=False, file=sys.stderr)   # stacks if stuck
        os.environ.update(env)
        if os.environ.get("MP4X_TEST_LOG"):
            import logging
            logging.basicConfig(level=logging.INFO, stream=sys.stderr,
                                format="%(asctime)s %(name)s %(levelname)s %(message)s")
        import torch
        torch.cuda.set_device(0)
        from mp4x import ProcessCommSlave, ThreadCommSlave
        if threads:
            comm = ThreadCommSlave("t", threads, "127.0.0.1", port, heartbeat=False)
            rank = comm.getRank()
        else:
            comm = ProcessCommSlave("t", "127.0.0.1", port, heartbeat=False)
            rank = comm.getRank()
        res = fn(comm, *args)
        comm.close(0)
        q.put((rank, "ok", res))
    except BaseException:  # noqa
        q.put((-1, "err", traceback.format_exc()))


def run_spawn(p, fn, args=(), env=None, timeout=240, threads=0):
    from mp4x import CommMaster
    e = {"MP4X_DEVICE_BACKEND": "gloo", "MP4X_DEVICE_INDEX": "0", "MP4X_WATCHDOG": "0"}
    e.update(env or {})
    m = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(fn, m.port, args, e, threads, q, min(100, max(10, timeout - 60))))
             for _ in range(p)]
    for pr in procs:
        pr.start()
    out = {}
    try:
        for _ in range(p):
            r, st, val = q.get(timeout=timeout)
            assert st == "ok", val
            out[r] = val
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
                pr.join(timeout=5)
        m.stop(timeout=5)
    return out
