"""Spawned multi-rank harness for GPU tests: a CommMaster + p fresh (spawned) rank processes.
``fn(comm, *args)`` must be a module-level function (it is pickled by name); its return value
comes back per rank.  ``threads`` > 0 gives each rank a ThreadCommSlave.

Two device plans (:func:`device_plan`):

* ``shared`` — every rank on cuda:0 (the 1-GPU box).  Device collectives other than the IPC
  kernels go through gloo (``MP4X_DEVICE_BACKEND=gloo``): RCCL refuses two ranks on one GPU;
  the IPC kernels run for real (same-device "remote" reads).
* ``multi`` — rank r on cuda:r with the nccl (= RCCL) backend, one GPU per rank: RCCL at p >= 2,
  cross-device IPC mappings over xGMI, the cross-GPU coherence the zero-copy protocol relies on.
  Chosen by ``mode="multi"`` (or ``"auto"`` when ``torch.cuda.device_count() >= p``).
"""
import multiprocessing as mp
import os
import tempfile
import traceback


def multi_dryrun() -> bool:
    """``MP4X_TEST_MULTI_DRYRUN=1``: the cross-GPU tests (``mode="multi"``) run with every rank on
    cuda:0 and gloo underneath instead of skipping on a box with fewer GPUs than ranks — every
    exact-value check of tests/test_multigpu_gpu.py runs before first contact with a real node;
    only what needs real RCCL or distinct device ordinals is skipped there."""
    return os.environ.get("MP4X_TEST_MULTI_DRYRUN", "0") == "1"


def device_plan(p, ndev, mode="shared"):
    """(plan, env) for ``p`` ranks on a box with ``ndev`` GPUs.  ``mode``: shared | multi | auto
    (``multi`` is planned as ``shared`` in a dry run, :func:`multi_dryrun`)."""
    if mode not in ("shared", "multi", "auto"):
        raise ValueError(mode)
    if mode == "multi" and multi_dryrun():
        mode = "shared"
    multi = mode == "multi" or (mode == "auto" and ndev >= p)
    if multi and ndev < p:
        raise ValueError(f"multi-GPU plan needs {p} GPUs, the box has {ndev}")
    if multi:
        return "multi", {"MP4X_DEVICE_BACKEND": "nccl", "MP4X_WATCHDOG": "0"}
    env = {"MP4X_DEVICE_BACKEND": "gloo", "MP4X_DEVICE_INDEX": "0", "MP4X_WATCHDOG": "0"}
    if p > 4:
        # p processes x 4 hardware queues each oversubscribe one GPU's queue slots beyond 4
        # ranks: the scheduler then time-slices the queues and every barrier kernel waits a
        # slice (8 ranks: 32 ms per 256 MiB allreduce with 4 queues each, 1.4 ms with 2:
        # profiles/r3/round/rehearsal_np8_queues.jsonl).  One process per GPU never needs this.
        env["GPU_MAX_HW_QUEUES"] = "2"
    return "shared", env


def rank_device(plan, rank):
    """The GPU ordinal rank ``rank`` uses under ``plan``."""
    return rank if plan == "multi" else 0


def _worker(fn, port, args, env, threads, q, dump_after, plan):
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
        if plan == "shared":
            torch.cuda.set_device(0)
        from mp4x import ProcessCommSlave, ThreadCommSlave
        if threads:
            comm = ThreadCommSlave("t", threads, "127.0.0.1", port, heartbeat=False)
        else:
            comm = ProcessCommSlave("t", "127.0.0.1", port, heartbeat=False)
        rank = comm.getRank()
        if plan == "multi":
            # the rank is known only after the rendezvous: bind this process to cuda:rank before
            # anything touches the device (the device engine then picks it up too)
            os.environ["MP4X_DEVICE_INDEX"] = str(rank_device(plan, rank))
            torch.cuda.set_device(rank_device(plan, rank))
        res = fn(comm, *args)
        comm.close(0)
        q.put((rank, "ok", res))
    except BaseException:  # noqa
        q.put((-1, "err", traceback.format_exc()))


def run_spawn(p, fn, args=(), env=None, timeout=240, threads=0, mode="shared"):
    from mp4x import CommMaster
    ndev = 1
    if mode != "shared" and not multi_dryrun():
        import torch
        ndev = torch.cuda.device_count()      # does not initialise the GPU in this process
    plan, e = device_plan(p, ndev, mode)
    e.update(env or {})
    m = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker,
                         args=(fn, m.port, args, e, threads, q, min(100, max(10, timeout - 60)), plan))
             for _ in range(p)]
    for pr in procs:
        pr.start()
    out = {}
    import queue as _queue
    import time as _time
    t_start = _time.monotonic()
    deadline = t_start + timeout
    beat = t_start
    progress = os.environ.get("MP4X_TEST_PROGRESS")
    try:
        while len(out) < p:
            if progress and _time.monotonic() - beat > 30:
                # a heartbeat for long multi-rank tests: a GPU call with nothing new on its outputs
                # for minutes is taken to be hung
                beat = _time.monotonic()
                with open(progress, "a") as f:
                    f.write(f"{_time.strftime('%H:%M:%S')} run_spawn {getattr(fn, '__name__', fn)} p={p}: "
                            f"{len(out)}/{p} ranks done after {beat - t_start:.0f} s\n")
            try:
                r, st, val = q.get(timeout=1.0)
            except _queue.Empty:
                # a rank that died without reporting (segfault, abort) fails the test now instead
                # of leaving it waiting silently until the timeout
                dead = [pr.exitcode for pr in procs if pr.exitcode not in (None, 0)]
                if dead and q.empty():
                    raise AssertionError(f"rank process(es) died with exit codes {dead}")
                if _time.monotonic() > deadline:
                    raise AssertionError(f"ranks did not finish within {timeout} s")
                continue
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
