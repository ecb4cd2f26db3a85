"""Local multi-process harness: a CommMaster thread + p rank processes on 127.0.0.1.

The reference's integration checks run a real master and N slave JVMs
(bin/comm_cluster_error_check.sh); this is the same topology on one host.
"""
import multiprocessing as mp
import os
import traceback

from mp4x.control.master import CommMaster

# exit codes of the rank processes and the master's remote-log lines of the last run_ranks call
LAST = {}


def _worker(fn, rank_hint, port, args, q, kind, threads):
    try:
        import sys
        if "torch" in sys.modules:
            # a parent that already ran a parallel torch op (e.g. a single-process reference
            # optimizer step) leaves an OpenMP team that does not survive fork: the child's
            # first parallel op would wait on it forever.  One intra-op thread never enters it.
            sys.modules["torch"].set_num_threads(1)
        from mp4x import ProcessCommSlave, ThreadCommSlave
        if kind == "thread":
            comm = ThreadCommSlave("test", threads, "127.0.0.1", port, heartbeat=False)
        else:
            comm = ProcessCommSlave("test", "127.0.0.1", port, heartbeat=False)
        res = fn(comm, *args)
        comm.close(0)
        q.put((comm.getRank(), "ok", res))
    except BaseException as e:  # noqa
        q.put((rank_hint, "err", traceback.format_exc()))


def run_ranks(p, fn, args=(), timeout=120, kind="process", threads=1, master_kwargs=None, expect_fail=False,
              env=None):
    ctx = mp.get_context("fork")
    import tempfile
    mk = dict(master_kwargs or {})
    mk.setdefault("workdir", tempfile.mkdtemp(prefix="mp4x_master_"))
    master = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, **mk).start()
    q = ctx.Queue()
    old = {}
    for k, v in (env or {}).items():
        old[k] = os.environ.get(k)
        os.environ[k] = v
    try:
        procs = [ctx.Process(target=_worker, args=(fn, i, master.port, args, q, kind, threads)) for i in range(p)]
        for pr in procs:
            pr.start()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    results = {}
    errors = []
    import queue as _q
    import time as _t
    deadline = _t.monotonic() + timeout
    try:
        got = 0
        while got < p and _t.monotonic() < deadline:
            try:
                r, st, val = q.get(timeout=0.25)
            except _q.Empty:
                # a rank that died without reporting (fault injection) ends the wait
                if any(pr.exitcode not in (None, 0) for pr in procs) and q.empty():
                    alive = [pr for pr in procs if pr.exitcode is None]
                    if not alive:
                        break
                    if expect_fail and got + len(alive) < p and all(pr.exitcode is not None for pr in procs):
                        break
                continue
            got += 1
            if st == "ok":
                results[r] = val
            else:
                errors.append(val)
                if not expect_fail:
                    break
    finally:
        for pr in procs:
            pr.join(timeout=5)
            if pr.is_alive():
                pr.kill()
                pr.join(timeout=5)
        code = master.stop(timeout=5)
        LAST["exitcodes"] = [pr.exitcode for pr in procs]
        LAST["logs"] = list(master.logs)
    if errors and not expect_fail:
        raise AssertionError("rank failed:\n" + "\n".join(errors))
    if not expect_fail and len(results) != p:
        raise AssertionError(f"only {len(results)}/{p} ranks finished")
    return results, code, errors
