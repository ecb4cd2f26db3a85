"""The communicator's stream order (VERDICT r5 Next #1; mp4x/parallel/order.py,
csrc/runtime/order.hip): collectives issued back to back from TWO streams, with no
synchronisation between them, still run one after the other on every rank — exact results, no
protocol error — at 2, 4 and 8 ranks sharing GPU 0 with per-rank jitter.  The same workload with
the guard disabled (MP4X_TEST_NO_STREAM_ORDER=1, tests only) fails: the test has teeth.

Every batch starts from fresh per-rank data and chains ~12 collectives over four tensors (each
call consumes the previous call's output on the same tensor), alternating streams call by call:
the slotted one-shot (fast path), the fused reduce-scatter and copy plans (fast paths), the
slotted and the staged two-shot, a zero-copy call on a registered tensor.  A random
``torch.cuda._sleep`` queued on the issuing stream before a call delays it there while the next
call is issued on the other stream.  The oracle is the same batch run once with a device
synchronisation after every call.

Reference: one send and one receive queue per process totally order its collectives
(/root/reference/src/main/java/com/fenbi/mp4j/comm/ProcessCommSlave.java:84-127, :1367)."""
import pytest

torch = pytest.importorskip("torch")

from spawn_ranks import run_spawn  # noqa: E402

pytestmark = pytest.mark.gpu


def _ops(comm, eng, inst, T):
    from mp4x import CommUtils, Operands, Operators
    from mp4x.parallel.ipc import TWOSHOT
    from mp4x.operators import for_dtype, DType
    p = comm.getSlaveNum()
    D, F = Operands.DOUBLE_OPERAND(), Operands.FLOAT_OPERAND()
    DS, FS = Operators.Double.SUM, Operators.Float.SUM
    f32sum = for_dtype(FS, DType.F32)
    a, b, c, z = T["a"], T["b"], T["c"], T["z"]
    na = a.numel()
    fr, to = CommUtils.createProcessArrayFroms(na, p), CommUtils.createProcessArrayTos(na, p)
    counts = [t - f for f, t in zip(fr, to)]
    nc = c.numel()
    cc = [nc // p] * p
    return [
        ("ar_a", lambda: comm.allreduceArray(a, D, DS, 0, na)),                  # slotted one-shot, fast path
        ("ar_a2", lambda: comm.allreduceArray(a, D, DS, 0, na)),
        ("rs_a", lambda: comm.reduceScatterArray(a, D, DS, 0, counts)),          # fused RS, fast path
        ("ag_a", lambda: comm.allgatherArray(a, D, list(fr), list(to))),        # copy plan, fast path
        ("ar_b_2shot", lambda: inst.allreduce(b, f32sum, algo=TWOSHOT)),         # slotted two-shot (1 MiB)
        ("bc_a", lambda: comm.broadcastArray(a, D, 0, na, p - 1)),              # copy plan, fast path
        ("ar_c_staged", lambda: inst.allreduce(c, f32sum, algo=TWOSHOT)),        # staged two-shot (6 MiB)
        ("ar_z_zc", lambda: comm.allreduceArray(z, F, FS, 0, z.numel())),        # zero-copy (registered)
        ("ar_b", lambda: comm.allreduceArray(b, F, FS, 0, b.numel())),
        ("ar_a3", lambda: comm.allreduceArray(a, D, DS, 0, na)),
        ("ar_z_avg", lambda: comm.allreduceArray(z, F, FS, 0, z.numel(), scale=1.0 / p)),
        ("rs_c", lambda: comm.reduceScatterArray(c, F, FS, 0, cc)),
    ]


def _fill(T, r):
    for k, t in T.items():
        i = torch.arange(t.numel(), device="cuda", dtype=torch.int64) % 13
        t.copy_((i + r + (3 if k == "c" else 0)).to(t.dtype))


def _order_fn(comm, batches, jitter, stop_on_failure):
    import random
    from mp4x.exceptions import Mp4jException
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    inst = eng.ipc()
    assert inst is not None
    T = {"a": torch.empty(1024, device="cuda", dtype=torch.float64),
         "b": torch.empty((1 << 20) // 4, device="cuda"),
         "c": torch.empty(6 * (1 << 20) // 4, device="cuda"),
         "z": torch.empty(8 * (1 << 20) // 4, device="cuda")}
    assert comm.registerBuffer(T["z"])
    ops = _ops(comm, eng, inst, T)
    # the oracle: one batch with a device synchronisation after every call
    _fill(T, r)
    torch.cuda.synchronize()
    for _, fn in ops:
        fn()
        torch.cuda.synchronize()
    ref = {k: t.clone() for k, t in T.items()}
    i = torch.arange(1024, device="cuda", dtype=torch.int64) % 13
    s1 = (i * p + p * (p - 1) // 2).double()
    oracle_ok = bool((ref["a"] == s1 * p ** 3).all())
    comm.barrier()
    rng = random.Random(1000 + 7 * r)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    calls = bad = raised = 0
    failed_batch = None
    first_err = None
    sw0 = eng.order.switches
    for bi in range(batches):
        _fill(T, r)
        torch.cuda.synchronize()
        for k, (name, fn) in enumerate(ops):
            with torch.cuda.stream(streams[k % 2]):
                if jitter and rng.random() < 0.5:
                    torch.cuda._sleep(rng.randint(1000, 200000))
                try:
                    fn()
                except Mp4jException as e:
                    raised += 1
                    first_err = first_err or f"{name}: {e}"
                calls += 1
        torch.cuda.synchronize()
        nb = sum(int((T[k] != ref[k]).sum()) for k in T)
        try:
            eng.check_failed()
        except Mp4jException as e:
            raised += 1
            first_err = first_err or f"after batch: {e}"
        bad += nb
        if stop_on_failure:
            anyfail = comm.server.call("allgather_obj", r, bool(nb or raised))
            if any(anyfail):
                failed_batch = bi
                break
    torch.cuda.synchronize()
    words = [i_.error_word(clear=True) for i_ in eng._ipc_all()]
    for i_ in eng._ipc_all():
        i_.error_word(clear=True)
    comm.barrier()
    comm.deregisterBuffer(T["z"])
    return {"calls": calls, "bad": bad, "raised": raised, "first_err": first_err, "words": words,
            "oracle_ok": oracle_ok, "switches": eng.order.switches - sw0, "failed_batch": failed_batch,
            "fast": {k: v for k, v in comm.stats["calls"].items()},
            "eng": {k: v for k, v in eng.stats.items() if "ipc" in k}}


def _record(name, out):
    """Per-rank outcomes as JSON lines into ``MP4X_TEST_RECORD`` (evidence for profiles/)."""
    import json
    import os
    path = os.environ.get("MP4X_TEST_RECORD")
    if path:
        with open(path, "a") as f:
            for r, o in sorted(out.items()):
                f.write(json.dumps({"test": name, "rank": r, **o}, default=str) + "\n")


@pytest.mark.parametrize("p,batches", [(2, 90), (4, 90), (8, 90)])
def test_two_stream_soak_is_exact(p, batches):
    out = run_spawn(p, _order_fn, args=(batches, True, False), timeout=600)
    _record(f"soak_p{p}", out)
    for r, o in out.items():
        assert o["oracle_ok"], (r, o)
        assert o["calls"] >= 1000, o
        assert o["bad"] == 0 and o["raised"] == 0, (r, o)
        assert all(w == 0 for w in o["words"]), (r, o)
        assert o["switches"] >= o["calls"] // 2, (r, o)       # nearly every call switched streams
        # the fast paths ran (not just the full path): fused RS and copy plans, one-shot
        eng = o["eng"]
        assert eng.get("reduce_scatter.ipc", 0) > 0 and eng.get("allgather.ipc", 0) > 0, eng
        assert any(k.endswith("ipc2z") or k.endswith("ipc_zc") for k in eng), eng


def test_without_the_guard_the_soak_fails():
    """Teeth: the same workload with the join disabled goes wrong (a wrong element or a protocol
    error / barrier timeout) within a few batches.  Short spin bound: a confused barrier gives up
    in 2 s instead of the fail-stop budget."""
    out = run_spawn(2, _order_fn, args=(40, True, True), timeout=400,
                    env={"MP4X_TEST_NO_STREAM_ORDER": "1", "MP4X_IPC_SPIN_S": "2"})
    _record("no_guard_p2", out)
    assert any(o["bad"] or o["raised"] or any(o["words"]) for o in out.values()), out
    assert all(o["switches"] == 0 for o in out.values()), out       # the guard really was off


def _capture_switch_fn(comm):
    from mp4x import Operands, Operators
    from mp4x.exceptions import Mp4jException
    r, p = comm.getRank(), comm.getSlaveNum()
    eng = comm.device
    eng.ipc()
    a = torch.ones(4096, device="cuda")
    b = torch.ones(4096, device="cuda")
    side = torch.cuda.Stream()
    F, SUM = Operands.FLOAT_OPERAND(), Operators.Float.SUM

    def step():
        comm.allreduceArray(a, F, SUM, 0, a.numel())
        side.wait_stream(torch.cuda.current_stream())        # fork a second stream ...
        try:
            with torch.cuda.stream(side):
                comm.allreduceArray(b, F, SUM, 0, b.numel())  # ... and issue the next collective on it
        finally:
            torch.cuda.current_stream().wait_stream(side)     # (joined back: the capture ends cleanly)
    raised = None
    try:
        eng.capture(step)
    except Mp4jException as e:
        raised = str(e)
    except RuntimeError as e:        # (torch reporting the capture the exception invalidated)
        raised = "runtime: " + str(e)
    torch.cuda.synchronize()
    comm.barrier()
    x = torch.full((4096,), float(r + 1), device="cuda")      # the job goes on, exact
    comm.allreduceArray(x, F, SUM, 0, x.numel())
    torch.cuda.synchronize()
    return raised, bool((x == p * (p + 1) / 2).all())


def test_a_stream_switch_inside_one_capture_is_refused():
    """Inside one graph capture the guard cannot join a forked stream to the previous launch (an
    eager event is not part of the graph): the second collective on another stream of the same
    capture raises, on every rank, and eager calls after it are exact (warm-up calls of the same
    step, eager, switch streams legally)."""
    out = run_spawn(2, _capture_switch_fn, timeout=240)
    for r, (raised, ok) in out.items():
        assert raised and "ONE stream" in raised, (r, raised)
        assert ok, r
