"""RCCL communicators with explicit channel counts (ncclConfig min/max CTAs) and the
autotune that measures them: plumbing check on a 1-rank RCCL job (one GPU)."""
import multiprocessing as mp
import tempfile
import traceback

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _job(port, q):
    try:
        import torch
        from mp4x import Operators, ProcessCommSlave
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("v", "127.0.0.1", port, heartbeat=False)
        eng = comm.device
        t = torch.full((1 << 20,), 3.0, device="cuda:0")
        for ctas in eng.RCCL_CTA_VARIANTS:
            eng.rccl_variant(ctas).all_reduce(t, 0)
        ok = bool(torch.all(t == 3.0).item())
        big = torch.ones(32 << 20, device="cuda:0")          # 128 MiB: variants are candidates
        import os
        os.environ.pop("MP4X_AUTOTUNE_EXTRA", None)
        default = eng.autotune_allreduce(big, Operators.Float.SUM, iters=1)
        os.environ["MP4X_AUTOTUNE_EXTRA"] = "1"               # the variants are opt-in schedules
        res = eng.autotune_allreduce(big, Operators.Float.SUM, iters=2)
        comm.close(0)
        q.put(("ok", ok, (default, res)))
    except BaseException:
        q.put(("err", traceback.format_exc(), None))


def test_rccl_cta_variants_and_autotune():
    from mp4x import CommMaster
    m = CommMaster(1, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_job, args=(m.port, q))
    pr.start()
    try:
        st, ok, res = q.get(timeout=300)
        assert st == "ok", ok
        assert ok
        default, res = res
        assert "rccl" in default and not any(k.startswith("rccl_c") for k in default), default
        assert {"rccl", "rccl_c64", "rccl_c112"} <= set(res), res
        assert all(v < float("inf") for k, v in res.items() if k.startswith("rccl")), res
    finally:
        pr.join(timeout=30)
        if pr.is_alive():
            pr.kill()
        m.stop(timeout=5)
