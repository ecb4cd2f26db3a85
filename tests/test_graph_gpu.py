"""hipGraph capture of device collectives (DeviceEngine.capture) on a 1-rank RCCL job: the
captured allreduce + K1 work replays with fresh inputs and gives the eager results."""
import multiprocessing as mp
import tempfile
import traceback

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _job(port, q):
    try:
        import torch
        from mp4x import Operands, Operators, ProcessCommSlave
        from mp4x.ops.device_ops import scale_
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("g", "127.0.0.1", port, heartbeat=False)
        eng = comm.device
        x = torch.zeros(1 << 20, device="cuda:0")
        y = torch.zeros(1 << 20, device="cuda:0")

        def step():   # "bucket" allreduces + the K1 average, as a DDP step would issue them
            eng.allreduce(x, 0, x.numel(), Operators.Float.SUM)
            eng.allreduce(y, 0, y.numel(), Operators.Float.MAX, Operands.FLOAT_OPERAND(compress=True))
            scale_(x, x, 0.5)

        g = eng.capture(step)
        bad = 0
        for i in range(5):
            x.fill_(float(i + 1))
            y.fill_(float(-i))
            g.replay()
            torch.cuda.synchronize()
            bad += int((x != (i + 1) * 0.5).sum()) + int((y != -i).sum())
        st = dict(eng.stats)
        comm.close(0)
        q.put(("ok", bad, st))
    except BaseException:
        q.put(("err", traceback.format_exc(), None))


def test_capture_replay_device_collectives():
    from mp4x import CommMaster
    m = CommMaster(1, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_job, args=(m.port, q))
    pr.start()
    try:
        st, bad, stats = q.get(timeout=300)
        assert st == "ok", bad
        assert bad == 0
        assert stats.get("allreduce.zs", 0) >= 2   # warm-up calls ran the lossless codec eagerly ...
        assert stats.get("allreduce.rccl", 0) >= 3  # ... the captured call switched to a capturable twin
    finally:
        pr.join(timeout=30)
        if pr.is_alive():
            pr.kill()
        m.stop(timeout=5)
