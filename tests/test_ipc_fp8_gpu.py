"""Fused fp8 two-shot allreduce over IPC (csrc/runtime/ipc.hip k_ipc_fp8_twoshot), p processes
sharing ONE GPU.  The result must be BIT-identical to the K6 reference pipeline run locally
(quantise every rank's input, dequant + f32 rank-order sum + requant, dequant) — the same
numerics as the RCCL fp8 schedule — and within the e4m3 error bound of the fp32 sum."""
import multiprocessing as mp
import tempfile
import traceback

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _fp8_worker(port, q, cases, nbytes_buf):
    try:
        import torch
        from mp4x import ProcessCommSlave
        from mp4x.ops import device_ops as K
        from mp4x.parallel.ipc import IpcAllreduce
        torch.cuda.set_device(0)
        comm = ProcessCommSlave("t", "127.0.0.1", port, heartbeat=False)
        r, p = comm.getRank(), comm.getSlaveNum()
        ipc = IpcAllreduce(comm, nbytes=nbytes_buf)
        out = []
        for n, dtype_name in cases:
            dt = getattr(torch, dtype_name)
            xs = [torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(500 + j)).to(dt)
                  for j in range(p)]
            y = xs[r].clone()
            ipc.allreduce_fp8(y)
            torch.cuda.synchronize()
            qs, ss = zip(*[K.quant_fp8(x) for x in xs])
            nb = (n + 255) // 256
            qo = torch.empty(nb * 256, dtype=torch.uint8, device="cuda")
            so = torch.empty(nb, dtype=torch.float32, device="cuda")
            K.dequant_reduce_fp8(None, list(qs), list(ss), n, q_out=qo, s_out=so, out_dtype=torch.float32)
            ref = torch.empty(n, dtype=dt, device="cuda")
            K.dequant_fp8(qo, so, n, ref)
            exact = sum(x.double() for x in xs)
            err = ((y.double() - exact).abs().max() / exact.abs().max()).item()
            diff = (y != ref).nonzero().view(-1)
            info = (int(diff.numel()), int(diff[0]) if diff.numel() else -1,
                    float((y.double() - ref.double()).abs().max()))
            out.append((n, dtype_name, bool(torch.equal(y, ref)), err, float(y.double().sum()), ipc.error_word(),
                        info))
        comm.barrier()
        ipc.close()
        comm.close(0)
        q.put((r, "ok", out))
    except BaseException:
        q.put((-1, "err", traceback.format_exc()))


def _run(p, cases, nbytes_buf):
    from mp4x import CommMaster
    m = CommMaster(p, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fp8_worker, args=(m.port, q, cases, nbytes_buf)) for _ in range(p)]
    for pr in procs:
        pr.start()
    res = {}
    try:
        for _ in range(p):
            r, st, val = q.get(timeout=240)
            assert st == "ok", val
            res[r] = val
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
        m.stop(timeout=5)
    return res


@pytest.mark.parametrize("p", [2, 4])
def test_fp8_ipc_allreduce_matches_k6_pipeline(p):
    # one piece with a partial last block; several pieces through a 64 KiB buffer; bf16 input
    cases = [(256 * p * 3 + 100, "float32"), (200_000, "float32"), (70_004, "bfloat16")]
    res = _run(p, cases, nbytes_buf=64 << 10)
    assert sorted(res) == list(range(p))
    for i, (n, dt) in enumerate(cases):
        rows = [res[r][i] for r in range(p)]
        for (_, _, bit_equal, err, _, ew, info) in rows:
            assert ew == 0
            assert bit_equal, (n, dt, info)
            assert err < 2 ** -3, (n, dt, err)       # two e4m3 quantisations of the sum
        assert len({row[4] for row in rows}) == 1    # every rank holds the same result
