"""Node-aware allreduce on the GPU (mp4x/parallel/hier.py): 4 processes on one MI355X simulated as
2 nodes x 2 ranks (``MP4X_SIM_NODE_SIZE=2``).  Steps 1 and 3 run the IPC reduce-scatter /
copy-plan kernels inside each simulated node; gloo stands in for RCCL across nodes."""
import pytest

from spawn_ranks import run_spawn

pytestmark = pytest.mark.gpu


def hier_gpu_body(comm, n):
    import torch
    from mp4x import Operators
    eng = comm.device
    p, r = comm.getSlaveNum(), comm.getRank()
    dev = eng.device
    h = eng.hier()
    assert h is not None and eng.layout.hier_ok() and not eng.ipc_enabled
    idx = torch.arange(n, device=dev, dtype=torch.int64) % 13
    t = (idx + r).to(torch.float32)
    eng.allreduce(t, 0, n, Operators.Float.SUM)
    torch.cuda.synchronize()
    ok_sum = torch.equal(t, (idx * p + p * (p - 1) // 2).to(torch.float32))
    b = (idx * (r + 1)).to(torch.float32)
    eng.allreduce(b, 0, n, Operators.Float.MAX)
    ok_max = torch.equal(b, (idx * p).to(torch.float32))
    g = (idx + r).to(torch.float32)
    eng.allreduce(g, 0, n, Operators.Float.SUM, scale=1.0 / p)
    ok_avg = torch.allclose(g, (idx * p + p * (p - 1) / 2).to(torch.float32) / p)
    torch.cuda.synchronize()
    return ok_sum, ok_max, ok_avg, h.ipc is not None, h.stats["ipc_pieces"], h.selftest, \
        eng.stats.get("allreduce.hier", 0)


@pytest.mark.parametrize("n,piece", [(1 << 20, 1 << 20), (3 * (1 << 20) + 4096, 4 << 20)])
def test_hier_allreduce_two_simulated_nodes(n, piece):
    res = run_spawn(4, hier_gpu_body, args=(n,), timeout=200,
                    env={"MP4X_SIM_NODE_SIZE": "2", "MP4X_HIER_MIN_BYTES": "0", "MP4X_HIER": "1",
                         "MP4X_HIER_PIECE_BYTES": str(piece)})
    for r, (ok_sum, ok_max, ok_avg, has_ipc, ipc_pieces, st, calls) in res.items():
        assert ok_sum and ok_max and ok_avg, (r, ok_sum, ok_max, ok_avg)
        assert has_ipc and st["ok"] and st["ipc_nodes"] == 2, st
        assert ipc_pieces >= 3 and calls == 3
