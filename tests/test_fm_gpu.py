"""FM sparse DP on the GPU (ranks share cuda:0): the per-step allreduceSparse of the embedding
gradient rows (1 + k = 8 floats: whole 16-byte vectors) runs the IPC sparse exchange and the
K4b / K5 kernels; the loss trajectory matches one process on the whole batch."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from spawn_ranks import run_spawn  # noqa: E402

pytestmark = pytest.mark.gpu


def _fm(comm):
    from mp4x.models.fm import train_fm
    before = dict(comm.device.stats)
    losses = train_fm(comm, steps=6, global_batch=240, k=7, device="cuda")
    used = {k: c - before.get(k, 0) for k, c in comm.device.stats.items() if c != before.get(k, 0)}
    ref = train_fm(None, steps=6, global_batch=240, k=7, device="cuda") if comm.getRank() == 0 else None
    return losses, ref, used


@pytest.mark.parametrize("p", [2, 3])
def test_fm_sparse_dp_gpu(p):
    out = run_spawn(p, _fm)
    ref = out[0][1]
    for r, (losses, _, used) in out.items():
        np.testing.assert_allclose(losses, ref, rtol=1e-4, atol=1e-6)
        assert used.get("sparse.a2a.ipc", 0) >= 6, used
