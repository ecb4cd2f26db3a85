"""ZeroOptimizer on the GPU: p ranks share cuda:0, the memAlloc parameter / gradient arenas make
the reduce-scatter and the all-gather run the zero-copy IPC kernels; the sharded AdamW
trajectory must match unsharded AdamW on the full batch (f32 and bf16 parameters, the latter
with an f32 master slice)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from spawn_ranks import run_spawn  # noqa: E402

pytestmark = pytest.mark.gpu


def _train(comm, dtype_name, clip, kw):
    from mp4x.models.zero import train_single_adamw, train_zero
    dtype = getattr(torch, dtype_name)
    before = dict(comm.device.stats)
    losses = train_zero(comm, steps=6, global_batch=48, device="cuda", dtype=dtype, max_grad_norm=clip, **kw)
    used = {k: c - before.get(k, 0) for k, c in comm.device.stats.items() if c != before.get(k, 0)}
    ref = train_single_adamw(steps=6, global_batch=48, device="cuda", dtype=dtype, max_grad_norm=clip) \
        if comm.getRank() == 0 else None
    return losses, ref, used


# the reduce-scatters launch from the backward hooks on a side stream (overlap, the GPU default);
# bucket_mb=0.01 splits the MLP into 2 buckets, micro=2 accumulates under no_sync()
@pytest.mark.parametrize("p,dtype,clip,kw", [(2, "float32", None, {}), (3, "float32", 0.05, {}),
                                             (2, "bfloat16", None, {}),
                                             (3, "float32", None, {"bucket_mb": 0.01, "micro": 2}),
                                             (2, "float32", None, {"overlap": False})])
def test_zero_gpu_matches_single(p, dtype, clip, kw):
    out = run_spawn(p, _train, args=(dtype, clip, kw))
    ref = out[0][1]
    tol = dict(rtol=1e-3, atol=1e-5) if dtype == "float32" else dict(rtol=3e-2, atol=1e-3)
    for r, (losses, _, used) in out.items():
        np.testing.assert_allclose(losses, ref, **tol)
        assert used.get("reduce_scatter.ipc_zc", 0) >= 6 and used.get("allgather.ipc_zc", 0) >= 6, used
