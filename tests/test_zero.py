"""ZeroOptimizer (mp4x/models/zero.py): sharded AdamW over reduceScatterArray + allgatherArray
must follow the same loss trajectory as unsharded AdamW on the concatenated batch, with and
without global-norm clipping; a sharded checkpoint restores the exact state."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from harness import run_ranks  # noqa: E402


def _zero(comm, clip, kw):
    from mp4x.models.zero import train_zero
    return train_zero(comm, steps=6, global_batch=48, max_grad_norm=clip, **kw)


# bucket_mb=0.01: the MLP's 10.4k parameters in 2 buckets; overlap: the reduce-scatters launch from
# the backward hooks; micro=2: gradient accumulation with the first micro-batch under no_sync()
@pytest.mark.parametrize("p,clip,kw", [(2, None, {}), (3, None, {}), (2, 0.05, {}),
                                       (3, None, {"bucket_mb": 0.01, "overlap": True}),
                                       (2, 0.05, {"bucket_mb": 0.01, "overlap": True, "micro": 2})])
def test_zero_matches_single_adamw(p, clip, kw):
    from mp4x.models.zero import train_single_adamw
    ref = train_single_adamw(steps=6, global_batch=48, max_grad_norm=clip)
    res, _, _ = run_ranks(p, _zero, (clip, kw), timeout=120)
    assert len(res) == p
    for losses in res.values():
        np.testing.assert_allclose(losses, ref, rtol=2e-5, atol=1e-6)


def _layout(comm):
    from mp4x.models.mlp import MLP
    from mp4x.models.zero import ZeroOptimizer
    torch.manual_seed(0)
    m = MLP(5, 7, 3)                                    # 5*7+7+7*3+3 = 66 f32: padded to 16 * p / 4 multiples
    before = [q.detach().clone() for q in m.parameters()]
    opt = ZeroOptimizer(comm, m.parameters(), torch.optim.SGD, lr=0.0)
    assert len(opt.buckets) == 1
    g = opt.buckets[0]
    same = all(torch.equal(a, q) for a, q in zip(before, m.parameters()))
    views = all(q.data.data_ptr() >= g.param.data_ptr() and q.grad.data_ptr() >= g.grad.data_ptr()
                for q in m.parameters())
    out = (g.n, g.shard, g.lo, g.hi, same, views, g.aliased)
    opt.close()
    return out


def test_zero_layout_shards_are_vector_aligned():
    res, _, _ = run_ranks(3, _layout, timeout=60)
    for r, (n, shard, lo, hi, same, views, aliased) in res.items():
        assert n % 3 == 0 and shard == n // 3 and (shard * 4) % 16 == 0 and n >= 66
        assert (lo, hi) == (r * shard, (r + 1) * shard)
        assert same and views and aliased


def _ckpt(comm, tmp):
    import os
    from mp4x.models.mlp import MLP, synthetic_batch
    from mp4x.models.zero import ZeroOptimizer
    p, r = comm.getSlaveNum(), comm.getRank()

    def make():
        torch.manual_seed(0)
        m = MLP(16, 32, 4)
        return m, ZeroOptimizer(comm, m.parameters(), torch.optim.AdamW, lr=0.01)

    def run(m, opt, s0, s1):
        out = []
        for s in range(s0, s1):
            x, y = synthetic_batch(s, 16, 16, 4, "cpu")
            xs, ys = x[r * 8:(r + 1) * 8], y[r * 8:(r + 1) * 8]
            opt.zero_grad()
            loss = torch.nn.functional.mse_loss(m(xs), ys)
            loss.backward()
            opt.step()
            out.append(float(loss))
        return out

    m, opt = make()
    full = run(m, opt, 0, 6)
    opt.close()
    m, opt = make()
    run(m, opt, 0, 3)
    path = os.path.join(tmp, f"shard{r}.pt")
    torch.save(opt.state_dict(), path)
    opt.close()
    m, opt = make()                                     # fresh model: everything comes from the shards
    opt.load_state_dict(torch.load(path, weights_only=True))
    resumed = run(m, opt, 3, 6)
    opt.close()
    return full[3:], resumed


def test_zero_sharded_checkpoint_resume(tmp_path):
    res, _, _ = run_ranks(2, _ckpt, (str(tmp_path),), timeout=120)
    for full, resumed in res.values():
        assert full == resumed


def test_zero_single_process_is_plain_optimizer():
    from mp4x.models.zero import ZeroOptimizer

    class _Solo:
        def getSlaveNum(self):
            return 1

        def getRank(self):
            return 0

    torch.manual_seed(0)
    a = torch.nn.Linear(6, 3)
    b = torch.nn.Linear(6, 3)
    b.load_state_dict(a.state_dict())
    za = ZeroOptimizer(_Solo(), a.parameters(), torch.optim.AdamW, lr=0.1)
    ob = torch.optim.AdamW(b.parameters(), lr=0.1)
    x = torch.randn(10, 6)
    for _ in range(3):
        za.zero_grad()
        ob.zero_grad()
        a(x).square().sum().backward()
        b(x).square().sum().backward()
        za.step()
        ob.step()
    for qa, qb in zip(a.parameters(), b.parameters()):
        assert torch.equal(qa, qb)
    with pytest.raises(ValueError):
        ZeroOptimizer(_Solo(), [torch.nn.Parameter(torch.zeros(3, dtype=torch.int32), requires_grad=False)])
