"""Factorization machine with sparse gradient sync (mp4x/models/fm.py): sparse embedding
gradients of every rank are merged with ONE allreduceSparse per step; the DP loss trajectory
(sparse Adagrad and SGD) equals one process on the concatenated batch."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from harness import run_ranks  # noqa: E402


def _fm(comm, adagrad):
    from mp4x.models.fm import train_fm
    return train_fm(comm, steps=8, global_batch=240, adagrad=adagrad)


@pytest.mark.parametrize("p,adagrad", [(2, True), (3, True), (2, False)])
def test_fm_sparse_dp_matches_single(p, adagrad):
    from mp4x.models.fm import train_fm
    ref = train_fm(None, steps=8, global_batch=240, adagrad=adagrad)
    assert ref[-1] < ref[0]                                  # it learns
    res, _, _ = run_ranks(p, _fm, (adagrad,), timeout=120)
    assert len(res) == p
    for losses in res.values():
        np.testing.assert_allclose(losses, ref, rtol=1e-5, atol=1e-7)


def test_fm_sparse_rows_cover_only_touched_features():
    from mp4x.models.fm import FM, _sparse_rows
    m = FM(50, 4)
    idx = torch.tensor([[1, 2, 3], [3, 4, 5]])
    torch.nn.functional.binary_cross_entropy_with_logits(m(idx), torch.ones(2)).backward()
    ids, rows = _sparse_rows(m)
    assert sorted(ids.tolist()) == [1, 2, 3, 4, 5] and rows.shape == (5, 5)
