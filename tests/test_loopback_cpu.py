"""Device engine over the in-process loopback back-end, CPU tensors (no GPU needed)."""
import pytest

from loopback_cases import dense_cases, run_virtual, scatter_family_cases, sparse_cases, zs_cases


@pytest.mark.parametrize("p", [2, 3, 5])
def test_loopback_dense(p):
    assert all(run_virtual(p, dense_cases))


@pytest.mark.parametrize("p", [2, 4])
def test_loopback_sparse(p):
    assert all(run_virtual(p, sparse_cases))


@pytest.mark.parametrize("p", [2, 3])
def test_loopback_zs_lossless(p):
    assert all(run_virtual(p, zs_cases))


@pytest.mark.parametrize("p", [2, 3])
def test_loopback_scatter_maps(p):
    assert all(run_virtual(p, scatter_family_cases))
