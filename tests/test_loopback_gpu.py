"""Device engine with p virtual ranks on ONE MI355X (LoopbackColl): every schedule runs the
real HIP kernels — K1 rank-ordered reduce, K6 fp8 codec, K4/K5 sparse — without RCCL."""
import pytest

from loopback_cases import codec_cases, dense_cases, run_virtual, scatter_family_cases, sparse_cases, zs_cases

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("p", [2, 3, 8])
def test_loopback_dense_gpu(p):
    assert all(run_virtual(p, dense_cases, device="cuda:0"))


@pytest.mark.parametrize("p", [2, 4, 8])
def test_loopback_codecs_gpu(p):
    assert all(run_virtual(p, codec_cases, device="cuda:0"))


@pytest.mark.parametrize("p", [2, 5])
def test_loopback_sparse_gpu(p):
    assert all(run_virtual(p, sparse_cases, device="cuda:0"))


@pytest.mark.parametrize("p", [2, 4])
def test_loopback_zs_lossless_gpu(p):
    assert all(run_virtual(p, zs_cases, device="cuda:0"))


@pytest.mark.parametrize("p", [2, 4])
def test_loopback_scatter_maps_gpu(p):
    assert all(run_virtual(p, scatter_family_cases, device="cuda:0"))
