"""GPU parity of the opt-in filtered assign path (vqgnn_assign_filter(1),
DESIGN.md §4.1): the bf16-split MFMA filter + exact resolve + exact list pass
must give the exact kernel's outputs bit for bit — indices, codes and the
int64 EMA statistics — and pass the same oracle / golden-vector checks."""
import pytest
import torch

import test_gpu_vq as exact_tests
from helpers import golden_cases
from vq_gnn_amd import kernels
from vq_gnn_amd._lib import lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture
def filter_on():
    lib().vqgnn_assign_filter(1)
    yield
    lib().vqgnn_assign_filter(-1)


def _run(X, G, coef, emb, D, W, codes, bidx, stats):
    nb = emb.shape[0]
    idx = torch.full((nb, X.shape[0]), -1, dtype=torch.int64, device=DEV)
    c = codes.clone() if codes is not None else None
    parts = kernels.vq_assign(X, G, coef, 0.75, emb, D, W, idx_out=idx, codes=c,
                              batch_idx=bidx, want_stats=stats)
    torch.cuda.synchronize()
    return idx, c, parts


@pytest.mark.parametrize("B,M,W,stats,near", [
    (20000, 256, 8, True, False), (20000, 256, 4, False, False), (3001, 37, 8, True, False),
    (2100, 1030, 8, True, False), (4000, 64, 8, True, True), (777, 256, 4, True, True)])
def test_filter_equals_exact_kernel(B, M, W, stats, near):
    """Filter on vs off on the same inputs: identical indices, codes and EMA
    statistics.  near: codebooks with duplicated and 1-ulp-perturbed rows, so
    many rows are undecided and take the exact list pass."""
    D, nb = 4, 8
    g = torch.Generator().manual_seed(B + M + W)
    X = (torch.randn(B, nb * D, generator=g) * 1.5).to(DEV)
    G = (torch.randn(B, nb * D, generator=g) * 1e-3).to(DEV) if W == 2 * D else None
    emb = torch.randn(nb, M, 2 * D, generator=g)
    if near:
        h = M // 2
        emb[:, h:2 * h] = emb[:, :h]
        emb[:, h:2 * h:3] = torch.nextafter(emb[:, h:2 * h:3], torch.tensor(10.0))
    emb = emb.to(DEV)
    coef = torch.zeros(6, nb * D)
    coef[0], coef[1] = 1.1, -0.05
    coef[2], coef[3] = 0.9, 0.01
    coef = coef.to(DEV)
    N = B + 500
    codes = torch.zeros(N, nb, dtype=torch.int16, device=DEV)
    bidx = torch.randperm(N, generator=g)[:B].to(DEV)
    lib().vqgnn_assign_filter(0)
    try:
        ref = _run(X, G, coef, emb, D, W, codes, bidx, stats)
        lib().vqgnn_assign_filter(1)
        got = _run(X, G, coef, emb, D, W, codes, bidx, stats)
        again = _run(X, G, coef, emb, D, W, codes, bidx, stats)
    finally:
        lib().vqgnn_assign_filter(-1)
    assert torch.equal(ref[0], got[0])
    assert torch.equal(ref[1], got[1])
    assert torch.equal(got[0], again[0])
    if stats:
        assert torch.equal(ref[2].sum(0), got[2].sum(0))


@pytest.mark.parametrize("M,D,W,B,tie", [
    (256, 4, 8, 3000, False), (256, 4, 4, 3000, False), (37, 4, 8, 1000, False),
    (1030, 4, 8, 2100, False), (64, 4, 8, 999, True)])
def test_filter_bit_exact_vs_oracle(filter_on, M, D, W, B, tie):
    exact_tests.test_assign_bit_exact_given_coefficients(M, D, W, B, tie)


@pytest.mark.parametrize("name", golden_cases())
def test_filter_vq_step_vs_reference_golden(filter_on, name):
    exact_tests.test_vq_step_vs_reference_golden(name)
