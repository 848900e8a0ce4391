"""The BatchNorm finalize folded into the assign's prologue
(kernels.bn_stats_partial + vq_assign(BnFold), include/vqgnn.h §3a) leaves
exactly the state of the separate finalize (VQGNN_BN_FOLD=0): indices, codes,
running statistics, num_batches_tracked, the batch stash and the codebook
after the EMA update, bit for bit -- in every BatchNorm mode, for update()
(W = 2D) and feature_update() (W = D), over several row parts."""
import pytest
import torch

import vq_gnn_amd.vq as vqmod
from vq_gnn_amd import kernels
from vq_gnn_amd.vq import VQBank

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

STATE = ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g", "nbt_f", "nbt_g")


def _bank(nb, M, D, seed=0):
    torch.manual_seed(seed)
    bank = VQBank(nb, M, D, warm_up_flag=True)
    for b in range(nb):
        bank.init_branch(b)
    return bank.to(DEV)


def _run(monkeypatch, fold, nb, M, D, B, N, steps, feature, training, seed, pad):
    monkeypatch.setenv("VQGNN_BN_FOLD", "1" if fold else "0")
    monkeypatch.setattr(vqmod, "STRICT_BAD_INIT", False)
    gen = torch.Generator(device="cpu").manual_seed(seed)
    # a strided [B, nb*D] view, as the layers pass x (the reference's slices:
    # the STRIDED arithmetic, vq.py:162 / models.py:162-165)
    Xf = torch.randn(B, nb * D + pad, generator=gen).to(DEV) * 2.0 + 0.5
    Gf = torch.randn(B, nb * D + pad, generator=gen).to(DEV) * 1e-3
    X, G = Xf[:, :nb * D], Gf[:, :nb * D]
    bidx = torch.randperm(N, generator=gen)[:B].to(DEV)
    bank = _bank(nb, M, D, seed)
    codes = torch.zeros(N, nb, dtype=torch.int16, device=DEV)
    out = []
    for step in range(steps):
        idx = torch.empty(nb, B, dtype=torch.int64, device=DEV)
        if feature:
            bank.feature_update(X, 0, nb, training, idx_out=idx, codes=codes, batch_idx=bidx)
        else:
            bank.update(X, G, 0, nb, training, idx_out=idx, codes=codes, batch_idx=bidx)
        bank.finish_update()
        out.append(idx.clone())
        X = X * 1.01 + 0.003
    torch.cuda.synchronize()
    state = {k: getattr(bank, k).clone() for k in STATE}
    state["codes"] = codes.clone()
    state["idx"] = torch.stack(out)
    if not feature:
        state["batch"] = bank.last_batch.clone()
    return state


@pytest.mark.parametrize("nb,M,D,B,feature,training,pad", [
    (8, 64, 4, 3000, False, True, 3),       # update, train + init, then train (any-W rows)
    (32, 256, 4, 20000, False, True, 4),    # the arxiv shape's branches, float4 rows, row parts
    (32, 256, 4, 84_670, False, True, 0),   # the bench's own shape (contiguous [B, F])
    (16, 128, 4, 9000, True, True, 4),      # feature_update (W = D)
    (8, 64, 4, 3000, False, False, 4),      # eval + init, then eval
])
def test_fold_equals_separate_finalize(monkeypatch, nb, M, D, B, feature, training, pad):
    W = D if feature else 2 * D
    assert kernels.bn_fold_supported(B, nb, D, M, W)
    N = B + 777
    a = _run(monkeypatch, False, nb, M, D, B, N, 3, feature, training, 5, pad)
    b = _run(monkeypatch, True, nb, M, D, B, N, 3, feature, training, 5, pad)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_fold_supported_bounds():
    assert kernels.bn_fold_supported(84_670, 32, 4, 256, 8)
    assert kernels.bn_fold_supported(84_670, 32, 4, 256, 4)
    assert not kernels.bn_fold_supported(1, 32, 4, 256, 8)          # B <= 1
    assert not kernels.bn_fold_supported(1000, 32, 4, 256, 16)      # W > 8: the exact kernel
    assert not kernels.bn_fold_supported((1 << 23) + 1, 1, 4, 64, 8)
    assert not kernels.bn_fold_supported(30_000, 13, 4, 4096, 8)    # chunk-outer passes


def test_fold_is_single_use():
    X = torch.randn(500, 16, device=DEV)
    G = torch.randn(500, 16, device=DEV)
    rm, rv = torch.zeros(16, device=DEV), torch.ones(16, device=DEV)
    f = kernels.bn_stats_partial(X, G, 16, kernels.BN_TRAIN, 0.1, 1e-5, 0.1, 1e-5, 1e-5,
                                 rm, rv, rm.clone(), rv.clone())
    emb = torch.randn(4, 32, 8, device=DEV)
    kernels.vq_assign(X, G, f, 1.0, emb, 4, 8)
    with pytest.raises(ValueError):
        kernels.vq_assign(X, G, f, 1.0, emb, 4, 8)
    g = kernels.bn_stats_partial(X, G, 16, kernels.BN_TRAIN, 0.1, 1e-5, 0.1, 1e-5, 1e-5,
                                 rm, rv, rm.clone(), rv.clone())
    with pytest.raises(ValueError):                   # another X than the statistics'
        kernels.vq_assign(X.clone(), G, g, 1.0, emb, 4, 8)
