"""update(defer=True) + finish_update() leaves exactly the state of update()
(GPU; the multi-GPU overlap itself is exercised by the 2-rank tests)."""
import pytest
import torch

from vq_gnn_amd.vq import VQBank
import vq_gnn_amd.vq as vqmod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _bank(nb, M, D):
    torch.manual_seed(0)
    bank = VQBank(nb, M, D, warm_up_flag=True)
    for b in range(nb):
        bank.init_branch(b)
    return bank.to(DEV)


def test_deferred_finalize_same_state(monkeypatch):
    monkeypatch.setattr(vqmod, "STRICT_BAD_INIT", False)
    nb, M, D, B, N = 8, 64, 4, 3000, 5000
    X = torch.randn(B, nb * D, device=DEV)
    G = torch.randn(B, nb * D, device=DEV) * 1e-3
    bidx = torch.randperm(N, device=DEV)[:B]
    a, b = _bank(nb, M, D), _bank(nb, M, D)
    ca = torch.zeros(N, nb, dtype=torch.int16, device=DEV)
    cb = ca.clone()
    for step in range(3):
        a.update(X, G, 0, nb, True, codes=ca, batch_idx=bidx)
        emb_before = b.emb_out.clone()
        b.update(X, G, 0, nb, True, codes=cb, batch_idx=bidx, defer=True)
        # until finish_update the codebook is the pre-update one
        assert torch.equal(b.emb_out, emb_before)
        b.finish_update()
        for name in ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g"):
            assert torch.equal(getattr(a, name), getattr(b, name)), (step, name)
        assert torch.equal(ca, cb)
        X = X * 1.01
    # a new update finishes a pending one first
    b.update(X, G, 0, nb, True, codes=cb, batch_idx=bidx, defer=True)
    b.update(X, G, 0, nb, True, codes=cb, batch_idx=bidx)
    a.update(X, G, 0, nb, True, codes=ca, batch_idx=bidx)
    a.update(X, G, 0, nb, True, codes=ca, batch_idx=bidx)
    assert torch.equal(a.emb_out, b.emb_out)
    a.check_bad_init()
    b.check_bad_init()
