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


@pytest.mark.parametrize("semantics,M", [("update", 256), ("feature_update", 256),
                                         ("update", 1024)])
def test_finalize_fused_into_codebook_spmm(monkeypatch, semantics, M):
    """The deferred EMA finalize run inside the codebook-source SpMM's fix-up
    launch (VQBank.take_fused_finalize + spmm_codebook(finalize=...),
    vqgnn_spmm_task_cb_fin) leaves the SpMM output and every piece of VQ
    state bit-identical to the SpMM followed by finish_update(), step after
    step (the SpMM reads the pre-update codebook in both).  M = 1,024: the
    finalize's two-kernel form, launched after the fix-up by the same entry."""
    from vq_gnn_amd import graph, kernels
    monkeypatch.setattr(vqmod, "STRICT_BAD_INIT", False)
    cfg = dict(graph.CONFIGS["arxiv_gcn"])
    g, _, bt = graph.make_batch(cfg)
    F, D = 128, 4
    nb = F // D
    bidx, subset, adj = graph.batch_to_device(bt, DEV)
    gen = torch.Generator(device="cpu").manual_seed(5)
    X = torch.randn(bt.B, F, generator=gen).to(DEV)
    G = (torch.randn(bt.B, F, generator=gen) * 1e-3).to(DEV)
    a, b = _bank(nb, M, D), _bank(nb, M, D)
    ca = torch.randint(0, M, (cfg["N"], nb), dtype=torch.int16, generator=gen).to(DEV)
    cb = ca.clone()
    pcb = adj.plan_codebook(bt.B, subset, cfg["N"])
    supported = kernels.codebook_source_ok(X, F, M, D, codes=ca, n_rows=bt.n, n_branches=nb)
    assert supported
    for step in range(3):
        for bank, codes, fused in ((a, ca, False), (b, cb, True)):
            if semantics == "update":
                bank.update(X, G, 0, nb, True, codes=codes, batch_idx=bidx, defer=True)
            else:
                bank.feature_update(X, 0, nb, True, codes=codes, batch_idx=bidx)
            fin = bank.take_fused_finalize() if fused else None
            if semantics == "update":
                assert (fin is not None) == fused
            else:                   # feature_update finalizes at once: nothing pending
                assert fin is None
            out = kernels.spmm_codebook(adj.rowptr, bt.n, bt.nnz, X, F, bt.B, codes,
                                        bank.emb_out, D, pcb, finalize=fin)
            bank.finish_update()
            if fused:
                out_b = out
            else:
                out_a = out
        assert torch.equal(out_a, out_b), step
        for name in ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g",
                     "bad_flag", "stats_u", "stats_f"):
            assert torch.equal(getattr(a, name), getattr(b, name)), (step, name)
        assert torch.equal(ca, cb)
        X = X * 1.01
    a.check_bad_init()
    b.check_bad_init()


@pytest.mark.parametrize("M,deferred", [(256, True), (256, False), (1024, True)])
def test_walk_beside_update_then_fixup(monkeypatch, M, deferred):
    """The overlapped step (bench.py's default): the codebook-source walk on a
    side stream (vqgnn_spmm_task_cb_walk) beside the VQ update on the main
    stream, then the fix-up with the update's EMA finalize
    (vqgnn_spmm_task_cb_fixup) after both -- the SpMM output and every piece
    of VQ state bit-identical to the serial update + spmm_codebook(finalize)
    form, step after step.  M = 1,024: the finalize's two-kernel form.
    deferred: the walk queued from the update's before_assign hook, after the
    BatchNorm launches (bench.py's order)."""
    from vq_gnn_amd import graph, kernels
    monkeypatch.setattr(vqmod, "STRICT_BAD_INIT", False)
    cfg = dict(graph.CONFIGS["arxiv_gcn"])
    g, _, bt = graph.make_batch(cfg)
    F, D = 128, 4
    nb = F // D
    bidx, subset, adj = graph.batch_to_device(bt, DEV)
    gen = torch.Generator(device="cpu").manual_seed(6)
    X = torch.randn(bt.B, F, generator=gen).to(DEV)
    G = (torch.randn(bt.B, F, generator=gen) * 1e-3).to(DEV)
    a, b = _bank(nb, M, D), _bank(nb, M, D)
    ca = torch.randint(0, M, (cfg["N"], nb), dtype=torch.int16, generator=gen).to(DEV)
    cb = ca.clone()
    pcb = adj.plan_codebook(bt.B, subset, cfg["N"])
    side = torch.cuda.Stream()
    for step in range(3):
        a.update(X, G, 0, nb, True, codes=ca, batch_idx=bidx, defer=True)
        out_a = kernels.spmm_codebook(adj.rowptr, bt.n, bt.nnz, X, F, bt.B, ca, a.emb_out, D,
                                      pcb, finalize=a.take_fused_finalize())
        a.finish_update()
        wk = kernels.spmm_codebook_walk(adj.rowptr, bt.n, bt.nnz, X, F, bt.B, cb, b.emb_out,
                                        D, pcb, stream=side, deferred=deferred)
        b.update(X, G, 0, nb, True, codes=cb, batch_idx=bidx, defer=True,
                 before_assign=wk.launch if deferred else None)
        assert wk.launched
        fin = b.take_fused_finalize()
        assert fin is not None
        out_b = kernels.spmm_codebook_fixup(wk, finalize=fin)
        b.finish_update()
        with pytest.raises(RuntimeError):
            kernels.spmm_codebook_fixup(wk)
        torch.cuda.synchronize()
        assert torch.equal(out_a, out_b), step
        for name in ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g",
                     "bad_flag", "stats_u", "stats_f"):
            assert torch.equal(getattr(a, name), getattr(b, name)), (step, name)
        assert torch.equal(ca, cb)
        X = X * 1.01
    a.check_bad_init()
    b.check_bad_init()
