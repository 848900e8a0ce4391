"""End-to-end drop-in parity: LowRankGNNLayer / LowRankGNN on the GPU vs the
oracle restatement of models.py:144-231 (VQ init + gather + aggregation)."""
import numpy as np
import pytest
import torch

from oracle import conv_ref, vq_ref
from vq_gnn_amd import graph
from vq_gnn_amd.models import LowRankGNN, LowRankGNNLayer

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _small_batch(conv="GCN", seed=0):
    g = graph.synthetic_graph(2500, 5, 9000, seed=seed)
    rp, cl, vl = graph.norm_adj(g, conv)
    b = graph.k_hop_batch(rp, cl, vl, g.N, graph.cluster_batch(g, [1, 3]))
    return g, b


def _layer(F_in, F_out, M, N, conv="GCN", **kw):
    return LowRankGNNLayer(F_in, F_out, 0.0, M, 4, N, 0, 'vq', False, True, 10, True, True,
                           False, 0, False, False, 0.5, [1, 1], True, False, True, 0.1, conv,
                           False, **kw)


@pytest.mark.parametrize("conv", ["GCN", "SAGE"])
def test_layer_forward_backward_vs_oracle(conv):
    torch.manual_seed(0)
    g, b = _small_batch(conv)
    F_in, F_out, M, D = 32, 16, 64, 4
    nb = F_in // D
    layer = _layer(F_in, F_out, M, g.N, conv)
    # oracle pre-state = the layer's initial state (CPU, before .to())
    states = []
    for i in range(nb):
        st = vq_ref.new_state(M, D, warm_up=True)
        for k, src in (("embedding", layer._bank.emb), ("ema_w", layer._bank.ema_w),
                       ("embedding_output", layer._bank.emb_out),
                       ("ema_cluster_size", layer._bank.cs)):
            st[k] = src[i].clone()
        states.append(st)
    codes_ref = layer._codes.clone()
    lin_w = layer.gnn_transform.weight.detach().clone()
    lin_b = layer.gnn_transform.bias.detach().clone()
    layer = layer.to(DEV).train()

    x = torch.randn(b.B, F_in)
    xg = x.clone().to(DEV).requires_grad_(True)
    batch_A = graph.batch_to_device(b, DEV)
    out, errors, _, _, losses, info_b, hooked = layer(xg, batch_A, 1.0, False)
    assert out.shape == (b.B, F_out) and len(errors) == nb and losses == 0

    # --- oracle forward ---
    for i in range(nb):
        idx = vq_ref.feature_update(states[i], x[:, i * D:(i + 1) * D])
        codes_ref[torch.from_numpy(b.batch_idx), i] = idx[:, 0].to(torch.int16)
    got_codes = layer._codes.cpu()
    mism = int((got_codes != codes_ref).sum())
    assert mism <= 2, f"{mism} code mismatches"
    emb_out = np.stack([st["embedding_output"].numpy() for st in states])
    torch.testing.assert_close(layer._bank.emb_out.cpu(), torch.from_numpy(emb_out),
                               rtol=1e-4, atol=1e-4)
    xin = conv_ref.gather_input(x, b.subset, b.B, got_codes.numpy(),
                                layer._bank.emb_out.cpu().numpy(), D)
    xin.requires_grad_(True)
    A = torch.sparse_coo_tensor(
        torch.stack([torch.from_numpy(np.repeat(np.arange(b.n), np.diff(b.rowptr))),
                     torch.from_numpy(b.col)]), torch.from_numpy(b.val), (b.n, b.n))
    agg = torch.sparse.mm(A, xin)
    ref = agg[:b.B] @ lin_w.t() + lin_b
    if conv == "SAGE":
        ref = ref + (x @ layer.fc_sage.weight.detach().cpu().t() + layer.fc_sage.bias.detach().cpu())
    torch.testing.assert_close(out.detach().cpu(), ref.detach(), rtol=1e-4, atol=1e-4)
    # info_backward is identically 0 in v2 (grad halves never updated)
    assert float(info_b) == 0.0

    # --- backward: d/dx through the aggregation (A^T) and the Linear ---
    R = torch.randn(b.B, F_out)
    (out * R.to(DEV)).sum().backward()
    xr = x.clone().requires_grad_(True)
    xin2 = torch.cat([xr, xin.detach()[b.B:]])
    ref2 = torch.sparse.mm(A, xin2)[:b.B] @ lin_w.t() + lin_b
    if conv == "SAGE":
        ref2 = ref2 + (xr @ layer.fc_sage.weight.detach().cpu().t())
    (ref2 * R).sum().backward()
    torch.testing.assert_close(xg.grad.cpu(), xr.grad, rtol=1e-4, atol=1e-4)
    for blk in layer.gnn_block:
        assert blk.X_B is not None and blk.batch_indices is not None


def test_model_init_train_eval_steps():
    """LowRankGNN through main_node.py's init -> train step -> eval flow."""
    torch.manual_seed(1)
    g, b = _small_batch("GCN", seed=1)
    model = LowRankGNN(32, 16, 7, 3, 0.0, 64, 4, g.N, no_second_fc=True, skip=True,
                       grad_scale=[1, 1], act='leaky_gelu', bn_flag=True, warm_up_flag=True,
                       conv_type='GCN').to(DEV)
    batch_A = graph.batch_to_device(b, DEV)
    x = torch.randn(b.B, 32, device=DEV)
    model.train()
    with torch.no_grad():
        for layer_idx in range(1, 4):
            model.init((x, batch_A), layer_idx)
    for layer in model.convs:
        for blk in layer.gnn_block:
            blk.inited = True
    opt = torch.optim.RMSprop(model.parameters(), lr=1e-3, alpha=0.99)
    y = torch.randint(0, 7, (b.B,), device=DEV)
    emb_before = model.convs[1]._bank.emb.clone()
    for _ in range(2):
        opt.zero_grad()
        out, vq_losses, info_b = model((x, batch_A), 1.0)
        loss = torch.nn.functional.cross_entropy(out, y) + info_b
        loss.backward()
        opt.step()
        assert torch.isfinite(loss)
    # v2: codebooks do not move in training steps (dead hooks)
    assert torch.equal(model.convs[1]._bank.emb, emb_before)
    model.eval()
    with torch.no_grad():
        out, _, _ = model((x, batch_A))
    assert out.shape == (b.B, 7) and torch.isfinite(out).all()


def test_opt_in_backward_vq_update_moves_codebooks():
    torch.manual_seed(2)
    g, b = _small_batch("GCN", seed=2)
    model = LowRankGNN(32, 16, 7, 2, 0.0, 64, 4, g.N, no_second_fc=True, skip=False,
                       grad_scale=[1, 1], warm_up_flag=True, vq_update_in_backward=True).to(DEV)
    batch_A = graph.batch_to_device(b, DEV)
    x = torch.randn(b.B, 32, device=DEV)
    model.train()
    with torch.no_grad():
        for layer_idx in range(1, 3):
            model.init((x, batch_A), layer_idx)
    for layer in model.convs:
        for blk in layer.gnn_block:
            blk.inited = True
    emb_before = model.convs[1]._bank.emb.clone()
    out, _, info_b = model((x, batch_A), 1.0)
    out.sum().backward()
    assert not torch.equal(model.convs[1]._bank.emb, emb_before)
    assert model.convs[1]._bank.bn_inited[0]
