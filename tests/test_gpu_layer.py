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


@pytest.mark.parametrize("conv,F_in", [("GCN", 32), ("SAGE", 32), ("GCN", 128), ("SAGE", 128)])
def test_layer_forward_backward_vs_oracle(conv, F_in):
    """F_in = 128: the aggregation reads the out-of-batch rows from the
    codebook (CodebookInput -> kernels.spmm_codebook); 32: gathered rows."""
    torch.manual_seed(0)
    g, b = _small_batch(conv)
    F_out, M, D = 16, 64, 4
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
    assert mism == 0, f"{mism} code mismatches"          # bit-exact indices
    emb_out = torch.from_numpy(np.stack([st["embedding_output"].numpy() for st in states]))
    got_eo = layer._bank.emb_out.cpu()
    rel = ((got_eo - emb_out).abs() / (1.0 + emb_out.abs().amax(-1, keepdim=True))).max()
    assert rel < 1e-5, f"embedding_output rel err {rel:.2e}"
    xin = conv_ref.gather_input(x, b.subset, b.B, got_codes.numpy(),
                                layer._bank.emb_out.cpu().numpy(), D)
    xin.requires_grad_(True)
    A = torch.sparse_coo_tensor(
        torch.stack([torch.from_numpy(np.repeat(np.arange(b.n), np.diff(b.rowptr))),
                     torch.from_numpy(b.col)]), torch.from_numpy(b.val), (b.n, b.n))
    agg = torch.sparse.mm(A, xin)
    # fp64 reference and its absolute-value bound: |got - ref| <= 1e-5 * scale
    # (north_star: fp32 messages within 1e-5 relative)
    A64, Aabs = A.double(), torch.sparse_coo_tensor(A._indices(), A._values().abs().double(),
                                                    A.shape)
    x64 = xin.detach().double()
    agg64, aggabs = torch.sparse.mm(A64, x64), torch.sparse.mm(Aabs, x64.abs())
    ref64 = agg64[:b.B] @ lin_w.double().t() + lin_b.double()
    scale = aggabs[:b.B] @ lin_w.double().abs().t() + lin_b.double().abs()
    if conv == "SAGE":
        fw, fb = layer.fc_sage.weight.detach().cpu().double(), layer.fc_sage.bias.detach().cpu().double()
        ref64 = ref64 + x.double() @ fw.t() + fb
        scale = scale + x.double().abs() @ fw.abs().t() + fb.abs()
    err = ((out.detach().cpu().double() - ref64).abs() / (scale + 1e-30)).max().item()
    assert err < 1e-5, f"layer output rel err {err:.2e}"
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
    # fp64 bound of the backward chain: |R| |W| |A|^T
    gabs = (R.double().abs() @ lin_w.double().abs())
    gpad = torch.zeros(b.n, F_in, dtype=torch.float64)
    gpad[:b.B] = gabs
    gscale = torch.sparse.mm(Aabs.t(), gpad)[:b.B]
    if conv == "SAGE":
        gscale = gscale + R.double().abs() @ layer.fc_sage.weight.detach().cpu().double().abs()
    gerr = ((xg.grad.cpu().double() - xr.grad.double()).abs() / (gscale + 1e-30)).max().item()
    assert gerr < 1e-5, f"dX rel err {gerr:.2e}"
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


def test_opt_in_backward_vq_update_vs_oracle():
    """SURVEY §8(f)2 (v1 hook semantics, vq_gnn_v1/models.py:71-125, batched
    over branches): the update run from the aggregation's backward equals
    vq_ref.update(X_B[:, branch], dOut[:B, branch]) per branch -- indices
    bit-exact (scattered into c_indices), BatchNorm state bit-exact, EMA state
    within 1e-5 -- and once the gradient halves of the codebooks have moved,
    info_backward (vq_gnn_v2/models.py:198) equals the oracle's
    sum(A[B:] @ x_input * grad_first_order) within 1e-5 of its magnitude."""
    torch.manual_seed(5)
    g, b = _small_batch("GCN", seed=5)
    F_in, F_out, M, D = 32, 16, 64, 4
    nb = F_in // D
    layer = _layer(F_in, F_out, M, g.N, "GCN", vq_update_in_backward=True).to(DEV).train()
    x = torch.randn(b.B, F_in)
    xd = x.to(DEV)
    batch_A = graph.batch_to_device(b, DEV)
    layer(xd, batch_A, 1.0, False)                 # init pass (feature_update)
    for blk in layer.gnn_block:
        blk.inited = True
    bank = layer._bank
    states = []
    for i in range(nb):
        st = vq_ref.new_state(M, D, warm_up=True)
        for k, src in (("embedding", bank.emb), ("ema_w", bank.ema_w),
                       ("embedding_output", bank.emb_out), ("ema_cluster_size", bank.cs),
                       ("rm_f", bank.rm_f), ("rv_f", bank.rv_f), ("rm_g", bank.rm_g),
                       ("rv_g", bank.rv_g)):
            st[k] = src[i].detach().cpu().clone()
        st["bn_inited"] = bank.bn_inited[i]
        states.append(st)
    captured = {}
    orig = layer._backward_vq_update

    def spy(x_det, grad_B, bidx):
        captured["g"] = grad_B.detach().clone()
        orig(x_det, grad_B, bidx)

    layer._backward_vq_update = spy
    xg = xd.clone().requires_grad_(True)
    out, *_ = layer(xg, batch_A, 1.0, False)
    R = torch.randn(b.B, F_out, device=DEV)
    (out * R).sum().backward()
    torch.cuda.synchronize()
    gB = captured["g"].cpu()
    assert gB.shape == (b.B, F_in) and gB.abs().max() > 0
    codes = layer._codes.cpu()
    bidx = torch.from_numpy(b.batch_idx)
    for i in range(nb):
        sl = slice(i * D, (i + 1) * D)
        idx, _, _ = vq_ref.update(states[i], x[:, sl], gB[:, sl])
        assert torch.equal(codes[bidx, i].long(), idx[:, 0]), f"branch {i}: index mismatch"
        for k, mine in (("rm_f", bank.rm_f), ("rv_f", bank.rv_f), ("rm_g", bank.rm_g),
                        ("rv_g", bank.rv_g)):
            assert torch.equal(mine[i].cpu(), states[i][k]), f"branch {i} {k}"
        for k, mine in (("embedding", bank.emb), ("embedding_output", bank.emb_out),
                        ("ema_cluster_size", bank.cs), ("ema_w", bank.ema_w)):
            a, r = mine[i].detach().cpu(), states[i][k]
            scale = 1.0 + (r.abs().amax(dim=-1, keepdim=True) if r.dim() == 2 else r.abs())
            err = ((a - r).abs() / scale).max().item()
            assert err < 1e-5, f"branch {i} {k}: rel err {err:.2e}"
    # the gradient halves moved: info_backward is live and matches the oracle
    emb_out = bank.emb_out.detach().cpu()
    assert emb_out[:, :, D:].abs().max() > 0
    layer._backward_vq_update = orig
    with torch.no_grad():
        _, _, _, _, _, info_b, _ = layer(xd, batch_A, 0.5, False)
    codes = layer._codes.cpu()
    xin = conv_ref.gather_input(x, b.subset, b.B, codes.numpy(), emb_out.numpy(), D).double()
    gfo = conv_ref.grad_first_order(b.subset, b.B, codes.numpy(), emb_out.numpy(), D).double()
    rows = np.repeat(np.arange(b.n), np.diff(b.rowptr))
    A = torch.sparse_coo_tensor(torch.stack([torch.from_numpy(rows), torch.from_numpy(b.col)]),
                                torch.from_numpy(b.val).double(), (b.n, b.n))
    agg = torch.sparse.mm(A, xin)[b.B:]
    ref = float((agg * gfo * 0.5).sum())
    mag = float((torch.sparse.mm(A.abs(), xin.abs())[b.B:]
                 * gfo.abs() * 0.5).sum())
    assert abs(float(info_b) - ref) <= 1e-5 * mag, (float(info_b), ref, mag)
    assert abs(ref) > 0


def test_layer_gat_forward_backward_vs_oracle():
    """conv_type='GAT' (models.py:93-97, :178-189): codebook gather, ones
    column, attention aggregation, normalisation of the batch rows, Linear."""
    torch.manual_seed(3)
    g, b = _small_batch("GAT", seed=3)
    F_in, F_out, M, D = 32, 16, 64, 4
    layer = _layer(F_in, F_out, M, g.N, "GAT")
    att_l = layer.conv.att_l.detach().view(-1).clone()
    att_r = layer.conv.att_r.detach().view(-1).clone()
    lin_w = layer.gnn_transform.weight.detach().clone()
    lin_b = layer.gnn_transform.bias.detach().clone()
    layer = layer.to(DEV).train()
    x = torch.randn(b.B, F_in)
    xg = x.clone().to(DEV).requires_grad_(True)
    out, *_ = layer(xg, graph.batch_to_device(b, DEV), 1.0, False)
    codes = layer._codes.cpu().numpy()
    emb_out = layer._bank.emb_out.cpu().numpy()
    xin = conv_ref.gather_input(x, b.subset, b.B, codes, emb_out, D).numpy()
    xin1 = np.concatenate([xin, np.ones((b.n, 1), np.float32)], 1)
    agg, _ = conv_ref.gat_forward(xin1, att_l.numpy(), att_r.numpy(), b.rowptr, b.col, b.val,
                                  B=b.B, normalize=True)
    # fp64 chain and its magnitude bound: |got - ref64| <= 1e-5 * scale, with
    # scale = (sum_e coef_e |x_j| / den) |W| + |b| (north_star: 1e-5 relative)
    x64 = x.double().requires_grad_(True)
    agg64 = conv_ref.gat_forward_fp64(x64, torch.from_numpy(xin[b.B:]), att_l.double(),
                                      att_r.double(), b.rowptr, b.col, b.val, b.B)
    with torch.no_grad():
        xin_abs = torch.from_numpy(np.abs(xin1)).double()
        _, coef = conv_ref.gat_forward(xin1, att_l.numpy(), att_r.numpy(), b.rowptr, b.col,
                                       b.val)
        rows = np.repeat(np.arange(b.n), np.diff(b.rowptr))
        Ac = torch.sparse_coo_tensor(torch.stack([torch.from_numpy(rows), torch.from_numpy(b.col)]),
                                     coef.double(), (b.n, b.n))
        aabs = torch.sparse.mm(Ac, xin_abs)[:b.B]
        aabs = aabs[:, :-1] / (aabs[:, -1:] + 1e-16)
        scale = aabs @ lin_w.double().abs().t() + lin_b.double().abs()
        ref64 = agg64[:b.B] @ lin_w.double().t() + lin_b.double()
        err = ((out.detach().cpu().double() - ref64).abs() / scale).max().item()
    assert err < 1e-5, f"GAT layer output rel err {err:.2e}"
    # backward vs fp64 autograd of the same chain, normwise within 1e-5
    R = torch.randn(b.B, F_out)
    (out * R.to(DEV)).sum().backward()
    ((agg64[:b.B] @ lin_w.double().t() + lin_b.double()) * R.double()).sum().backward()
    gerr = ((xg.grad.cpu().double() - x64.grad).abs().max() / x64.grad.abs().max()).item()
    assert gerr < 1e-5, f"GAT dX normwise rel err {gerr:.2e}"
    assert layer.conv.att_l.grad is not None and torch.isfinite(layer.conv.att_l.grad).all()


def test_model_gat_train_step():
    torch.manual_seed(4)
    g, b = _small_batch("GAT", seed=4)
    model = LowRankGNN(32, 16, 7, 2, 0.0, 64, 4, g.N, no_second_fc=True, skip=True,
                       grad_scale=[1, 1], warm_up_flag=True, conv_type='GAT').to(DEV)
    batch_A = graph.batch_to_device(b, DEV)
    x = torch.randn(b.B, 32, device=DEV)
    model.train()
    with torch.no_grad():
        for layer_idx in range(1, 3):
            model.init((x, batch_A), layer_idx)
    y = torch.randint(0, 7, (b.B,), device=DEV)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    for _ in range(2):
        opt.zero_grad()
        out, _, info_b = model((x, batch_A), 1.0)
        loss = torch.nn.functional.cross_entropy(out, y) + info_b
        loss.backward()
        opt.step()
        assert torch.isfinite(loss)


@pytest.mark.parametrize("conv", ["GCN", "GAT"])
def test_backward_update_on_side_stream_is_identical(conv, monkeypatch):
    """VQGNN_HOOK_OVERLAP=1 runs the hook's batched update on a side stream
    beside the layer's A^T product (convs._VQHook.start): the same codes,
    codebook state and input gradient, bit for bit, as the update run in
    stream order before the product."""
    g, b = _small_batch(conv, seed=7)
    F_in, F_out, M = 32, 16, 64
    batch_A = graph.batch_to_device(b, DEV)
    x = torch.randn(b.B, F_in, generator=torch.Generator().manual_seed(7)).to(DEV)
    R = torch.randn(b.B, F_out, generator=torch.Generator().manual_seed(8)).to(DEV)
    res = {}
    for overlap in ("0", "1"):
        monkeypatch.setenv("VQGNN_HOOK_OVERLAP", overlap)
        torch.manual_seed(5)
        layer = _layer(F_in, F_out, M, g.N, conv, vq_update_in_backward=True).to(DEV).train()
        layer(x, batch_A, 1.0, False)             # init pass
        for blk in layer.gnn_block:
            blk.inited = True
        xg = x.clone().requires_grad_(True)
        for _ in range(2):
            out, *_ = layer(xg, batch_A, 1.0, False)
            (out * R).sum().backward()
        torch.cuda.synchronize()
        bank = layer._bank
        res[overlap] = dict(codes=layer._codes.clone(), emb=bank.emb.clone(),
                            emb_out=bank.emb_out.clone(), cs=bank.cs.clone(),
                            ema_w=bank.ema_w.clone(), rm_g=bank.rm_g.clone(),
                            rv_g=bank.rv_g.clone(), dx=xg.grad.clone())
    for k in res["0"]:
        assert torch.equal(res["0"][k], res["1"][k]), k
