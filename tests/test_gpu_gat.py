"""GPU parity of the GAT attention aggregation (convs.py:165-266 +
models.py:178-189) against the oracle restatement (fp32, reference op order)
and its gradients against an fp64 autograd restatement.  Parity of this half
is pinned by KATs (tests/test_host_logic.py::test_gat_oracle_known_answer):
the reference conv modules are not importable here (no torch_geometric)."""
import numpy as np
import pytest
import torch

from oracle import conv_ref
from vq_gnn_amd import graph, kernels
from vq_gnn_amd.convs_gat import OurGATConv
from vq_gnn_amd.sparse import CSR

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _batch(seed=0):
    g = graph.synthetic_graph(2500, 5, 9000, seed=seed)
    rp, cl, vl = graph.norm_adj(g, "GAT")
    b = graph.k_hop_batch(rp, cl, vl, g.N, graph.cluster_batch(g, [0, 2]))
    return g, b


def _conv(F, seed=0):
    torch.manual_seed(seed)
    return OurGATConv(F + 1, F + 1, bias=False, add_self_loops=False)


@pytest.mark.parametrize("F", [128, 64, 32])
def test_gat_fused_forward_vs_oracle(F):
    g, b = _batch()
    rng = np.random.default_rng(F)
    x = rng.standard_normal((b.B, F)).astype(np.float32)
    xf = rng.standard_normal((b.n - b.B, F)).astype(np.float32)
    conv = _conv(F).to(DEV)
    _, _, adj = graph.batch_to_device(b, DEV)
    out = conv.fused_forward(torch.from_numpy(x).to(DEV), adj, torch.from_numpy(xf).to(DEV), b.B)
    xin = np.concatenate([np.concatenate([x, xf]), np.ones((b.n, 1), np.float32)], 1)
    ref, _ = conv_ref.gat_forward(xin, conv.att_l.detach().cpu().numpy(),
                                  conv.att_r.detach().cpu().numpy(), b.rowptr, b.col, b.val,
                                  B=b.B, normalize=True)
    assert out.shape == (b.n, F)
    # exp and the alpha dot products differ from ATen by a few ulps
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-6)


def test_gat_coefficients_and_alpha():
    g, b = _batch(1)
    F = 64
    rng = np.random.default_rng(3)
    x = rng.standard_normal((b.n, F)).astype(np.float32)
    conv = _conv(F, 2).to(DEV)
    _, _, adj = graph.batch_to_device(b, DEV)
    xd = torch.from_numpy(x).to(DEV)
    al, ar, params = kernels.gat_alpha(xd[:b.B], conv.att_l.view(-1), conv.att_r.view(-1), F,
                                       X2=xd[b.B:], B=b.B, ones=True)
    xin = torch.cat([torch.from_numpy(x), torch.ones(b.n, 1)], 1)
    al_ref = (xin * conv.att_l.detach().cpu().view(-1)).sum(-1)
    torch.testing.assert_close(al.cpu(), al_ref, rtol=1e-5, atol=1e-5)
    assert float(params[0]) == pytest.approx(float(al.max()), abs=0)
    coef, den = kernels.gat_coef(adj.rowptr, adj.col, adj.value, b.n, b.nnz, al, ar, params)
    _, coef_ref = conv_ref.gat_forward(xin.numpy(), conv.att_l.detach().cpu().numpy(),
                                       conv.att_r.detach().cpu().numpy(), b.rowptr, b.col, b.val)
    np.testing.assert_allclose(coef.cpu().numpy(), coef_ref.numpy(), rtol=2e-6, atol=1e-7)
    # den = the ones column: sum of the row's coefficients in CSR order
    ref_den = conv_ref.spmm_seq(b.rowptr, b.col, coef_ref.numpy(), np.ones((b.n, 1), np.float32))
    np.testing.assert_allclose(den.cpu().numpy(), ref_den[:, 0], rtol=2e-6, atol=1e-7)


def test_gat_backward_vs_fp64_autograd():
    g, b = _batch(2)
    F = 32
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.standard_normal((b.B, F)).astype(np.float32))
    xf = torch.from_numpy(rng.standard_normal((b.n - b.B, F)).astype(np.float32))
    R = torch.from_numpy(rng.standard_normal((b.n, F)).astype(np.float32))
    conv = _conv(F, 7)
    att_l0 = conv.att_l.detach().view(-1).clone()
    att_r0 = conv.att_r.detach().view(-1).clone()
    conv = conv.to(DEV)
    _, _, adj = graph.batch_to_device(b, DEV)
    xd = x.to(DEV).requires_grad_(True)
    out = conv.fused_forward(xd, adj, xf.to(DEV), b.B)
    (out * R.to(DEV)).sum().backward()
    # fp64 reference gradients
    x64 = x.double().requires_grad_(True)
    al64 = att_l0.double().requires_grad_(True)
    ar64 = att_r0.double().requires_grad_(True)
    ref = conv_ref.gat_forward_fp64(x64, xf, al64, ar64, b.rowptr, b.col, b.val, b.B)
    (ref * R.double()).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-4,
                               atol=1e-5)
    np.testing.assert_allclose(xd.grad.cpu().numpy(), x64.grad.numpy(), rtol=2e-3, atol=2e-4)
    np.testing.assert_allclose(conv.att_l.grad.view(-1).cpu().numpy(), al64.grad.numpy(),
                               rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(conv.att_r.grad.view(-1).cpu().numpy(), ar64.grad.numpy(),
                               rtol=2e-3, atol=2e-3)


def test_gat_reference_forward_dense_input():
    """OurGATConv.forward(x [n, C], adj): the reference conv call on a dense x
    (C = F + 1 not a multiple of 4: padded internally), no normalisation."""
    g, b = _batch(3)
    C = 33
    rng = np.random.default_rng(9)
    x = rng.standard_normal((b.n, C)).astype(np.float32)
    conv = _conv(C - 1, 4).to(DEV)
    adj = CSR(torch.as_tensor(b.rowptr), torch.as_tensor(b.col), torch.as_tensor(b.val),
              (b.n, b.n)).to(DEV)
    out = conv(torch.from_numpy(x).to(DEV), adj)
    ref, _ = conv_ref.gat_forward(x, conv.att_l.detach().cpu().numpy(),
                                  conv.att_r.detach().cpu().numpy(), b.rowptr, b.col, b.val)
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-6)
