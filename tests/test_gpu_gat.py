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
    al, ar, params, als, ars = kernels.gat_alpha(xd[:b.B], conv.att_l.view(-1),
                                                 conv.att_r.view(-1), F, X2=xd[b.B:], B=b.B,
                                                 ones=True)
    xin = torch.cat([torch.from_numpy(x), torch.ones(b.n, 1)], 1)
    al_ref = (xin * conv.att_l.detach().cpu().view(-1)).sum(-1)
    torch.testing.assert_close(al.cpu(), al_ref, rtol=1e-5, atol=1e-5)
    assert float(params[0]) == pytest.approx(float(al.max()), abs=0)
    # alpha / s per node: the reference's own division (convs.py:209-211)
    s = params[2].cpu()
    assert torch.equal(als.cpu(), al.cpu() / s) and torch.equal(ars.cpu(), ar.cpu() / s)
    coef, den = kernels.gat_coef(adj.rowptr, adj.col, adj.value, b.n, b.nnz, als, ars)
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
    mag = _gat_grad_magnitudes(x, xf, att_l0, att_r0, b, R)
    # every element within 1e-5 of the magnitude of the terms it sums
    for got, want, m, name in (
            (out.detach().cpu().double(), ref.detach(), mag["out"], "out"),
            (xd.grad.cpu().double(), x64.grad, mag["dx"], "dx"),
            (conv.att_l.grad.view(-1).cpu().double(), al64.grad, mag["datt_l"], "att_l"),
            (conv.att_r.grad.view(-1).cpu().double(), ar64.grad, mag["datt_r"], "att_r")):
        rel = ((got - want).abs() / (m + 1e-30)).max().item()
        assert rel < 1e-5, f"{name}: max error / magnitude {rel:.2e}"


def _gat_grad_magnitudes(x, xf, att_l, att_r, b, R, slope=0.2):
    """fp64 magnitudes (sums of |terms|) of the GAT layer output and of the
    gradients of sum(out * R), following the chain of convs_gat.GATFunction:
    the bound an fp32 evaluation of that chain must meet elementwise."""
    n, B, F = b.n, b.B, x.shape[1]
    xin = torch.cat([torch.cat([x, xf]).double(), torch.ones(n, 1, dtype=torch.float64)], 1)
    al, ar = xin @ att_l.double(), xin @ att_r.double()
    ml, mr = al.max(), ar.max()
    s = torch.sqrt(ml ** 2 + 1) * torch.sqrt(mr ** 2 + 1)
    row = torch.as_tensor(np.repeat(np.arange(n), np.diff(b.rowptr)))
    j = torch.as_tensor(b.col.astype(np.int64))
    a = al[j] / s + ar[row] / s
    c = torch.nn.functional.leaky_relu(a, slope).exp() * torch.as_tensor(b.val, dtype=torch.float64)
    den = torch.zeros(n, dtype=torch.float64).index_add(0, row, c)
    yabs = torch.zeros(n, F, dtype=torch.float64).index_add(0, row, xin[j, :F].abs() * c[:, None])
    q = torch.ones(n, 1, dtype=torch.float64)
    q[:B, 0] = den[:B] + 1e-16
    zabs = yabs / q
    dz = R.double().abs()
    dy = dz / q
    dden = torch.zeros(n, dtype=torch.float64)
    dden[:B] = (dz[:B] * zabs[:B]).sum(1) / q[:B, 0]
    qe = ((xin[j, :F].abs() * dy[row]).sum(1) + dden[row]) * c / s    # |leaky'| <= 1
    dal = torch.zeros(n, dtype=torch.float64).index_add(0, j, qe)
    dar = torch.zeros(n, dtype=torch.float64).index_add(0, row, qe)
    ds = (qe * a.abs()).sum()
    dml = ml.abs() / torch.sqrt(ml ** 2 + 1) * torch.sqrt(mr ** 2 + 1)   # |ds/dmax_l|
    dmr = mr.abs() / torch.sqrt(mr ** 2 + 1) * torch.sqrt(ml ** 2 + 1)
    dal = dal + (al == ml).double() * ds * dml
    dar = dar + (ar == mr).double() * ds * dmr
    dx = torch.zeros(n, F, dtype=torch.float64).index_add(0, j, dy[row] * c[:, None])[:B]
    dx = dx + dal[:B, None] * att_l.double().abs()[:F] + dar[:B, None] * att_r.double().abs()[:F]
    return dict(out=zabs, dx=dx, datt_l=xin.abs().t() @ dal, datt_r=xin.abs().t() @ dar)


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


def _hub_csr(n, B, rng, empty_runs=False):
    """A batch-like CSR with hub rows (cut by the task split), empty rows and
    single-edge rows; GAT-normalised (D^-1) positive weights.  empty_runs:
    also runs of 30-100 consecutive empty rows (the row-end records' skip
    escape: the fused kernel then reads the rows from erow)."""
    deg = rng.integers(1, 20, size=n)
    deg[[5, n // 2, B - 1]] = [700, 333, 1200]
    deg[rng.random(n) < 0.05] = 0
    if empty_runs:
        for a, ln in ((100, 30), (200, 31), (300, 32), (1000, 100), (B - 40, 39), (n // 2 + 1, 64)):
            deg[a:a + ln] = 0
    rowptr = np.zeros(n + 1, np.int64)
    rowptr[1:] = np.cumsum(deg)
    col = np.concatenate([np.sort(rng.choice(n, size=d, replace=d > n)) for d in deg])
    val = np.repeat(1.0 / np.maximum(deg, 1), deg).astype(np.float32)
    return rowptr, col.astype(np.int64), val


@pytest.mark.parametrize("F,empty_runs", [(32, False), (128, False), (256, False), (128, True),
                                          (32, True)])
def test_gat_fused_kernel_matches_coefficient_path(F, empty_runs):
    """vqgnn_gat_spmm_task (coefficients in the aggregation kernel) against the
    coefficient pass + task SpMM on coefficient records + normalise, on hub
    rows cut across tasks,
    empty rows and a multi-tile F; the optional coef / den outputs equal
    vqgnn_gat_coef's."""
    rng = np.random.default_rng(F + 1)
    n, B = 3000, 1800
    rowptr, col, val = _hub_csr(n, B, rng, empty_runs)
    adj = CSR(torch.as_tensor(rowptr), torch.as_tensor(col), torch.as_tensor(val),
              (n, n)).to(DEV)
    nnz = adj.nnz()
    x = torch.randn(B, F, device=DEV)
    xf = torch.randn(n - B, F, device=DEV)
    conv = _conv(F, 3).to(DEV)
    _, _, _, als, ars = kernels.gat_alpha(x, conv.att_l.view(-1), conv.att_r.view(-1), F, X2=xf,
                                          B=B, ones=True)
    plan = adj.plan(F, B=B)
    assert isinstance(plan, kernels.TaskPlan)
    out, den, coef = kernels.gat_spmm(adj.rowptr, adj.col, adj.value, n, nnz, x, F, als, ars,
                                      plan, adj.rows(), X2=xf, B=B, norm_B=B,
                                      want_den=True, want_coef=True)
    coef_ref, den_ref = kernels.gat_coef(adj.rowptr, adj.col, adj.value, n, nnz, als, ars)
    assert torch.equal(coef, coef_ref)                    # same op order, same bits
    torch.testing.assert_close(den, den_ref, rtol=1e-6, atol=0)
    # the unfused chain: the same task plan with the coefficients as weights
    ref = kernels.spmm(adj.rowptr, adj.col, coef_ref, n, nnz, x, F, X2=xf, B=B,
                       plan=plan.with_values(adj.col, coef_ref))
    kernels.gat_normalize(ref, B, F, den_ref, 1e-16)
    # fp64 bound: |got - ref64| <= 1e-5 * sum |coef| |x| / (den + eps) (rows < B)
    xin = torch.cat([x, xf]).double().cpu().numpy()
    c64 = coef_ref.double().cpu().numpy()
    ref64 = conv_ref.spmm_fp64(rowptr, col, c64, xin)
    sc = conv_ref.spmm_fp64(rowptr, col, np.abs(c64), np.abs(xin))
    d64 = den_ref.double().cpu().numpy()[:, None] + 1e-16
    ref64[:B] /= d64[:B]
    sc[:B] /= d64[:B]
    for got in (out, ref):
        err = np.abs(got.cpu().numpy() - ref64)
        assert (err <= 1e-5 * sc + 1e-30).all(), f"rel err {(err / (sc + 1e-30)).max():.2e}"
    # the fused rows are the raw sum times v_rcp_f32(den + 1e-16); gat_normalize
    # divides (the reference's /=, models.py:188): a few ulp apart (measured
    # up to 5 ulp of the quotient), pinned at 2^-20 relative (include/vqgnn.h
    # §8b; the north_star bound is 1e-5); rows >= B (never normalised)
    # bit-identical
    o, rr = out.cpu().numpy(), ref.cpu().numpy()
    ulp = np.spacing(np.abs(rr[:B]).astype(np.float32))
    assert (np.abs(o[:B] - rr[:B]) <= 2.0 ** -20 * np.abs(rr[:B]) + 1e-45).all(), \
        f"fused vs divided: {(np.abs(o[:B] - rr[:B]) / np.maximum(ulp, 1e-45)).max():.1f} ulp"
    assert np.array_equal(o[B:], rr[B:])
    assert torch.equal(out[torch.as_tensor(np.diff(rowptr) == 0, device=DEV)],
                       torch.zeros_like(out[torch.as_tensor(np.diff(rowptr) == 0, device=DEV)]))
    again, _, _ = kernels.gat_spmm(adj.rowptr, adj.col, adj.value, n, nnz, x, F, als, ars,
                                   plan, adj.rows(), X2=xf, B=B, norm_B=B)
    assert torch.equal(out, again)
    # the layer path runs the same fused kernel
    assert torch.equal(conv.fused_forward(x, adj, xf, B), out)


def test_gat_cut_and_uncut_rows_share_the_normalisation():
    """The walker (rows that end inside a task) and the fix-up (rows cut
    across tasks) normalise a row the same way: every normalised row < B is
    its raw coefficient-weighted sum times ONE reciprocal r_i of den_i +
    1e-16 (v_rcp_f32, within 1 ulp of 1/(den_i + 1e-16)), so identical rows
    get identical bits wherever the plan cuts them (an IEEE division in one
    path and a reciprocal in the other would not satisfy this)."""
    rng = np.random.default_rng(17)
    n, B, F = 3000, 1800, 128
    rowptr, col, val = _hub_csr(n, B, rng)
    adj = CSR(torch.as_tensor(rowptr), torch.as_tensor(col), torch.as_tensor(val),
              (n, n)).to(DEV)
    nnz = adj.nnz()
    x = torch.randn(B, F, device=DEV)
    xf = torch.randn(n - B, F, device=DEV)
    conv = _conv(F, 9).to(DEV)
    _, _, _, als, ars = kernels.gat_alpha(x, conv.att_l.view(-1), conv.att_r.view(-1), F, X2=xf,
                                          B=B, ones=True)
    plan = adj.plan(F, B=B)
    raw, _, _ = kernels.gat_spmm(adj.rowptr, adj.col, adj.value, n, nnz, x, F, als, ars, plan,
                                 adj.rows(), X2=xf, B=B, norm_B=0)
    out, den, _ = kernels.gat_spmm(adj.rowptr, adj.col, adj.value, n, nnz, x, F, als, ars, plan,
                                   adj.rows(), X2=xf, B=B, norm_B=B, want_den=True)
    raw, out, den = raw.cpu().numpy(), out.cpu().numpy(), den.cpu().numpy()
    lens = np.diff(rowptr)
    assert (lens[:B] > plan.K // 2).any()          # rows < B that the plan cuts across tasks
    q = (den[:B] + np.float32(1e-16)).astype(np.float32)
    r0 = (np.float32(1) / q).astype(np.float32)
    ok = np.zeros(B, bool)
    for step in (0, 1, -1):                        # r_i = 1/q_i or a neighbouring float
        r = r0 if step == 0 else np.nextafter(r0, np.float32(np.inf * step)).astype(np.float32)
        ok |= ((raw[:B] * r[:, None]).astype(np.float32) == out[:B]).all(1)
    assert ok[lens[:B] > 0].all(), f"{int((~ok[lens[:B] > 0]).sum())} rows not raw * r_i"
    assert np.array_equal(out[B:], raw[B:])        # rows >= B stay unnormalised


@pytest.mark.parametrize("F", [32, 128, 36])
def test_gat_edge_grad_and_att_grad_kernels(F):
    """The coefficient-chain backward (16-lane group kernel for aligned F,
    per-edge kernel otherwise) against an fp64 restatement of the chain
    (within 1e-5 of the magnitude), and gat_att_grad = x_in^T d alpha in
    fp64 within 1e-5."""
    g, b = _batch(seed=7)
    n, B = b.n, b.B
    adj = CSR(torch.from_numpy(b.rowptr), torch.from_numpy(b.col), torch.from_numpy(b.val),
              (n, n)).to(DEV)
    torch.manual_seed(F)
    x = torch.randn(B, F, device=DEV)
    xf = torch.randn(n - B, F, device=DEV)
    conv = _conv(F, 5).to(DEV)
    al, ar, params, als, ars = kernels.gat_alpha(x, conv.att_l.view(-1), conv.att_r.view(-1), F,
                                                 X2=xf, B=B, ones=True)
    coef, den = kernels.gat_coef(adj.rowptr, adj.col, adj.value, n, adj.nnz(), als, ars)
    dy = torch.randn(n, F, device=DEV)
    dden = torch.randn(n, device=DEV)
    dal, dar, dsr = kernels.gat_edge_grad(adj.rows(), adj.col, coef, adj.nnz(), x, F, dy, dden,
                                          als, ars, params, X2=xf, B=B)
    # fp64 chain: q_e = (x_in[j] . dy[i] + dden[i]) coef_e leaky'(a_e) / s
    rows, cols = adj.rows().long(), adj.col.long()
    xin = torch.cat([x, xf]).double()
    s = params[2].double()
    a = al.double()[cols] / s + ar.double()[rows] / s
    dot = (xin[cols] * dy.double()[rows]).sum(1) + dden.double()[rows]
    q = dot * coef.double() * torch.where(a > 0, 1.0, 0.2).double() / s
    qa = (dot.abs() * coef.double() / s)
    n_ = al.numel()
    for got, idx, val, mag_v in ((dal, cols, q, qa), (dar, rows, q, qa),
                                 (dsr, rows, -q * a, (qa * a.abs()))):
        ref = torch.zeros(n_, dtype=torch.float64, device=DEV).index_add_(0, idx, val)
        mag = torch.zeros(n_, dtype=torch.float64, device=DEV).index_add_(0, idx, mag_v)
        assert ((got.double() - ref).abs() / (mag + 1e-30)).max().item() < 1e-5
    if F % 4:
        return
    gl, gr = kernels.gat_att_grad(x, F, dal, dar, X2=xf, B=B, ones=True)
    xin1 = torch.cat([xin, torch.ones(n, 1, dtype=torch.float64, device=DEV)], 1)
    for got, da in ((gl, dal), (gr, dar)):
        ref = xin1.t() @ da.double()
        mag = xin1.abs().t() @ da.double().abs()
        assert ((got.double() - ref).abs() / (mag + 1e-30)).max().item() < 1e-5
