"""GPU parity of the codeword gather + two-source task SpMM and the CSR
transpose: every output row within 1e-5 of sum |w| |x| of the fp64 sum
(north_star: fp32 messages within 1e-5 relative)."""
import numpy as np
import pytest
import torch

from oracle import conv_ref
from vq_gnn_amd import graph, kernels
from vq_gnn_amd.sparse import CSR

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dev_csr(rowptr, col, val, n_rows, n_cols):
    return CSR(torch.as_tensor(np.asarray(rowptr)), torch.as_tensor(np.asarray(col)),
               torch.as_tensor(np.asarray(val, dtype=np.float32)), (n_rows, n_cols)).to(DEV)


def _assert_fp64(out, rowptr, col, val, x):
    ref = conv_ref.spmm_fp64(rowptr, col, val, x)
    scale = conv_ref.spmm_fp64(rowptr, col, np.abs(val), np.abs(x))
    err = np.abs(out.cpu().numpy().astype(np.float64) - ref)
    assert (err <= 1e-5 * scale + 1e-30).all(), f"max rel err {(err / (scale + 1e-30)).max():.3e}"


def _random_csr(n_rows, n_cols, deg_max, rng, hub_rows=(), hub_deg=0, empty_frac=0.1):
    deg = rng.integers(0, deg_max + 1, size=n_rows)
    deg[rng.random(n_rows) < empty_frac] = 0
    for h in hub_rows:
        deg[h] = hub_deg
    rowptr = np.zeros(n_rows + 1, np.int64)
    rowptr[1:] = np.cumsum(deg)
    col = np.concatenate([np.sort(rng.choice(n_cols, size=d, replace=d > n_cols))
                          for d in deg]) if rowptr[-1] else np.zeros(0, np.int64)
    val = rng.standard_normal(col.shape[0]).astype(np.float32)
    return rowptr, col.astype(np.int64), val


@pytest.mark.parametrize("F", [4, 16, 32, 64, 128, 256, 604, 1024])
def test_spmm_short_rows(F):
    rng = np.random.default_rng(F)
    rowptr, col, val = _random_csr(700, 500, 12, rng)
    x = rng.standard_normal((500, F)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, 700, 500)
    out = kernels.spmm(a.rowptr, a.col, a.value, 700, a.nnz(), torch.from_numpy(x).to(DEV), F)
    _assert_fp64(out, rowptr, col, val, x)
    assert np.all(out.cpu().numpy()[np.diff(rowptr) == 0] == 0)


def test_spmm_hub_rows_span_chunks():
    rng = np.random.default_rng(1)
    rowptr, col, val = _random_csr(3000, 4000, 20, rng, hub_rows=(5, 1700, 2999), hub_deg=3900)
    x = rng.standard_normal((4000, 128)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, 3000, 4000)
    out = kernels.spmm(a.rowptr, a.col, a.value, 3000, a.nnz(), torch.from_numpy(x).to(DEV), 128)
    _assert_fp64(out, rowptr, col, val, x)


@pytest.mark.parametrize("F", [16, 64, 128, 256, 604])
def test_spmm_many_adjacent_long_rows(F):
    """Runs of rows much longer than a task (K = 64 edges): every task of
    such a run holds a cut row, the fix-up sums their partials."""
    rng = np.random.default_rng(F + 7)
    n_rows, n_cols = 400, 900
    deg = rng.integers(0, 30, size=n_rows)
    deg[100:160] = rng.integers(257, 700, size=60)
    deg[300:303] = 900
    rowptr = np.zeros(n_rows + 1, np.int64)
    rowptr[1:] = np.cumsum(deg)
    col = np.concatenate([np.sort(rng.choice(n_cols, size=d, replace=False)) for d in deg])
    val = rng.standard_normal(col.shape[0]).astype(np.float32)
    x = rng.standard_normal((n_cols, F)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, n_rows, n_cols)
    xd = torch.from_numpy(x).to(DEV)
    out = kernels.spmm(a.rowptr, a.col, a.value, n_rows, a.nnz(), xd, F)
    _assert_fp64(out, rowptr, col, val, x)
    again = kernels.spmm(a.rowptr, a.col, a.value, n_rows, a.nnz(), xd, F)
    assert torch.equal(out, again)      # fixed task order: deterministic


def test_spmm_empty_and_degenerate():
    x = torch.randn(10, 8, device=DEV)
    a = _dev_csr([0, 0, 0, 0], [], [], 3, 10)
    out = kernels.spmm(a.rowptr, a.col, a.value, 3, 0, x, 8)
    assert torch.count_nonzero(out) == 0
    # trailing empty rows + leading empty rows
    rowptr = [0, 0, 2, 2, 3, 3, 3]
    a = _dev_csr(rowptr, [1, 4, 9], [1.0, 2.0, 3.0], 6, 10)
    out = kernels.spmm(a.rowptr, a.col, a.value, 6, 3, x, 8).cpu()
    xc = x.cpu()
    exp = torch.zeros(6, 8)
    exp[1] = 1.0 * xc[1] + 2.0 * xc[4]
    exp[3] = 3.0 * xc[9]
    assert torch.equal(out, exp)


@pytest.mark.parametrize("F,D", [(128, 4), (32, 4), (256, 4), (64, 8), (48, 2), (60, 3)])
def test_codeword_gather_and_two_source_spmm_vs_oracle(F, D):
    g = graph.synthetic_graph(4000, 8, 20000, seed=F + D)
    rp, cl, vl = graph.norm_adj(g, "GCN")
    b = graph.k_hop_batch(rp, cl, vl, g.N, graph.cluster_batch(g, [0, 2, 5]))
    nb, M = F // D, 50
    rng = np.random.default_rng(0)
    X = rng.standard_normal((b.B, F)).astype(np.float32)
    emb_out = rng.standard_normal((nb, M, 2 * D)).astype(np.float32)
    codes = rng.integers(0, M, size=(g.N, nb)).astype(np.int16)
    bidx, subset, adj = graph.batch_to_device(b, DEV)
    codes_d = torch.from_numpy(codes).to(DEV)
    emb_d = torch.from_numpy(emb_out).to(DEV)
    xt, lcodes = kernels.gather_codewords(subset, b.B, codes_d, emb_d, D, want_codes=True)
    assert torch.equal(lcodes.cpu(), torch.from_numpy(codes[b.subset[b.B:]]))
    gfo, _ = kernels.gather_codewords(subset, b.B, codes_d, emb_d, D, col_offset=D)
    torch.testing.assert_close(gfo.cpu(), conv_ref.grad_first_order(b.subset, b.B, codes,
                                                                    emb_out, D), rtol=0, atol=0)
    out = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, torch.from_numpy(X).to(DEV),
                       F, X2=xt, B=b.B)
    xin = conv_ref.gather_input(X, b.subset, b.B, codes, emb_out, D).numpy()
    _assert_fp64(out, b.rowptr, b.col, b.val, xin)


def test_two_source_far_apart_inputs():
    """x and x_first_order more than 4 GiB apart: the task kernel switches
    from one 32-bit buffer range to 64-bit row addresses (FAR); same bits as
    the near path on the same rows."""
    rng = np.random.default_rng(7)
    n, B, F = 900, 500, 128
    rowptr, col, val = _random_csr(n, n, 14, rng)
    x = rng.standard_normal((n, F)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, n, n)
    # both inputs carved out of one allocation, 5 GiB apart
    gap = 5 << 30
    nb2 = (n - B) * F * 4
    big = torch.empty(gap + nb2, dtype=torch.uint8, device=DEV)
    xd = big[:B * F * 4].view(torch.float32).view(B, F)
    x2d = big[gap:gap + nb2].view(torch.float32).view(n - B, F)
    xd.copy_(torch.from_numpy(x[:B]))
    x2d.copy_(torch.from_numpy(x[B:]))
    assert x2d.data_ptr() - xd.data_ptr() >= (4 << 30)
    out = kernels.spmm(a.rowptr, a.col, a.value, n, a.nnz(), xd, F, X2=x2d, B=B)
    _assert_fp64(out, rowptr, col, val, x)
    near = kernels.spmm(a.rowptr, a.col, a.value, n, a.nnz(), xd.clone(), F, X2=x2d.clone(), B=B)
    assert torch.equal(out, near)
    del big


def test_scatter_codes():
    N, nb, B = 100, 5, 30
    codes = torch.zeros(N, nb, dtype=torch.int16, device=DEV)
    bidx = torch.randperm(N)[:B].to(DEV)
    local = torch.randint(0, 99, (B, nb), dtype=torch.int16, device=DEV)
    pad = torch.cat([bidx, torch.full((4,), -1, device=DEV)])
    lpad = torch.cat([local, torch.zeros(4, nb, dtype=torch.int16, device=DEV)])
    kernels.scatter_codes(pad, lpad, codes)
    assert torch.equal(codes[bidx], local)
    mask = torch.ones(N, dtype=torch.bool, device=DEV)
    mask[bidx] = False
    assert int(codes[mask].abs().sum()) == 0


@pytest.mark.parametrize("n_rows,n_cols", [(500, 700), (1, 9), (300, 300)])
def test_csr_transpose_and_backward_product(n_rows, n_cols):
    rng = np.random.default_rng(n_rows)
    rowptr, col, val = _random_csr(n_rows, n_cols, 15, rng, hub_rows=(0,), hub_deg=min(n_cols, 400))
    a = _dev_csr(rowptr, col, val, n_rows, n_cols)
    t = a.transposed()
    r = np.repeat(np.arange(n_rows), np.diff(rowptr))
    order = np.lexsort((r, col))
    exp_ptr = np.zeros(n_cols + 1, np.int64)
    exp_ptr[1:] = np.cumsum(np.bincount(col, minlength=n_cols))
    assert np.array_equal(t.rowptr.cpu().numpy(), exp_ptr)
    assert np.array_equal(t.col.cpu().numpy(), r[order])
    assert np.array_equal(t.value.cpu().numpy(), val[order])
    d = rng.standard_normal((n_rows, 16)).astype(np.float32)
    dx = kernels.spmm(t.rowptr, t.col, t.value, n_cols, t.nnz(), torch.from_numpy(d).to(DEV), 16)
    exp = np.zeros((n_cols, 16))
    np.add.at(exp, col, val[:, None].astype(np.float64) * d[r])
    scale = np.zeros((n_cols, 16))
    np.add.at(scale, col, np.abs(val[:, None].astype(np.float64) * d[r]))
    err = np.abs(dx.cpu().numpy() - exp)
    assert (err <= 1e-5 * scale + 1e-30).all()


def test_arxiv_shaped_properties():
    """Full arxiv-shaped batch: SpMM vs fp64 (size-independent bound) and
    linearity out(a x + y) = a out(x) + out(y) to fp32 rounding."""
    cfg = graph.CONFIGS["arxiv_gcn"]
    g, _, b = graph.make_batch(cfg)
    bidx, subset, adj = graph.batch_to_device(b, DEV)
    F = 128
    x = torch.randn(b.n, F, device=DEV)
    y = torch.randn(b.n, F, device=DEV)
    ox = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, x, F)
    oy = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, y, F)
    oxy = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, 2 * x + y, F)
    # linearity within the per-row fp32 chain bound of both sides
    scale = conv_ref.spmm_fp64(b.rowptr, b.col, np.abs(b.val),
                               np.abs((2 * x).cpu().numpy()) + np.abs(y.cpu().numpy()))
    lin = np.abs((oxy - (2 * ox + oy)).cpu().numpy())
    assert (lin <= 4e-5 * scale + 1e-30).all()
    _assert_fp64(ox, b.rowptr, b.col, b.val, x.cpu().numpy())
