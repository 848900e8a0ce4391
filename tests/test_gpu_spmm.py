"""GPU parity of the fused gather-SpMM, code gather and CSR transpose."""
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
def test_spmm_bit_exact_short_rows(F):
    """Rows inside one edge chunk are summed in CSR order with mul+add ->
    bit-identical to torch_sparse spmm_sum's CPU loop."""
    rng = np.random.default_rng(F)
    rowptr, col, val = _random_csr(700, 500, 12, rng)
    x = rng.standard_normal((500, F)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, 700, 500)
    out = kernels.spmm(a.rowptr, a.col, a.value, 700, a.nnz(), torch.from_numpy(x).to(DEV), F)
    ref = conv_ref.spmm_seq(rowptr, col, val, x)
    deg = np.diff(rowptr)
    inside = deg <= 128   # rows of <= L edges are summed whole by their owner
    o = out.cpu().numpy()
    assert np.array_equal(o[inside], ref[inside])
    np.testing.assert_allclose(o, ref, rtol=1e-5, atol=1e-5)
    assert np.all(o[deg == 0] == 0)


def test_spmm_hub_rows_span_chunks():
    rng = np.random.default_rng(1)
    rowptr, col, val = _random_csr(3000, 4000, 20, rng, hub_rows=(5, 1700, 2999), hub_deg=3900)
    x = rng.standard_normal((4000, 128)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, 3000, 4000)
    out = kernels.spmm(a.rowptr, a.col, a.value, 3000, a.nnz(), torch.from_numpy(x).to(DEV), 128)
    ref = conv_ref.spmm_fp64(rowptr, col, val, x)
    scale = conv_ref.spmm_fp64(rowptr, col, np.abs(val), np.abs(x)) + 1e-6
    assert np.max(np.abs(out.cpu().numpy() - ref) / scale) < 1e-5


@pytest.mark.parametrize("F", [16, 64, 128, 256, 604])
def test_spmm_many_adjacent_long_rows(F):
    """Runs of rows longer than L = 256 edges: several rows end inside one
    wave's 64 chunks, so the fixup sums up to 64/F4 rows at a time."""
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
    ref = conv_ref.spmm_fp64(rowptr, col, val, x)
    scale = conv_ref.spmm_fp64(rowptr, col, np.abs(val), np.abs(x)) + 1e-6
    assert np.max(np.abs(out.cpu().numpy() - ref) / scale) < 1e-5
    again = kernels.spmm(a.rowptr, a.col, a.value, n_rows, a.nnz(), xd, F)
    assert torch.equal(out, again)      # fixed chunk order: deterministic


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
    ref = conv_ref.spmm_seq(b.rowptr, b.col, b.val, xin)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)
    inside = np.diff(b.rowptr) <= 128
    assert np.array_equal(out.cpu().numpy()[inside], ref[inside])


def test_two_source_far_apart_inputs():
    """x and x_first_order more than 4 GiB apart: the wave kernel switches
    from one 32-bit buffer range to 64-bit row addresses; same results."""
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
    ref = conv_ref.spmm_seq(rowptr, col, val, x)
    inside = np.diff(rowptr) <= 128
    assert np.array_equal(out.cpu().numpy()[inside], ref[inside])
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
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
    np.testing.assert_allclose(dx.cpu().numpy(), exp, rtol=1e-4, atol=1e-5)


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
    torch.testing.assert_close(oxy, 2 * ox + oy, rtol=1e-4, atol=1e-4)
    ref = conv_ref.spmm_fp64(b.rowptr, b.col, b.val, x.cpu().numpy())
    assert np.abs(ox.cpu().numpy() - ref).max() < 1e-4


@pytest.mark.parametrize("F,D,M", [(128, 4, 256), (128, 4, 50), (64, 4, 512), (256, 4, 128),
                                   (64, 2, 200)])
def test_spmm_codes_vs_two_source(F, D, M):
    """Code-source SpMM (x_first_order never materialised, codebooks in LDS):
    bit-identical to the two-source SpMM on the gathered x_first_order and
    to the spmm_sum loop on rows of at most L edges."""
    nb = F // D
    assert kernels.spmm_codes_supported(F, nb, M, D)
    g = graph.synthetic_graph(6000, 10, 40000, seed=F + M)
    rp, cl, vl = graph.norm_adj(g, "GCN")
    b = graph.k_hop_batch(rp, cl, vl, g.N, graph.cluster_batch(g, [1, 4, 6, 7]))
    rng = np.random.default_rng(M)
    X = rng.standard_normal((b.B, F)).astype(np.float32)
    emb_out = rng.standard_normal((nb, M, 2 * D)).astype(np.float32)
    codes = rng.integers(0, M, size=(g.N, nb)).astype(np.int16)
    bidx, subset, adj = graph.batch_to_device(b, DEV)
    codes_d = torch.from_numpy(codes).to(DEV)
    emb_d = torch.from_numpy(emb_out).to(DEV)
    xd = torch.from_numpy(X).to(DEV)
    xt, lcodes = kernels.gather_codewords(subset, b.B, codes_d, emb_d, D, want_codes=True)
    two = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, xd, F, X2=xt, B=b.B)
    plan = adj.plan(F, kind="chunk")
    fused = kernels.spmm_codes(adj.rowptr, adj.col, adj.value, b.n, b.nnz, xd, F, lcodes, emb_d,
                               D, b.B, plan=plan)
    assert torch.equal(fused, two)
    nop = kernels.spmm_codes(adj.rowptr, adj.col, adj.value, b.n, b.nnz, xd, F, lcodes, emb_d,
                             D, b.B)
    assert torch.equal(nop, two)
    xin = conv_ref.gather_input(X, b.subset, b.B, codes, emb_out, D).numpy()
    ref = conv_ref.spmm_seq(b.rowptr, b.col, b.val, xin)
    inside = np.diff(b.rowptr) <= 128
    assert np.array_equal(fused.cpu().numpy()[inside], ref[inside])
    np.testing.assert_allclose(fused.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)
    # the grad halves (grad_first_order source) through col_offset
    g2 = kernels.spmm_codes(adj.rowptr, adj.col, adj.value, b.n, b.nnz, xd, F, lcodes, emb_d,
                            D, b.B, plan=plan, col_offset=D)
    gt, _ = kernels.gather_codewords(subset, b.B, codes_d, emb_d, D, col_offset=D)
    assert torch.equal(g2, kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, xd, F,
                                        X2=gt, B=b.B))


def test_spmm_codes_unsorted_rows_hubs_and_edges():
    """Rows whose columns alternate between X and code sources (not CSR
    sorted), rows longer than L (carries), empty rows, and B = n_cols (no
    code rows) / B = 0 (codes only)."""
    rng = np.random.default_rng(11)
    F, D, M = 128, 4, 256
    nb = F // D
    n_rows, n_cols, B = 2500, 3000, 1700
    rowptr, col, val = _random_csr(n_rows, n_cols, 40, rng, hub_rows=(3, 1200), hub_deg=2900)
    # shuffle the columns inside each row: X and code runs interleave
    for i in range(n_rows):
        s, e = rowptr[i], rowptr[i + 1]
        col[s:e] = rng.permutation(col[s:e])
    X = rng.standard_normal((B, F)).astype(np.float32)
    emb_out = rng.standard_normal((nb, M, 2 * D)).astype(np.float32)
    lc = rng.integers(0, M, size=(n_cols - B, nb)).astype(np.int16)
    a = _dev_csr(rowptr, col, val, n_rows, n_cols)
    xd = torch.from_numpy(X).to(DEV)
    emb_d = torch.from_numpy(emb_out).to(DEV)
    lcd = torch.from_numpy(lc).to(DEV)
    out = kernels.spmm_codes(a.rowptr, a.col, a.value, n_rows, a.nnz(), xd, F, lcd, emb_d, D, B)
    xin = np.concatenate([X, emb_out[np.arange(nb)[None, :], lc.astype(np.int64), :D]
                          .reshape(n_cols - B, F)])
    ref = conv_ref.spmm_seq(rowptr, col, val, xin)
    inside = np.diff(rowptr) <= 128
    assert np.array_equal(out.cpu().numpy()[inside], ref[inside])
    ref64 = conv_ref.spmm_fp64(rowptr, col, val, xin)
    scale = conv_ref.spmm_fp64(rowptr, col, np.abs(val), np.abs(xin)) + 1e-6
    assert np.max(np.abs(out.cpu().numpy() - ref64) / scale) < 1e-5
    # B = n_cols: a plain SpMM over X
    xfull = torch.from_numpy(np.ascontiguousarray(xin)).to(DEV)
    o2 = kernels.spmm_codes(a.rowptr, a.col, a.value, n_rows, a.nnz(), xfull, F,
                            lcd[:0], emb_d, D, n_cols)
    assert torch.equal(o2, kernels.spmm(a.rowptr, a.col, a.value, n_rows, a.nnz(), xfull, F))
    # B = 0: every source is a code record
    lc_all = torch.from_numpy(rng.integers(0, M, size=(n_cols, nb)).astype(np.int16)).to(DEV)
    o3 = kernels.spmm_codes(a.rowptr, a.col, a.value, n_rows, a.nnz(), xd[:0], F, lc_all,
                            emb_d, D, 0)
    xin3 = emb_out[np.arange(nb)[None, :], lc_all.cpu().numpy().astype(np.int64), :D] \
        .reshape(n_cols, F)
    assert np.array_equal(o3.cpu().numpy()[inside],
                          conv_ref.spmm_seq(rowptr, col, val, xin3)[inside])
    # empty CSR
    e = _dev_csr([0] * 6, [], [], 5, n_cols)
    o4 = kernels.spmm_codes(e.rowptr, e.col, e.value, 5, 0, xd, F, lcd, emb_d, D, B)
    assert torch.count_nonzero(o4) == 0
    assert not kernels.spmm_codes_supported(128, 32, 1024, 4)   # 512 KiB of codebook


@pytest.mark.parametrize("nb,M,B", [(32, 1024, 1700), (151, 1024, 1700), (12, 300, 1700),
                                    (32, 1024, 0), (32, 1024, 3000)])
def test_spmm_task_codes_vs_task_two_source(nb, M, B):
    """Task-split code-source SpMM (include/vqgnn.h §6g; reddit's M = 1024 and
    F = 604's partial last tile): bit-identical to the task SpMM over the
    gathered rows (same records, order, fix-up), within 1e-5 of fp64; rows
    interleaving X and code columns, hub rows cut across tasks, empty rows,
    B = 0 (codes only) and B = n_cols (no codes)."""
    D = 4
    F = nb * D
    assert kernels.spmm_task_codes_supported(F, nb, M, D)
    rng = np.random.default_rng(nb * 7 + M + B)
    n_rows, n_cols = 2500, 3000
    rowptr, col, val = _random_csr(n_rows, n_cols, 40, rng, hub_rows=(3, 1200), hub_deg=2900)
    for i in range(n_rows):
        s, e = rowptr[i], rowptr[i + 1]
        col[s:e] = rng.permutation(col[s:e])
    X = rng.standard_normal((max(B, 1), F)).astype(np.float32)
    emb_out = rng.standard_normal((nb, M, 2 * D)).astype(np.float32)
    lc = rng.integers(0, M, size=(n_cols - B, nb)).astype(np.int16)
    a = _dev_csr(rowptr, col, val, n_rows, n_cols)
    xd = torch.from_numpy(X).to(DEV)
    emb_d = torch.from_numpy(emb_out).to(DEV)
    lcd = torch.from_numpy(lc).to(DEV)
    plan = a.plan(F, kind="task")
    for off in (0, D):
        out = kernels.spmm_codes(a.rowptr, a.col, a.value, n_rows, a.nnz(), xd, F, lcd, emb_d, D,
                                 B, plan=plan, col_offset=off)
        xt = emb_out[np.arange(nb)[None, :], lc.astype(np.int64), off:off + D].reshape(-1, F)
        xtd = torch.from_numpy(np.ascontiguousarray(xt)).to(DEV)
        if B == 0:
            two = kernels.spmm(a.rowptr, a.col, a.value, n_rows, a.nnz(), xtd, F, plan=plan)
        elif B == n_cols:
            two = kernels.spmm(a.rowptr, a.col, a.value, n_rows, a.nnz(), xd, F, plan=plan)
        else:
            two = kernels.spmm(a.rowptr, a.col, a.value, n_rows, a.nnz(), xd, F, X2=xtd, B=B,
                               plan=plan)
        assert torch.equal(out, two), f"col_offset={off}"
        xin = np.concatenate([X[:B], xt]) if B < n_cols else X
        ref64 = conv_ref.spmm_fp64(rowptr, col, val, xin)
        scale = conv_ref.spmm_fp64(rowptr, col, np.abs(val), np.abs(xin)) + 1e-6
        assert np.max(np.abs(out.cpu().numpy() - ref64) / scale) < 1e-5
    assert not kernels.spmm_task_codes_supported(F, nb, 2048, D)


# --- segment-pair SpMM (include/vqgnn.h §6d): bit-identical to vqgnn_spmm ---

def _pair_vs_chunk(rowptr, col, val, n_rows, n_cols, F, B=None, x2_rows=0, seed=0):
    rng = np.random.default_rng(seed)
    a = _dev_csr(rowptr, col, val, n_rows, n_cols)
    if x2_rows:
        X = torch.from_numpy(rng.standard_normal((B, F)).astype(np.float32)).to(DEV)
        X2 = torch.from_numpy(rng.standard_normal((x2_rows, F)).astype(np.float32)).to(DEV)
    else:
        X = torch.from_numpy(rng.standard_normal((n_cols, F)).astype(np.float32)).to(DEV)
        X2 = None
    chunk = kernels.spmm_plan(a.rowptr, n_rows, a.nnz(), F)
    pp = kernels.spmm_pair_plan(a.rowptr, n_rows, a.nnz(), F, B if B is not None else n_rows,
                                chunk=chunk)
    ref = kernels.spmm(a.rowptr, a.col, a.value, n_rows, a.nnz(), X, F, X2=X2, B=B, plan=chunk)
    got = kernels.spmm(a.rowptr, a.col, a.value, n_rows, a.nnz(), X, F, X2=X2, B=B, plan=pp)
    return ref, got, pp, X, X2


def test_pair_plan_covers_every_row_once():
    rng = np.random.default_rng(3)
    deg = rng.integers(0, 40, size=5000)
    deg[rng.random(5000) < 0.2] = 0
    deg[[7, 2500, 4999]] = [300, 1000, 257]       # long rows: S-aligned pieces
    rowptr = np.zeros(5001, np.int64)
    rowptr[1:] = np.cumsum(deg)
    a = _dev_csr(rowptr, np.zeros(rowptr[-1], np.int64), np.zeros(rowptr[-1]), 5000, 10)
    pp = kernels.spmm_pair_plan(a.rowptr, 5000, a.nnz(), 128, 3000)
    hdr = pp.buf[:16].cpu().numpy()
    nseg, nlong = int(hdr[0]), int(hdr[1])
    xb = hdr[2:11]
    assert xb[0] == 0 and xb[8] == nseg and np.all(np.diff(xb) >= 0)
    segs = pp.buf[16:16 + 4 * nseg].view(-1, 4).cpu().numpy()
    rows = segs[segs[:, 2] >= 0, 2]
    long_rows = np.nonzero(deg > 256)[0]
    assert nlong == len(long_rows)
    # every short row exactly once (empty rows too), long rows only as pieces
    assert np.array_equal(np.sort(rows), np.setdiff1d(np.arange(5000), long_rows))
    pieces = segs[segs[:, 2] <= -2]
    assert pieces[:, 1].sum() == deg[long_rows].sum()
    # edges covered exactly once
    cover = np.zeros(rowptr[-1], np.int32)
    for st, ln, _, _ in segs:
        cover[st:st + ln] += 1
    assert np.all(cover == 1)
    # inside each XCD range: row windows ascending, lengths descending per window
    for x in range(8):
        s = segs[xb[x]:xb[x + 1]]
        if len(s) < 2:
            continue
        assert np.all(s[:, 1] <= 511)


@pytest.mark.parametrize("seed", [0, 1])
def test_pair_bit_identical_random(seed):
    rng = np.random.default_rng(seed)
    rowptr, col, val = _random_csr(4000, 3000, 40, rng, hub_rows=(11, 1999), hub_deg=2900)
    ref, got, _, _, _ = _pair_vs_chunk(rowptr, col, val, 4000, 3000, 128, seed=seed)
    assert torch.equal(ref, got)


def test_pair_two_source_and_long_rows_vs_oracle():
    rng = np.random.default_rng(5)
    n_rows, B, n2 = 3000, 1800, 1200
    n_cols = B + n2
    deg = rng.integers(0, 30, size=n_rows)
    deg[100:140] = rng.integers(257, 900, size=40)
    rowptr = np.zeros(n_rows + 1, np.int64)
    rowptr[1:] = np.cumsum(deg)
    col = np.concatenate([np.sort(rng.choice(n_cols, size=d, replace=False)) for d in deg])
    val = rng.standard_normal(col.shape[0]).astype(np.float32)
    ref, got, _, X, X2 = _pair_vs_chunk(rowptr, col, val, n_rows, n_cols, 128, B=B, x2_rows=n2)
    assert torch.equal(ref, got)
    xin = np.concatenate([X.cpu().numpy(), X2.cpu().numpy()])
    exact = conv_ref.spmm_seq(rowptr, col, val, xin)
    short = np.diff(rowptr) <= 256
    assert np.array_equal(got.cpu().numpy()[short], exact[short])
    f64 = conv_ref.spmm_fp64(rowptr, col, val, xin)
    scale = conv_ref.spmm_fp64(rowptr, col, np.abs(val), np.abs(xin)) + 1e-6
    assert np.max(np.abs(got.cpu().numpy() - f64) / scale) < 1e-5


def test_pair_empty_rows_and_tiny():
    rowptr = [0, 0, 2, 2, 3, 3, 3]
    ref, got, _, _, _ = _pair_vs_chunk(rowptr, [1, 4, 9], [1.0, 2.0, 3.0], 6, 10, 128)
    assert torch.equal(ref, got)
    assert torch.count_nonzero(got[[0, 2, 4, 5]]) == 0


def test_pair_far_apart_falls_back():
    """X and X2 more than 4 GiB apart: the pair call runs the chunk kernels."""
    rng = np.random.default_rng(9)
    B, n2 = 500, 300
    rowptr, col, val = _random_csr(800, B + n2, 20, rng)
    a = _dev_csr(rowptr, col, val, 800, B + n2)
    X = torch.randn(B, 128, device=DEV)
    gap = torch.empty(5 << 30, dtype=torch.uint8, device=DEV)
    X2 = torch.randn(n2, 128, device=DEV)
    if abs(X2.data_ptr() - X.data_ptr()) < (4 << 30):
        pytest.skip("allocator placed the buffers close together")
    pp = a.plan(128, B=B)
    got = kernels.spmm(a.rowptr, a.col, a.value, 800, a.nnz(), X, 128, X2=X2, B=B, plan=pp)
    chunk = kernels.spmm_plan(a.rowptr, 800, a.nnz(), 128)
    ref = kernels.spmm(a.rowptr, a.col, a.value, 800, a.nnz(), X, 128, X2=X2, B=B, plan=chunk)
    del gap
    assert torch.equal(ref, got)


def test_pair_arxiv_batch_bit_identical():
    cfg = graph.CONFIGS["arxiv_gcn"]
    _, _, b = graph.make_batch(cfg)
    _, _, adj = graph.batch_to_device(b, DEV)
    F = 128
    X = torch.randn(b.B, F, device=DEV)
    X2 = torch.randn(b.n - b.B, F, device=DEV)
    pp = kernels.spmm_pair_plan(adj.rowptr, b.n, b.nnz, F, b.B)
    got = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=X2, B=b.B, plan=pp)
    chunk = kernels.spmm_plan(adj.rowptr, b.n, b.nnz, F)
    ref = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=X2, B=b.B, plan=chunk)
    assert torch.equal(ref, got)
