"""GPU parity of the task-split SpMM (include/vqgnn.h §6e, the default
aggregation kernel) against the fp64 sum: every row within 1e-5 of
sum |w| |x| (north_star: fp32 messages within 1e-5 relative), on ragged,
empty, hub and two-source inputs; deterministic across calls."""
import os

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


def _csr_from_deg(deg, n_cols, rng):
    rowptr = np.zeros(deg.size + 1, np.int64)
    rowptr[1:] = np.cumsum(deg)
    col = np.concatenate([np.sort(rng.choice(n_cols, size=d, replace=d > n_cols))
                          for d in deg]) if rowptr[-1] else np.zeros(0, np.int64)
    val = rng.standard_normal(col.shape[0]).astype(np.float32)
    return rowptr, col.astype(np.int64), val


def _check(out, rowptr, col, val, xin, n_rows=None):
    n = rowptr.size - 1 if n_rows is None else n_rows
    rp = rowptr[: n + 1]
    ref = conv_ref.spmm_fp64(rp, col[: rp[-1]], val[: rp[-1]], xin)
    scale = conv_ref.spmm_fp64(rp, col[: rp[-1]], np.abs(val[: rp[-1]]), np.abs(xin))
    o = out.cpu().numpy().astype(np.float64)
    err = np.abs(o - ref)
    assert (err <= 1e-5 * scale + 1e-30).all(), f"max rel err {(err / (scale + 1e-30)).max():.3e}"
    empty = np.diff(rp) == 0
    assert np.all(o[empty] == 0)


def _run(a, X, F, X2=None, B=None, n_rows=None, K=None):
    plan = kernels.spmm_task_plan(a.rowptr, a.col, a.value, a.size(0), a.nnz(), K)
    nr = a.size(0) if n_rows is None else n_rows
    return kernels.spmm(a.rowptr, a.col, a.value, nr, a.nnz(), X, F, X2=X2, B=B, plan=plan)


@pytest.mark.parametrize("F", [4, 8, 16, 32, 64, 124, 128, 132, 256, 604])
@pytest.mark.parametrize("K", [8, 64, 256])
def test_task_spmm_ragged_vs_fp64(F, K):
    rng = np.random.default_rng(F * 31 + K)
    deg = rng.integers(0, 24, size=900)
    deg[rng.random(900) < 0.1] = 0
    deg[[3, 450, 899]] = [700, 1300, 257]          # rows spanning many tasks
    rowptr, col, val = _csr_from_deg(deg, 1100, rng)
    x = rng.standard_normal((1100, F)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, 900, 1100)
    xd = torch.from_numpy(x).to(DEV)
    out = _run(a, xd, F, K=K)
    _check(out, rowptr, col, val, x)
    again = _run(a, xd, F, K=K)
    assert torch.equal(out, again)                 # deterministic


def test_task_spmm_two_sources_and_strides():
    rng = np.random.default_rng(5)
    B, n2, F = 700, 500, 128
    deg = rng.integers(1, 40, size=B + n2)
    rowptr, col, val = _csr_from_deg(deg, B + n2, rng)
    X = torch.randn(B, F + 12, device=DEV)[:, 4:4 + F]       # ld = F + 12
    X2 = torch.randn(n2, F, device=DEV)
    out = torch.full((B + n2, F + 8), 7.0, device=DEV)[:, :F]  # ldo = F + 8
    a = _dev_csr(rowptr, col, val, B + n2, B + n2)
    plan = kernels.spmm_task_plan(a.rowptr, a.col, a.value, B + n2, a.nnz())
    kernels.spmm(a.rowptr, a.col, a.value, B + n2, a.nnz(), X, F, X2=X2, B=B, out=out, plan=plan)
    xin = torch.cat([X, X2]).cpu().numpy()
    _check(out, rowptr, col, val, xin)


def test_task_spmm_far_path_matches_near():
    rng = np.random.default_rng(6)
    B, n2, F = 600, 400, 64
    rowptr, col, val = _csr_from_deg(rng.integers(0, 30, size=B + n2), B + n2, rng)
    a = _dev_csr(rowptr, col, val, B + n2, B + n2)
    X, X2 = torch.randn(B, F, device=DEV), torch.randn(n2, F, device=DEV)
    near = _run(a, X, F, X2=X2, B=B)
    os.environ["VQGNN_SPMM_FAR"] = "1"
    try:
        far = _run(a, X, F, X2=X2, B=B)
    finally:
        del os.environ["VQGNN_SPMM_FAR"]
    assert torch.equal(near, far)


def test_task_spmm_empty_runs_and_degenerate():
    rng = np.random.default_rng(7)
    deg = rng.integers(1, 9, size=400)
    deg[50:120] = 0            # 70 consecutive empty rows: the skip-count escape
    deg[200:230] = 0           # 30: below the escape
    deg[-40:] = 0              # trailing empty rows (eval adjacency)
    deg[:3] = 0                # leading
    rowptr, col, val = _csr_from_deg(deg, 300, rng)
    x = rng.standard_normal((300, 32)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, 400, 300)
    _check(_run(a, torch.from_numpy(x).to(DEV), 32, K=8), rowptr, col, val, x)
    z = _dev_csr([0, 0, 0, 0], [], [], 3, 10)
    out = _run(z, torch.randn(10, 8, device=DEV), 8)
    assert torch.count_nonzero(out) == 0
    one = _dev_csr([0, 1], [2], [3.0], 1, 5)
    xx = torch.randn(5, 4, device=DEV)
    assert torch.equal(_run(one, xx, 4)[0], 3.0 * xx[2])


def test_task_spmm_leading_rows_of_planned_csr():
    """A call over the first n_rows rows (the backward's batch rows of A^T)
    uses the plan of the whole CSR and writes only those rows."""
    rng = np.random.default_rng(8)
    rowptr, col, val = _csr_from_deg(rng.integers(0, 50, size=1000), 800, rng)
    a = _dev_csr(rowptr, col, val, 1000, 800)
    x = rng.standard_normal((800, 128)).astype(np.float32)
    plan = kernels.spmm_task_plan(a.rowptr, a.col, a.value, 1000, a.nnz())
    out = torch.full((600, 128), 5.0, device=DEV)
    kernels.spmm(a.rowptr, a.col, a.value, 600, a.nnz(), torch.from_numpy(x).to(DEV), 128,
                 out=out, plan=plan)
    _check(out, rowptr, col, val, x, n_rows=600)


def test_task_spmm_arxiv_batch_vs_fp64():
    cfg = dict(graph.CONFIGS["arxiv_gcn"])
    g, _, b = graph.make_batch(cfg)
    F = 128
    bidx, subset, adj = graph.batch_to_device(b, DEV)
    X = torch.randn(b.B, F, device=DEV)
    X2 = torch.randn(b.n - b.B, F, device=DEV)
    task = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=X2, B=b.B,
                        plan=adj.plan(F, B=b.B))
    again = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=X2, B=b.B,
                         plan=adj.plan(F, B=b.B))
    xin = torch.cat([X, X2]).cpu().numpy()
    _check(task, b.rowptr, b.col, b.val, xin)
    assert torch.equal(task, again)


def test_task_plan_rejects_other_values():
    a = _dev_csr([0, 2, 3], [0, 1, 1], [1.0, 2.0, 3.0], 2, 2)
    plan = a.plan(4)
    with pytest.raises(ValueError, match="other values"):
        kernels.spmm(a.rowptr, a.col, a.value * 2, 2, 3, torch.randn(2, 4, device=DEV), 4,
                     plan=plan)


def _cb_case(rng, B, n, N, F, M, D, deg_hi=40, K=None):
    """A layer-shaped case for the codebook-source SpMM: CSR over n = B + B'
    rows, subset (batch nodes first), c_indices [N, nb], emb_out [nb, M, 2D]."""
    nb = F // D
    deg = rng.integers(0, deg_hi, size=n)
    deg[rng.random(n) < 0.05] = 0
    rowptr, col, val = _csr_from_deg(deg, n, rng)
    a = _dev_csr(rowptr, col, val, n, n)
    subset = torch.from_numpy(rng.permutation(N)[:n].astype(np.int64)).to(DEV)
    codes = torch.from_numpy(rng.integers(0, M, size=(N, nb)).astype(np.int16)).to(DEV)
    emb_out = torch.randn(nb, M, 2 * D, device=DEV)
    X = torch.randn(B, F, device=DEV)
    plan = kernels.spmm_task_plan(a.rowptr, a.col, a.value, n, a.nnz(), K)
    return a, rowptr, col, val, subset, codes, emb_out, X, plan


@pytest.mark.parametrize("B,n,K", [(700, 1200, 64), (0, 900, 8), (900, 900, 64), (1, 1000, 256)])
def test_codebook_source_equals_gather_and_two_source(B, n, K):
    """vqgnn_spmm_task_cb (include/vqgnn.h §6b) against gather_codewords +
    the two-source task SpMM: the same records and fma chain, so the same
    floats; and within 1e-5 of the fp64 sum.  B = 0 (every column from the
    codebook) and B = n (none) included."""
    rng = np.random.default_rng(B * 7 + n)
    F, M, D, N = 128, 256, 4, 5000
    a, rowptr, col, val, subset, codes, emb_out, X, plan = _cb_case(rng, B, n, N, F, M, D, K=K)
    xf, _ = kernels.gather_codewords(subset, B, codes, emb_out, D)
    if B == 0:
        ref = kernels.spmm(a.rowptr, a.col, a.value, n, a.nnz(), xf, F, plan=plan)
    elif B == n:
        ref = kernels.spmm(a.rowptr, a.col, a.value, n, a.nnz(), X, F, plan=plan)
    else:
        ref = kernels.spmm(a.rowptr, a.col, a.value, n, a.nnz(), X, F, X2=xf, B=B, plan=plan)
    pcb = plan.with_codebook_source(B, subset, N)
    Xs = X if B > 0 else torch.zeros(1, F, device=DEV)
    out = kernels.spmm_codebook(a.rowptr, n, a.nnz(), Xs, F, B, codes, emb_out, D, pcb)
    assert torch.equal(out, ref)
    xin = torch.cat([X, xf]).cpu().numpy()
    _check(out, rowptr, col, val, xin)


def test_codebook_source_arxiv_batch_and_strides():
    """The bench batch (arxiv_gcn, M = 256, nb = 32): equal to gather +
    two-source on a strided X, codes (c_indices view with ld 35 > nb, as a
    column slice of a wider code table) and output, deterministic, and within
    1e-5 of the fp64 sum (the gather once took nb from the
    codes' 35 columns and read past the 32-branch codebook)."""
    cfg = dict(graph.CONFIGS["arxiv_gcn"])
    g, _, b = graph.make_batch(cfg)
    F, M, D = 128, cfg["M"], 4
    nb = F // D
    bidx, subset, adj = graph.batch_to_device(b, DEV)
    gen = torch.Generator(device="cpu").manual_seed(11)
    wide = torch.randint(0, M, (cfg["N"], nb + 3), dtype=torch.int16, generator=gen).to(DEV)
    codes = wide[:, :nb]                                     # ld = nb + 3
    emb_out = torch.randn(nb, M, 2 * D, generator=gen).to(DEV)
    X = torch.randn(b.B, F + 8, generator=gen).to(DEV)[:, 4:4 + F]
    xf, _ = kernels.gather_codewords(subset, b.B, codes, emb_out, D)
    assert xf.shape == (b.n - b.B, F)
    # the wide table through the gather: nb comes from the codebook (32), not
    # from the table's 35 columns, so the same rows
    xf_wide, _ = kernels.gather_codewords(subset, b.B, wide, emb_out, D)
    assert torch.equal(xf, xf_wide)
    ref = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=xf, B=b.B,
                       plan=adj.plan(F, B=b.B))
    out = torch.full((b.n, F + 4), 3.0, device=DEV)[:, :F]
    pcb = adj.plan_codebook(b.B, subset, cfg["N"])
    kernels.spmm_codebook(adj.rowptr, b.n, b.nnz, X, F, b.B, codes, emb_out, D, pcb, out=out)
    assert torch.equal(out, ref)
    again = kernels.spmm_codebook(adj.rowptr, b.n, b.nnz, X, F, b.B, codes, emb_out, D, pcb)
    assert torch.equal(again, ref)
    # the codewords of every out-of-batch row, restated on the host from the
    # codes (models.py:168-173), then the fp64 sum (convs.py:95)
    sub = subset.cpu().numpy()
    cod = codes.cpu().numpy().astype(np.int64)
    emb = emb_out.cpu().numpy()
    xf_host = emb[np.arange(nb)[None, :], cod[sub[b.B:]], :D].reshape(b.n - b.B, F)
    assert np.array_equal(xf.cpu().numpy(), xf_host)
    xin = np.concatenate([X.cpu().numpy(), xf_host])
    _check(out, b.rowptr, b.col, b.val, xin)


@pytest.mark.parametrize("F,M,G", [(128, 512, 16), (128, 1024, 8), (64, 639, 16), (96, 1279, 8),
                                   (32, 300, 8)])
def test_codebook_source_narrow_tiles(F, M, G):
    """Codebooks too large for a 128-column image (M > 319) walk narrower
    column tiles of 4G columns (include/vqgnn.h §6b; reddit / arxiv-GAT use M =
    1,024): bit-identical to gather + two-source SpMM and within 1e-5 of the
    fp64 sum, hub rows and empty rows included."""
    rng = np.random.default_rng(F + M)
    B, n, N, D = 600, 1500, 4000, 4
    a, rowptr, col, val, subset, codes, emb_out, X, plan = _cb_case(rng, B, n, N, F, M, D)
    assert kernels.codebook_source_ok(X, F, M, D, codes=codes, n_rows=n, n_branches=F // D)
    if F % 128 == 0 or M > 319:        # (the query gives the widest tile M alone allows)
        assert kernels.lib().vqgnn_spmm_task_cb_lds(M) == (M + 1) * 16 * G   # + the zero row
    xf, _ = kernels.gather_codewords(subset, B, codes, emb_out, D)
    ref = kernels.spmm(a.rowptr, a.col, a.value, n, a.nnz(), X, F, X2=xf, B=B, plan=plan)
    out = kernels.spmm_codebook(a.rowptr, n, a.nnz(), X, F, B, codes, emb_out, D,
                                plan.with_codebook_source(B, subset, N))
    assert torch.equal(out, ref)
    _check(out, rowptr, col, val, torch.cat([X, xf]).cpu().numpy())


def test_codebook_source_rejects_unsupported():
    rng = np.random.default_rng(3)
    a, rowptr, col, val, subset, codes, emb_out, X, plan = _cb_case(rng, 50, 100, 300, 128, 256,
                                                                    4)
    pcb = plan.with_codebook_source(50, subset, 300)
    with pytest.raises(RuntimeError, match="M=1300"):           # no tile fits 1,300 codewords
        big = torch.randint(0, 1300, (300, 32), dtype=torch.int16, device=DEV)
        kernels.spmm_codebook(a.rowptr, 100, a.nnz(), X, 128, 50, big,
                              torch.randn(32, 1300, 8, device=DEV), 4, pcb)
    with pytest.raises(ValueError, match="with_codebook_source"):
        kernels.spmm_codebook(a.rowptr, 100, a.nnz(), X, 128, 50, codes, emb_out, 4, plan)
    X40 = torch.randn(50, 40, device=DEV)
    with pytest.raises(RuntimeError, match="multiple of 32"):
        kernels.spmm_codebook(a.rowptr, 100, a.nnz(), X40, 40, 50, codes[:, :10],
                              emb_out[:10], 4, pcb)
    # F / D = 32 code columns against a 16-branch codebook: rejected, no read
    with pytest.raises(RuntimeError, match="branches"):
        kernels.spmm_codebook(a.rowptr, 100, a.nnz(), X, 128, 50, codes, emb_out[:16], 4, pcb)
    with pytest.raises(ValueError, match="branches"):
        kernels.gather_codewords(subset, 50, codes, emb_out[:16], 4, nb=32)
    with pytest.raises(ValueError, match="columns"):
        kernels.gather_codewords(subset, 50, codes[:, :8], emb_out, 4)
    with pytest.raises(ValueError, match="int64"):
        plan.with_codebook_source(50, subset.to(torch.int32), 300)
    with pytest.raises(ValueError, match="columns"):
        a.plan().with_codebook_source(50, subset[:99], 300)
    # CodebookInput falls back to the gathered rows where the kernel cannot
    from vq_gnn_amd.convs import CodebookInput
    assert CodebookInput(X, subset, codes, emb_out, 4).supported(100)
    assert not CodebookInput(X, subset, codes, torch.randn(32, 1300, 8, device=DEV), 4).supported(100)
    assert not CodebookInput(X, subset, codes, emb_out[:16], 4).supported(100)


def test_gather_bad_nodes_and_codes_read_nothing():
    """A node outside [0, N) or a code outside [0, M) gives a zero row (and
    lcodes -1 for the node), never a read past codes / emb_out."""
    M, D, nb, N = 16, 4, 4, 10
    codes = torch.randint(0, M, (N, nb), dtype=torch.int16, device=DEV)
    codes[3, 2] = M + 5
    codes[4, 1] = -1
    emb_out = torch.randn(nb, M, 2 * D, device=DEV)
    subset = torch.tensor([0, 1, 3, 4, 10, -2, 7], dtype=torch.int64, device=DEV)
    xt, lc = kernels.gather_codewords(subset, 2, codes, emb_out, D, want_codes=True)
    xt, lc = xt.cpu(), lc.cpu()
    e = emb_out.cpu()
    for j, node in enumerate([3, 4, 10, -2, 7]):
        for br in range(nb):
            seg = xt[j, br * D:(br + 1) * D]
            if not 0 <= node < N:
                assert lc[j, br] == -1 and torch.count_nonzero(seg) == 0
                continue
            c = int(codes[node, br])
            assert lc[j, br] == c
            if 0 <= c < M:
                assert torch.equal(seg, e[br, c, :D])
            else:
                assert torch.count_nonzero(seg) == 0


def test_codebook_source_bad_nodes_and_codes_add_nothing():
    """through spmm_codebook an out-of-range node (weight 0 in the
    rewritten records) and a code outside [0, M) (the LDS image's zero row)
    contribute nothing -- the same output as gather_codewords (zero rows for
    both) + the two-source SpMM."""
    rng = np.random.default_rng(77)
    F, M, D, N, B, n = 128, 256, 4, 3000, 300, 800
    a, rowptr, col, val, subset, codes, emb_out, X, plan = _cb_case(rng, B, n, N, F, M, D)
    subset[B + 3] = N + 7                 # a node past the codes
    subset[B + 11] = -5                   # a negative node
    used = subset[B + 20:B + 40]
    codes[used[:10], 2] = M + 9           # codes past the codebook
    codes[used[10:], 5] = -3
    xf, _ = kernels.gather_codewords(subset, B, codes, emb_out, D)
    ref = kernels.spmm(a.rowptr, a.col, a.value, n, a.nnz(), X, F, X2=xf, B=B, plan=plan)
    got = kernels.spmm_codebook(a.rowptr, n, a.nnz(), X, F, B, codes, emb_out, D,
                                a.plan_codebook(B, subset, N))
    assert torch.equal(ref, got)
    assert torch.isfinite(got).all()


def test_codebook_plan_cache_follows_the_subset():
    """CSR.plan_codebook caches the rewritten records per subset tensor: an
    in-place change of the subset (or another tensor) rebuilds them."""
    rng = np.random.default_rng(21)
    F, M, D, N, B, n = 128, 256, 4, 3000, 300, 800
    a, rowptr, col, val, subset, codes, emb_out, X, plan = _cb_case(rng, B, n, N, F, M, D)

    def both():
        xf, _ = kernels.gather_codewords(subset, B, codes, emb_out, D)
        ref = kernels.spmm(a.rowptr, a.col, a.value, n, a.nnz(), X, F, X2=xf, B=B, plan=a.plan())
        got = kernels.spmm_codebook(a.rowptr, n, a.nnz(), X, F, B, codes, emb_out, D,
                                    a.plan_codebook(B, subset, N))
        return ref, got

    ref, got = both()
    assert torch.equal(ref, got)
    assert a.plan_codebook(B, subset, N) is a.plan_codebook(B, subset, N)
    subset[B:] = torch.from_numpy(rng.permutation(N)[:n - B].astype(np.int64)).to(DEV)
    ref2, got2 = both()
    assert not torch.equal(ref, ref2)
    assert torch.equal(ref2, got2)
