"""GPU parity of the hot-column tile SpMM (include/vqgnn.h §6h, the default
GCN/SAGE aggregation) against the fp64 sum (every row within 1e-5 of
sum |w| |x|: north_star's fp32 messages within 1e-5 relative) and against the
task kernel (§6): a row the plans do not cut is the same fma chain in CSR
order in both kernels, so it must be bit-identical whichever rows are hot.
Ragged, empty, hub, two-source, partial-slice, leading-row and far-address
inputs; the plan's hot sets checked against the tile's column counts."""
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


def _clustered_csr(n_rows, n_cols, rng, hubs=40, deg_hi=24, hub_rows=()):
    """Rows whose columns concentrate on a few hub columns per 300-row band
    (what a cluster batch looks like), plus uniform columns and empty rows."""
    deg = rng.integers(0, deg_hi, size=n_rows)
    deg[rng.random(n_rows) < 0.08] = 0
    for r, d in hub_rows:
        deg[r] = d
    cols = []
    for r in range(n_rows):
        d = int(deg[r])
        band = (r // 300) * 300 % max(n_cols - hubs, 1)
        hot = band + rng.integers(0, hubs, size=d)
        uni = rng.integers(0, n_cols, size=d)
        c = np.where(rng.random(d) < 0.7, np.minimum(hot, n_cols - 1), uni)
        cols.append(np.unique(c))
    deg = np.array([c.size for c in cols])
    rowptr = np.zeros(n_rows + 1, np.int64)
    rowptr[1:] = np.cumsum(deg)
    col = np.concatenate(cols).astype(np.int64) if rowptr[-1] else np.zeros(0, np.int64)
    val = rng.standard_normal(col.shape[0]).astype(np.float32)
    return rowptr, col, val


def _check(out, rowptr, col, val, xin, n_rows=None):
    n = rowptr.size - 1 if n_rows is None else n_rows
    rp = rowptr[: n + 1]
    ref = conv_ref.spmm_fp64(rp, col[: rp[-1]], val[: rp[-1]], xin)
    scale = conv_ref.spmm_fp64(rp, col[: rp[-1]], np.abs(val[: rp[-1]]), np.abs(xin))
    o = out[:n].cpu().numpy().astype(np.float64)
    err = np.abs(o - ref)
    assert (err <= 1e-5 * scale + 1e-30).all(), f"max rel err {(err / (scale + 1e-30)).max():.3e}"
    assert np.all(o[np.diff(rp) == 0] == 0)


def _both(a, X, F, X2=None, B=None, n_rows=None, K=64, Et=None, C=None, n_cols=None):
    nr = a.size(0) if n_rows is None else n_rows
    hp = kernels.spmm_hot_plan(a.rowptr, a.col, a.value, a.size(0), a.nnz(),
                               n_cols=a.size(1) if n_cols is None else n_cols, K=K, Et=Et, C=C)
    tp = kernels.spmm_task_plan(a.rowptr, a.col, a.value, a.size(0), a.nnz(), K)
    hot = kernels.spmm(a.rowptr, a.col, a.value, nr, a.nnz(), X, F, X2=X2, B=B, plan=hp)
    task = kernels.spmm(a.rowptr, a.col, a.value, nr, a.nnz(), X, F, X2=X2, B=B, plan=tp)
    return hot, task, hp


def _uncut_equal(hot, task, rowptr, K, n_rows=None):
    n = hot.shape[0] if n_rows is None else n_rows
    short = torch.as_tensor(np.diff(rowptr[: n + 1]) <= K // 2, device=DEV)
    assert torch.equal(hot[:n][short], task[:n][short]), "uncut rows differ from the task kernel"


@pytest.mark.parametrize("F", [4, 32, 36, 128, 256, 604])
@pytest.mark.parametrize("Et,C", [(16384, 1024), (512, 64), (128, 4), (256, 0)])
def test_hot_spmm_vs_fp64_and_task(F, Et, C):
    rng = np.random.default_rng(F * 7 + Et + C)
    rowptr, col, val = _clustered_csr(1500, 1800, rng,
                                      hub_rows=((3, 700), (700, 1300), (1499, 257)))
    x = rng.standard_normal((1800, F)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, 1500, 1800)
    xd = torch.from_numpy(x).to(DEV)
    hot, task, hp = _both(a, xd, F, Et=Et, C=C)
    _check(hot, rowptr, col, val, x)
    _uncut_equal(hot, task, rowptr, 64)
    again = kernels.spmm(a.rowptr, a.col, a.value, 1500, a.nnz(), xd, F, plan=hp)
    assert torch.equal(hot, again)                  # deterministic


def test_hot_plan_hot_sets():
    """Per tile: at most C hot rows, distinct, each referenced at least twice
    by the tile's edges, and no column left out that is referenced more often
    than one taken (the selection is by count)."""
    rng = np.random.default_rng(3)
    rowptr, col, val = _clustered_csr(3000, 2500, rng, hub_rows=((10, 900),))
    a = _dev_csr(rowptr, col, val, 3000, 2500)
    for Et, C in ((4096, 256), (1024, 16), (16384, 1024)):
        hp = kernels.spmm_hot_plan(a.rowptr, a.col, a.value, 3000, a.nnz(), n_cols=2500, Et=Et,
                                   C=C)
        tile_row, tile_task, hot_n, hot = (t.numpy() for t in hp.tile_info())
        assert tile_row[0] == 0 and tile_row[-1] == 3000 and (np.diff(tile_row) >= 0).all()
        assert (np.diff(tile_task) >= 0).all()
        taken = 0
        for t in range(hot_n.size):
            e0, e1 = rowptr[tile_row[t]], rowptr[tile_row[t + 1]]
            cnt = np.bincount(col[e0:e1], minlength=2500)
            h = hot[t, :hot_n[t]]
            assert hot_n[t] <= C and np.unique(h).size == h.size
            if h.size:
                assert cnt[h].min() >= 2
                left = np.setdiff1d(np.nonzero(cnt >= 2)[0], h)
                if left.size:
                    assert cnt[left].max() <= cnt[h].min()
                taken += cnt[h].sum()
            else:
                assert C == 0 or (cnt >= 2).sum() == 0
        if C >= 256:
            assert taken > 0.3 * a.nnz()               # the clustered rows do reuse columns


def test_hot_spmm_two_sources_strides_and_leading_rows():
    rng = np.random.default_rng(5)
    B, n2, F = 1200, 900, 128
    rowptr, col, val = _clustered_csr(B + n2, B + n2, rng)
    X = torch.randn(B, F + 12, device=DEV)[:, 4:4 + F]           # ld = F + 12
    X2 = torch.randn(n2, F, device=DEV)
    a = _dev_csr(rowptr, col, val, B + n2, B + n2)
    hp = kernels.spmm_hot_plan(a.rowptr, a.col, a.value, B + n2, a.nnz(), Et=1024, C=128)
    out = torch.full((B + n2, F + 8), 7.0, device=DEV)[:, :F]     # ldo = F + 8
    kernels.spmm(a.rowptr, a.col, a.value, B + n2, a.nnz(), X, F, X2=X2, B=B, out=out, plan=hp)
    xin = torch.cat([X, X2]).cpu().numpy()
    _check(out, rowptr, col, val, xin)
    # the first 1,000 rows only (the backward's batch rows of A^T): rows past
    # them untouched
    part = torch.full((1000, F), 5.0, device=DEV)
    kernels.spmm(a.rowptr, a.col, a.value, 1000, a.nnz(), X, F, X2=X2, B=B, out=part, plan=hp)
    _check(part, rowptr, col, val, xin, n_rows=1000)


def test_hot_spmm_far_path_matches_near():
    rng = np.random.default_rng(6)
    B, n2, F = 800, 700, 64
    rowptr, col, val = _clustered_csr(B + n2, B + n2, rng)
    a = _dev_csr(rowptr, col, val, B + n2, B + n2)
    X, X2 = torch.randn(B, F, device=DEV), torch.randn(n2, F, device=DEV)
    hp = kernels.spmm_hot_plan(a.rowptr, a.col, a.value, B + n2, a.nnz(), Et=1024, C=64)
    near = kernels.spmm(a.rowptr, a.col, a.value, B + n2, a.nnz(), X, F, X2=X2, B=B, plan=hp)
    os.environ["VQGNN_SPMM_FAR"] = "1"
    try:
        far = kernels.spmm(a.rowptr, a.col, a.value, B + n2, a.nnz(), X, F, X2=X2, B=B, plan=hp)
    finally:
        del os.environ["VQGNN_SPMM_FAR"]
    assert torch.equal(near, far)


def test_hot_spmm_empty_runs_and_degenerate():
    rng = np.random.default_rng(7)
    deg = rng.integers(1, 9, size=600)
    deg[50:120] = 0            # 70 consecutive empty rows: the skip-count escape
    deg[200:230] = 0
    deg[-40:] = 0              # trailing empty rows (eval adjacency)
    deg[:3] = 0
    rowptr = np.zeros(601, np.int64)
    rowptr[1:] = np.cumsum(deg)
    col = np.concatenate([np.sort(rng.choice(60, size=d, replace=False)) for d in deg])
    val = rng.standard_normal(col.size).astype(np.float32)
    x = rng.standard_normal((300, 32)).astype(np.float32)
    a = _dev_csr(rowptr, col, val, 600, 300)
    hot, task, _ = _both(a, torch.from_numpy(x).to(DEV), 32, K=8, Et=64, C=16)
    _check(hot, rowptr, col, val, x)
    _uncut_equal(hot, task, rowptr, 8)
    z = _dev_csr([0, 0, 0, 0], [], [], 3, 10)
    hp = kernels.spmm_hot_plan(z.rowptr, z.col, z.value, 3, 0, n_cols=10)
    out = kernels.spmm(z.rowptr, z.col, z.value, 3, 0, torch.randn(10, 8, device=DEV), 8,
                       plan=hp)
    assert torch.count_nonzero(out) == 0
    one = _dev_csr([0, 2], [2, 2 + 0], [3.0, 0.5], 1, 5)
    xx = torch.randn(5, 4, device=DEV)
    hp = kernels.spmm_hot_plan(one.rowptr, one.col, one.value, 1, 2, n_cols=5)
    got = kernels.spmm(one.rowptr, one.col, one.value, 1, 2, xx, 4, plan=hp)[0]
    x2 = xx[2].double().cpu().numpy()
    ref = (0.5 * x2 + (3.0 * x2).astype(np.float32)).astype(np.float32)   # fma(0.5, x, 3x)
    assert np.array_equal(got.cpu().numpy(), ref)


def test_hot_plan_with_values():
    """Other weights on the same structure (GAT coefficients on the
    transpose): the same tiles and hot slots with the weights replaced equal
    a fresh plan over those weights, bit for bit."""
    rng = np.random.default_rng(9)
    rowptr, col, val = _clustered_csr(1000, 1000, rng)
    a = _dev_csr(rowptr, col, val, 1000, 1000)
    hp = kernels.spmm_hot_plan(a.rowptr, a.col, a.value, 1000, a.nnz(), Et=2048, C=128)
    w2 = torch.randn(a.nnz(), device=DEV)
    x = torch.randn(1000, 64, device=DEV)
    got = kernels.spmm(a.rowptr, a.col, w2, 1000, a.nnz(), x, 64, plan=hp.with_values(a.col, w2))
    fresh = kernels.spmm_hot_plan(a.rowptr, a.col, w2, 1000, a.nnz(), Et=2048, C=128)
    ref = kernels.spmm(a.rowptr, a.col, w2, 1000, a.nnz(), x, 64, plan=fresh)
    assert torch.equal(got, ref)
    with pytest.raises(ValueError, match="other values"):
        kernels.spmm(a.rowptr, a.col, a.value, 1000, a.nnz(), x, 64, plan=hp.with_values(a.col, w2))


def test_hot_spmm_arxiv_batch_vs_fp64_and_task():
    """The bench batch (arxiv GCN, 2.07 M edges, two sources): within 1e-5 of
    fp64, uncut rows bit-identical to the task kernel, deterministic."""
    g, _, b = graph.make_batch(graph.CONFIGS["arxiv_gcn"])
    F = 128
    bidx, subset, adj = graph.batch_to_device(b, DEV)
    X = torch.randn(b.B, F, device=DEV)
    X2 = torch.randn(b.n - b.B, F, device=DEV)
    hot, task, hp = _both(adj, X, F, X2=X2, B=b.B)
    xin = torch.cat([X, X2]).cpu().numpy()
    _check(hot, b.rowptr, b.col, b.val, xin)
    _uncut_equal(hot, task, b.rowptr, 64)
    again = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=X2, B=b.B, plan=hp)
    assert torch.equal(hot, again)
    _, _, hot_n, _ = hp.tile_info()
    assert int(hot_n.sum()) > 0
