"""Tiled SpMM (include/vqgnn.h §6f, csrc/spmm_tiles.hip): dense (256-row x
128-column) blocks staged in LDS + the sparse remainder through the task
kernel in accumulate mode.  Checked against an fp64 sum of the same product
(north_star: fp32 messages within 1e-5 relative, here of each row's sum of
|w x|), run-to-run bit identity, the plan's edge partition, and the edge
cases: rows and columns not multiples of 256, empty rows, F not a multiple of
the 64-float slice, two sources, a non-finite value in an unreferenced row."""
import numpy as np
import pytest
import torch

from vq_gnn_amd import graph, kernels
from vq_gnn_amd.sparse import CSR

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _blocky(N=5000, parts=5, edges=400_000, seed=0, conv="GCN"):
    g = graph.synthetic_graph(N, parts, edges, seed=seed)
    rp, cl, vl = graph.norm_adj(g, conv)
    return rp, cl, vl, g.N


def _fp64_check(out, rp, cl, vl, xin, rows=None):
    rp, cl = rp.cpu().numpy().astype(np.int64), cl.cpu().numpy().astype(np.int64)
    vl = vl.cpu().double().numpy()
    x = xin.cpu().double().numpy()
    o = out.cpu().double().numpy()
    rows = range(len(rp) - 1) if rows is None else rows
    worst = 0.0
    for r in rows:
        s, e = rp[r], rp[r + 1]
        contrib = vl[s:e, None] * x[cl[s:e]]
        ref = contrib.sum(0)
        mag = np.abs(contrib).sum(0)
        err = np.abs(o[r] - ref) / (mag + 1e-30)
        if e == s:
            assert np.all(o[r] == 0), r
        else:
            worst = max(worst, float(err.max()))
    return worst


@pytest.mark.parametrize("F,B", [(128, None), (604, 1700), (36, 900)])
def test_tile_spmm_vs_fp64(F, B):
    rp, cl, vl, N = _blocky()
    adj = CSR(torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vl), (N, N)).to(DEV)
    plan = adj.plan(F, B=B, kind="tile")
    assert isinstance(plan, kernels.TilePlan), "blocky graph should take the tiled plan"
    assert plan.n_dense > 0 and plan.dense_edges + plan.s_nnz == adj.nnz()
    assert plan.dense_edges > 0.5 * adj.nnz()
    gen = torch.Generator().manual_seed(F)
    if B is None:
        X = torch.randn(N, F, generator=gen).to(DEV)
        out = kernels.spmm(adj.rowptr, adj.col, adj.value, N, adj.nnz(), X, F, plan=plan)
        out2 = kernels.spmm(adj.rowptr, adj.col, adj.value, N, adj.nnz(), X, F, plan=plan)
        xin = X
    else:
        X = torch.randn(B, F, generator=gen).to(DEV)
        X2 = torch.randn(N - B, F, generator=gen).to(DEV)
        out = kernels.spmm(adj.rowptr, adj.col, adj.value, N, adj.nnz(), X, F, X2=X2, B=B,
                           plan=plan)
        out2 = kernels.spmm(adj.rowptr, adj.col, adj.value, N, adj.nnz(), X, F, X2=X2, B=B,
                            plan=plan)
        xin = torch.cat([X, X2])
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    rows = list(range(0, N, 7)) + list(range(N - 300, N))
    err = _fp64_check(out, adj.rowptr, adj.col, adj.value, xin, rows)
    assert err < 1e-5, f"F={F}: rel err {err:.2e}"
    # the task kernel alone gives the same product within the tolerance
    tp = adj.plan(F, B=B, kind="task")
    ref = kernels.spmm(adj.rowptr, adj.col, adj.value, N, adj.nnz(), X, F,
                       X2=None if B is None else X2, B=B, plan=tp)
    scale = (xin.abs().max() * adj.value.abs().max() * 600).item()
    assert (out - ref).abs().max().item() < 1e-5 * scale


def test_tile_plan_partitions_the_edges():
    """Decoded dense records + the sparse CSR = the input edges, each once,
    with the original weights; padding records are (zero row, weight 0)."""
    rp, cl, vl, N = _blocky(N=2600, parts=2, edges=200_000, seed=2)
    # empty rows: drop every edge of rows 5, 600..610 and the last row
    keep_rows = np.ones(N, bool)
    keep_rows[[5, *range(600, 611), N - 1]] = False
    row = np.repeat(np.arange(N), np.diff(rp))
    m = keep_rows[row]
    row, cl, vl = row[m], cl[m], vl[m]
    rp = np.zeros(N + 1, np.int64)
    rp[1:] = np.cumsum(np.bincount(row, minlength=N))
    adj = CSR(torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vl), (N, N)).to(DEV)
    plan = adj.plan(64, kind="tile")
    assert isinstance(plan, kernels.TilePlan)
    blocks = plan.blocks.cpu().numpy()
    rowptr_b = plan.rowptr_b.cpu().numpy().reshape(-1, 257)
    boff = plan.boff.cpu().numpy()
    drec = plan.drec.cpu().numpy()
    got = []
    for b in range(plan.n_dense):
        key = blocks[b]
        w, t = key // plan.T, key % plan.T
        for ri in range(256):
            lo, hi = boff[b] + rowptr_b[b, ri], boff[b] + rowptr_b[b, ri + 1]
            assert (hi - lo) % 4 == 0
            for rec in drec[lo:hi]:
                c = int(rec & 0xFFFFFFFF)
                wbits = np.uint32((int(rec) >> 32) & 0xFFFFFFFF)
                if c == plan.C:
                    assert wbits == 0
                    continue
                assert 0 <= c < plan.C
                got.append((w * 256 + ri, t * plan.C + c, wbits.view(np.float32)))
    srp = plan.s_rowptr.cpu().numpy()
    scl = plan.s_col.cpu().numpy()[:plan.s_nnz]
    svl = plan.s_val.cpu().numpy()[:plan.s_nnz]
    srow = np.repeat(np.arange(N), np.diff(srp))
    got += list(zip(srow.tolist(), scl.tolist(), svl.tolist()))
    got.sort()
    ref = sorted(zip(row.tolist(), cl.tolist(), vl.tolist()))
    assert len(got) == len(ref)
    assert got == ref
    # and the product with the empty rows (zeros)
    X = torch.randn(N, 64, device=DEV)
    out = kernels.spmm(adj.rowptr, adj.col, adj.value, N, adj.nnz(), X, 64, plan=plan)
    assert _fp64_check(out, adj.rowptr, adj.col, adj.value, X) < 1e-5


def test_tile_nonfinite_unreferenced_row():
    """A source row no edge reads may hold inf/NaN: the padding records read
    the LDS zero row, so no 0 * inf reaches any output."""
    rp, cl, vl, N = _blocky(N=2000, parts=2, edges=150_000, seed=4)
    # row 7 is never a column: drop every edge into node 7
    row = np.repeat(np.arange(N), np.diff(rp))
    m = cl != 7
    row, cl, vl = row[m], cl[m], vl[m]
    rp = np.zeros(N + 1, np.int64)
    rp[1:] = np.cumsum(np.bincount(row, minlength=N))
    adj = CSR(torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vl), (N, N)).to(DEV)
    plan = adj.plan(64, kind="tile")
    assert isinstance(plan, kernels.TilePlan)
    X = torch.randn(N, 64, device=DEV)
    X[7] = float("inf")
    X[7, 3] = float("nan")
    out = kernels.spmm(adj.rowptr, adj.col, adj.value, N, adj.nnz(), X, 64, plan=plan)
    assert torch.isfinite(out).all()
