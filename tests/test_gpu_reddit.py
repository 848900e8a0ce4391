"""Reddit-shaped layers on the GPU (BASELINE.json configs[3], README.md:75):
the synthetic reddit graph (N = 232,965, 57.3 M undirected edges) and a
10,000-node batch built on the device (graph.make_batch_device: ~233 K rows,
~115 M edges), layer 1 at F = 604 (602 features zero-padded, 151 branches of
D = 4; vq_gnn_v2/utils/misc.py:212-216) and layer 2 at F = 128, M = 1024.

At full size: exact batch construction on sampled rows, bit-exact codeword
indices and BatchNorm state against the oracle (vq_ref.update on the full
batch, for a spread of branches), exact EMA count conservation, exact
codeword gather, the SpMM within 1e-5 of an fp64 sum on sampled rows
(including the longest rows) and run-to-run bit identity."""
import numpy as np
import pytest
import torch

from oracle import vq_ref
from vq_gnn_amd import kernels
from vq_gnn_amd.graph import CONFIGS, make_batch_device
from vq_gnn_amd.vq import VQBank

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
M, D = 1024, 4


@pytest.fixture(scope="module")
def reddit():
    graph, (bidx, subset, adj) = make_batch_device(CONFIGS["reddit_gcn_l1"], device=DEV)
    torch.cuda.synchronize()
    return graph, bidx, subset, adj


def test_reddit_batch_rows_exact(reddit):
    """Rows of the device batch == the full graph's edges among the subset,
    relabelled, sorted by column (dataloader.py:98-148, misc.py:73)."""
    graph, bidx, subset, adj = reddit
    B, n = bidx.numel(), subset.numel()
    assert B == 10_000 and torch.equal(subset[:B], bidx)
    assert n > 200_000 and adj.nnz() > 100_000_000
    rp, cl, vl = adj.csr()
    remap = torch.full((graph.N,), -1, dtype=torch.int64, device=DEV)
    remap[subset] = torch.arange(n, device=DEV)
    gen = torch.Generator().manual_seed(0)
    lens = (rp[1:] - rp[:-1]).long()
    rows = torch.cat([torch.randint(0, B, (24,), generator=gen),
                      torch.randint(B, n, (24,), generator=gen),
                      torch.topk(lens, 4).indices.cpu()])
    for r in rows.tolist():
        g = int(subset[r])
        gc = graph.col[graph.rowptr[g]:graph.rowptr[g + 1]].long()
        gv = graph.value[graph.rowptr[g]:graph.rowptr[g + 1]]
        loc = remap[gc]
        keep = loc >= 0
        order = torch.argsort(loc[keep])
        assert torch.equal(cl[rp[r]:rp[r + 1]].long(), loc[keep][order]), r
        assert torch.equal(vl[rp[r]:rp[r + 1]], gv[keep][order]), r


def _inputs(B, F, seed):
    gen = torch.Generator().manual_seed(seed)
    X = torch.randn(B, F, generator=gen)
    if F == 604:                       # the reddit feature padding (misc.py:212-216)
        X[:, 602:] = 0
    G = torch.randn(B, F, generator=gen) * 1e-3
    return X, G


@pytest.mark.parametrize("F", [604, 128])
def test_reddit_vq_update_vs_oracle(reddit, F):
    """update() for all nb branches on the full 10,000-row batch: indices and
    BatchNorm running stats bit-exact, EMA state within 1e-5 (scale-relative),
    for a spread of branches; codes scattered for every branch."""
    graph, bidx, subset, adj = reddit
    B, nb = bidx.numel(), F // D
    X, G = _inputs(B, F, seed=F)
    torch.manual_seed(1)
    bank = VQBank(nb, M, D, warm_up_flag=True)
    for b in range(nb):
        bank.init_branch(b)
    sample = sorted(set([0, 1, nb // 3, nb // 2, nb - 2, nb - 1]))
    states = []
    for b in sample:
        st = vq_ref.new_state(M, D, warm_up=True)
        for k, src in (("embedding", bank.emb), ("ema_w", bank.ema_w),
                       ("embedding_output", bank.emb_out), ("ema_cluster_size", bank.cs)):
            st[k] = src[b].clone()
        states.append(st)
    bank = bank.to(DEV)
    codes = torch.zeros(graph.N, nb, dtype=torch.int16, device=DEV)
    idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
    bank.update(X.to(DEV), G.to(DEV), 0, nb, True, idx_out=idx, codes=codes, batch_idx=bidx)
    torch.cuda.synchronize()
    idx_c = idx.cpu()
    assert torch.equal(codes[bidx].long().cpu(), idx_c.T)
    for st, b in zip(states, sample):
        ref, _, _ = vq_ref.update(st, X[:, b * D:(b + 1) * D], G[:, b * D:(b + 1) * D])
        assert torch.equal(idx_c[b], ref[:, 0]), f"F={F} branch {b}: index mismatch"
        for k, mine in (("rm_f", bank.rm_f), ("rv_f", bank.rv_f), ("rm_g", bank.rm_g),
                        ("rv_g", bank.rv_g)):
            assert torch.equal(mine[b].cpu(), st[k]), f"F={F} branch {b} {k}"
        for k, mine in (("embedding", bank.emb), ("embedding_output", bank.emb_out),
                        ("ema_cluster_size", bank.cs), ("ema_w", bank.ema_w)):
            a, r = mine[b].cpu(), st[k]
            scale = 1.0 + (r.abs().amax(dim=-1, keepdim=True) if r.dim() == 2 else r.abs())
            err = ((a - r).abs() / scale).max().item()
            assert err < 1e-5, f"F={F} branch {b} {k}: rel err {err:.2e}"


def test_reddit_ema_count_conservation(reddit):
    """The int64 EMA statistic of the F = 604 assign: per branch the counts
    sum to B and equal the bincount of the indices (exact)."""
    graph, bidx, subset, adj = reddit
    B, F = bidx.numel(), 604
    nb = F // D
    X, G = _inputs(B, F, seed=7)
    X, G = X.to(DEV), G.to(DEV)
    torch.manual_seed(2)
    emb = torch.randn(nb, M, 2 * D, device=DEV)
    rm = torch.zeros(nb, D, device=DEV)
    rv = torch.ones(nb, D, device=DEV)
    coef, _, _ = kernels.bn_stats_finalize(X, G, F, kernels.BN_TRAIN, 0.1, 1e-5, 0.1, 1e-24,
                                           1e-24, rm.view(-1), rv.view(-1), rm.clone().view(-1),
                                           rv.clone().view(-1))
    idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
    stats = kernels.vq_assign(X, G, coef, 1.0, emb, D, 2 * D, idx_out=idx, want_stats=True,
                              stat_count=B)
    stats = kernels.vq_ema_reduce(stats).view(nb, M, 2 * D + 1)
    counts = stats[:, :, 0].cpu()
    assert torch.equal(counts.sum(1), torch.full((nb,), B, dtype=torch.int64))
    for b in range(nb):
        assert torch.equal(counts[b], torch.bincount(idx[b].cpu(), minlength=M)), b


@pytest.mark.parametrize("F", [604, 128])
def test_reddit_gather_and_spmm(reddit, F):
    """x_first_order gather exact; the two-source SpMM over all ~115 M edges
    within 1e-5 (of the row's sum of |w x|) of an fp64 sum on 1,024 random
    rows plus the 16 longest, and bit-identical across two runs."""
    graph, bidx, subset, adj = reddit
    B, n, nb = bidx.numel(), subset.numel(), F // D
    X, _ = _inputs(B, F, seed=3 * F)
    X = X.to(DEV)
    torch.manual_seed(3)
    emb_out = torch.randn(nb, M, 2 * D, device=DEV)
    codes = torch.randint(0, M, (graph.N, nb), dtype=torch.int16, device=DEV)
    x_first, _ = kernels.gather_codewords(subset, B, codes, emb_out, D)
    c = codes[subset[B:]].long()                                   # [n - B, nb]
    ref_first = emb_out[torch.arange(nb, device=DEV)[None], c][:, :, :D].reshape(n - B, F)
    assert torch.equal(x_first, ref_first)
    rp, cl, vl = adj.rowptr, adj.col, adj.value          # the int32 device arrays
    plan = adj.plan(F, B=B)
    out = kernels.spmm(rp, cl, vl, n, adj.nnz(), X, F, X2=x_first, B=B, plan=plan)
    out2 = kernels.spmm(rp, cl, vl, n, adj.nnz(), X, F, X2=x_first, B=B, plan=plan)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    lens = (rp[1:] - rp[:-1]).long()
    gen = torch.Generator().manual_seed(F)
    rows = torch.cat([torch.randint(0, n, (1024,), generator=gen).to(DEV),
                      torch.topk(lens, 16).indices])
    xin = torch.cat([X, x_first])
    for r0 in range(0, rows.numel(), 64):
        rs = rows[r0:r0 + 64]
        starts, ln = rp[rs].long(), lens[rs]
        seg = torch.repeat_interleave(torch.arange(rs.numel(), device=DEV), ln)
        off = torch.arange(int(ln.sum()), device=DEV) - torch.repeat_interleave(
            torch.cumsum(ln, 0) - ln, ln)
        e = torch.repeat_interleave(starts, ln) + off
        contrib = vl[e].double()[:, None] * xin[cl[e].long()].double()
        ref = torch.zeros(rs.numel(), F, dtype=torch.float64, device=DEV).index_add_(0, seg, contrib)
        mag = torch.zeros_like(ref).index_add_(0, seg, contrib.abs())
        err = ((out[rs].double() - ref).abs() / (mag + 1e-30)).max().item()
        assert err < 1e-5, f"F={F}: rel err {err:.2e} in rows {rs[:4].tolist()}..."
