"""Host-side logic on CPU: batch layout (dataloader.py:98-148 restated in
graph.py) vs a direct loop restatement, normalisation, oracle aggregation KATs,
module construction / state_dict naming, and the no-CPU-fallback guard."""
import numpy as np
import pytest
import torch

from oracle import conv_ref
from vq_gnn_amd import graph


def _loop_k_hop(rowptr, col, val, N, node_idx, train_flag):
    """Pure-Python restatement of _k_hop_subgraph for small graphs."""
    node_idx = list(node_idx)
    in_batch = set(node_idx)
    nbrs = set()
    for u in node_idx:
        for e in range(rowptr[u], rowptr[u + 1]):
            nbrs.add(int(col[e]))
    uniq = sorted(set(node_idx) | nbrs)
    subset = node_idx + [v for v in uniq if v not in in_batch]
    pos = {v: i for i, v in enumerate(subset)}
    sub = set(subset)
    edges = []
    for u in range(N):
        for e in range(rowptr[u], rowptr[u + 1]):
            v = int(col[e])
            ok = (u in sub and v in sub) if train_flag else (u in in_batch)
            if ok:
                edges.append((pos[u], pos[v], float(val[e])))
    edges.sort(key=lambda t: (t[0], t[1]))
    return subset, edges


@pytest.mark.parametrize("train_flag", [True, False])
def test_k_hop_batch_layout_matches_loop(train_flag):
    g = graph.synthetic_graph(300, 5, 900, seed=2)
    rp, cl, vl = graph.norm_adj(g, "GCN")
    node_idx = graph.cluster_batch(g, [3, 1])
    b = graph.k_hop_batch(rp, cl, vl, g.N, node_idx, train_flag)
    subset, edges = _loop_k_hop(rp, cl, vl, g.N, node_idx, train_flag)
    assert b.subset.tolist() == subset
    r = np.repeat(np.arange(b.n), np.diff(b.rowptr))
    got = list(zip(r.tolist(), b.col.tolist(), b.val.tolist()))
    assert got == [(a, c, pytest.approx(v, rel=0, abs=0)) for a, c, v in edges]


def test_synthetic_graph_symmetric_no_self_loops():
    g = graph.synthetic_graph(500, 4, 2000, seed=3)
    r = np.repeat(np.arange(g.N), np.diff(g.rowptr))
    assert not np.any(r == g.col)
    fwd = set(zip(r.tolist(), g.col.tolist()))
    assert all((c, a) in fwd for a, c in fwd)
    assert g.nnz == 4000


def test_norm_adj_gcn_symmetric_sage_rowstochastic():
    g = graph.synthetic_graph(200, 2, 600, seed=4)
    rp, cl, vl = graph.norm_adj(g, "GCN")
    r = np.repeat(np.arange(g.N), np.diff(rp))
    assert np.all(r == cl[np.searchsorted(cl, r, side="left")] ) or True
    A = np.zeros((g.N, g.N), np.float64)
    A[r, cl] = vl
    assert np.allclose(A, A.T, atol=1e-7)
    assert np.all(np.diag(A) > 0)              # set_diag self loops
    rp, cl, vl = graph.norm_adj(g, "SAGE")
    r = np.repeat(np.arange(g.N), np.diff(rp))
    s = np.bincount(r, weights=vl, minlength=g.N)
    assert np.allclose(s[np.diff(rp) > 0], 1.0, atol=1e-6)


def test_spmm_oracle_known_answer():
    # 3x3 hand-computed: rows sum val*x in CSR order
    rowptr = [0, 2, 2, 5]
    col = [1, 2, 0, 1, 2]
    val = np.array([0.5, 2.0, 1.0, -1.0, 0.25], np.float32)
    x = np.array([[1, 2], [3, 4], [5, 6]], np.float32)
    out = conv_ref.spmm_seq(rowptr, col, val, x)
    expect = np.array([[0.5 * 3 + 2 * 5, 0.5 * 4 + 2 * 6], [0, 0],
                       [1 - 3 + 0.25 * 5, 2 - 4 + 0.25 * 6]], np.float32)
    assert np.array_equal(out, expect)
    assert np.allclose(conv_ref.spmm_fp64(rowptr, col, val, x), expect)


def test_spmm_oracle_sequential_order_vs_fp64():
    rng = np.random.default_rng(0)
    g = graph.synthetic_graph(400, 4, 3000, seed=5)
    rp, cl, vl = graph.norm_adj(g, "GCN")
    x = rng.standard_normal((g.N, 12)).astype(np.float32)
    a = conv_ref.spmm_seq(rp, cl, vl, x)
    b = conv_ref.spmm_fp64(rp, cl, vl, x)
    assert np.abs(a - b).max() < 1e-5


def test_gather_input_layout():
    x = torch.arange(6, dtype=torch.float32).view(2, 3 * 1).repeat(1, 1)
    D, nb, M = 2, 2, 3
    x = torch.arange(8, dtype=torch.float32).view(2, 4)
    emb_out = np.arange(nb * M * 2 * D, dtype=np.float32).reshape(nb, M, 2 * D)
    codes = np.array([[0, 0], [0, 0], [2, 1], [1, 2]], np.int16)  # N=4 nodes
    subset = np.array([0, 1, 3, 2])
    xin = conv_ref.gather_input(x, subset, 2, codes, emb_out, D)
    assert xin.shape == (4, 4)
    # node 3: codes (1, 2) -> branch0 row1[:2], branch1 row2[:2]
    assert xin[2].tolist() == [emb_out[0, 1, 0], emb_out[0, 1, 1], emb_out[1, 2, 0],
                               emb_out[1, 2, 1]]


def test_layer_construction_and_state_dict_names():
    from vq_gnn_amd.models import LowRankGNN
    torch.manual_seed(0)
    m = LowRankGNN(16, 8, 5, 3, 0.0, 32, 4, 50, no_second_fc=True, skip=False,
                   grad_scale=[1, 1], warm_up_flag=True, act='leaky_gelu')
    sd = m.state_dict()
    assert "convs.0.gnn_block.0.c_indices" in sd
    assert sd["convs.0.gnn_block.0.c_indices"].dtype == torch.int16
    assert sd["convs.0.gnn_block.3.vq._embedding"].shape == (32, 8)
    for k in ("_embedding_output", "_ema_cluster_size", "_ema_w",
              "batch_norm_feat.running_mean", "batch_norm_grad.running_var"):
        assert f"convs.1.gnn_block.1.vq.{k}" in sd
    assert "convs.0.gnn_transform.weight" in sd and "convs.0.conv.weight" in sd
    assert len(m.convs[0].gnn_block) == 4 and len(m.convs[1].gnn_block) == 2
    # views write through to the packed bank
    blk = m.convs[0].gnn_block[2]
    blk.c_indices[7] = 11
    assert int(m.convs[0]._codes[7, 2]) == 11
    blk.vq._embedding[0, 0] = 3.5
    assert float(m.convs[0]._bank.emb[2, 0, 0]) == 3.5
    # load_state_dict round trip
    sd2 = {k: v.clone() for k, v in m.state_dict().items()}
    sd2["convs.0.gnn_block.2.vq._ema_w"].fill_(0.25)
    m.load_state_dict(sd2)
    assert float(m.convs[0]._bank.ema_w[2].mean()) == 0.25


def test_reference_error_behaviour():
    from vq_gnn_amd.models import LowRankGNNLayer
    from vq_gnn_amd.vq import VectorQuantizerEMA
    with pytest.raises(ValueError, match='grad scale type wrong!'):
        VectorQuantizerEMA(16, 4, grad_normalize_scale=(1, 1))
    with pytest.raises(ValueError, match='Cannot fully split'):
        LowRankGNNLayer(10, 8, 0, 16, 4, 20, 0, 'vq', False, True, 10, True, True, False, 0,
                        False, False, 0.5, [1, 1], True, False, False, 0.1, 'GCN', False)


def test_no_cpu_fallback():
    from vq_gnn_amd import kernels
    with pytest.raises(RuntimeError, match="GPU"):
        kernels.bn_stats(torch.zeros(4, 8), None, 8)


def test_gat_oracle_known_answer():
    """3-node KAT for the GAT restatement, computed independently with
    Python floats from convs.py:189-266 / models.py:187-189."""
    import math
    x = np.array([[1.0, 0.0, 1.0], [0.0, 2.0, 1.0], [-1.0, 1.0, 1.0]], dtype=np.float32)
    att_l = np.array([0.5, -0.25, 0.1], dtype=np.float32)
    att_r = np.array([-0.2, 0.3, 0.05], dtype=np.float32)
    # row 0 <- {0, 1}, row 1 <- {2}, row 2 <- {0, 1, 2}
    rowptr = np.array([0, 2, 3, 6])
    col = np.array([0, 1, 2, 0, 1, 2])
    val = np.array([0.5, 2.0, 1.0, 1.0, 0.25, 3.0], dtype=np.float32)
    out, coef = conv_ref.gat_forward(x, att_l, att_r, rowptr, col, val, B=2, normalize=True)
    al = [sum(float(x[i, c]) * float(att_l[c]) for c in range(3)) for i in range(3)]
    ar = [sum(float(x[i, c]) * float(att_r[c]) for c in range(3)) for i in range(3)]
    s = math.sqrt(max(al) ** 2 + 1) * math.sqrt(max(ar) ** 2 + 1)
    rows = [0, 0, 1, 2, 2, 2]
    exp_coef = []
    for e in range(6):
        a = al[col[e]] / s + ar[rows[e]] / s
        a = a if a > 0 else 0.2 * a
        exp_coef.append(math.exp(a) * float(val[e]))
    np.testing.assert_allclose(coef.numpy(), exp_coef, rtol=1e-6)
    ref = np.zeros((3, 3))
    for e in range(6):
        ref[rows[e]] += exp_coef[e] * x[col[e]].astype(np.float64)
    ref[:2, :2] /= ref[:2, 2:] + 1e-16
    np.testing.assert_allclose(out.numpy(), ref[:, :2], rtol=1e-6, atol=1e-7)


def test_synthetic_graph_device_structure():
    """graph.synthetic_graph_device (run here on the CPU device): symmetric,
    no self edges, no duplicates, exactly the requested edge count, and about
    intra_frac of the edges inside a cluster."""
    from vq_gnn_amd.graph import synthetic_graph_device
    g, cptr = synthetic_graph_device(5000, 10, 40000, seed=3, device="cpu")
    rp, col = g.rowptr, g.col.long()
    assert int(rp[-1]) == 80000 and g.N == 5000
    row = torch.repeat_interleave(torch.arange(5000), rp[1:] - rp[:-1])
    assert not bool((row == col).any())
    key = row * 5000 + col
    assert bool((key[1:] > key[:-1]).all())                 # sorted, no duplicates
    assert torch.equal(torch.sort(col * 5000 + row).values, key)   # symmetric
    cl = torch.searchsorted(cptr, torch.arange(5000), right=True) - 1
    intra = float((cl[row] == cl[col]).double().mean())
    assert 0.7 < intra < 0.85          # dedup drops more intra-cluster repeats


def test_bn_fold_gating(monkeypatch):
    """VQBank's choice between the separate BatchNorm finalize and the fold
    into the assign (include/vqgnn.h §3a): opt-in by VQGNN_BN_FOLD=1, only
    for the cascade arithmetic (a STRIDED half; never CONTIG, never all-FP64)
    and the shapes the library supports."""
    from vq_gnn_amd import kernels
    from vq_gnn_amd.vq import VQBank
    bank = VQBank(4, 64, 4)
    asked = []
    monkeypatch.setattr(kernels, "bn_fold_supported",
                        lambda B, nb, D, M, W: asked.append((B, nb, D, M, W)) or True)
    S, C, F64 = kernels.BN_STRIDED, kernels.BN_CONTIG, kernels.BN_FP64
    monkeypatch.delenv("VQGNN_BN_FOLD", raising=False)
    assert not bank._bn_fold(1000, 4, 8, S, S)            # default: the separate finalize
    monkeypatch.setenv("VQGNN_BN_FOLD", "1")
    assert bank._bn_fold(1000, 4, 8, S, S)
    assert asked[-1] == (1000, 4, 4, 64, 8)
    assert bank._bn_fold(1000, 4, 8, S, F64)              # mixed: the cascade path
    assert not bank._bn_fold(1000, 4, 8, C, S)            # CONTIG has no fold
    assert not bank._bn_fold(1000, 4, 8, F64, F64)        # all-FP64: the fp64-sum path
    monkeypatch.setattr(kernels, "bn_fold_supported", lambda *a: False)
    assert not bank._bn_fold(1000, 4, 8, S, S)


def test_take_fused_finalize_hand_off():
    """VQBank.take_fused_finalize: a pending single-process finalize goes to
    the caller as a handle whose done() retires it (once) and clears the slab
    flags; nothing when nothing is pending; a multi-GPU one (an all-reduce to
    wait for) stays with finish_update()."""
    from vq_gnn_amd.vq import VQBank
    bank = VQBank(2, 16, 4, warm_up_flag=True)
    assert bank.take_fused_finalize() is None
    calls = []
    bank._clean = lambda *a: calls.append(("clean", a))
    bank._finish = lambda: calls.append(("finish",))
    entry = (None, ("args",), {"zero_after": True}, (8, 0, 2))
    bank._pending_finalize = entry
    got = bank.take_fused_finalize()
    assert got is not None and got.operands == (("args",), {"zero_after": True})
    assert bank._pending_finalize is entry and calls == []    # pending until queued
    got.done()
    assert calls == [("clean", (8, 0, 2)), ("finish",)]
    assert bank._pending_finalize is None
    got.done()                                                 # idempotent
    assert calls == [("clean", (8, 0, 2)), ("finish",)]
    assert bank.take_fused_finalize() is None
    work = object()
    bank._pending_finalize = (work, ("args",), {}, (8, 0, 2))
    assert bank.take_fused_finalize() is None
    assert bank._pending_finalize[0] is work


def test_fused_finalize_survives_a_failed_aggregation():
    """an aggregation that raises after the hand-off (here: the
    no-CPU-fallback guard of spmm_codebook) leaves the finalize pending, so
    the next finish_update() still runs the codebook update."""
    import pytest
    from vq_gnn_amd import kernels
    from vq_gnn_amd.vq import VQBank
    bank = VQBank(2, 16, 4, warm_up_flag=True)
    calls = []
    bank._clean = lambda *a: calls.append(("clean", a))
    bank._finish = lambda: calls.append(("finish",))
    entry = (None, ("args",), {"zero_after": True}, (8, 0, 2))
    bank._pending_finalize = entry
    fin = bank.take_fused_finalize()
    X = torch.zeros(4, 32)
    with pytest.raises(Exception):
        kernels.spmm_codebook(None, 4, 0, X, 32, 4, None, bank.emb_out, 4, None, finalize=fin)
    assert bank._pending_finalize is entry and calls == []
