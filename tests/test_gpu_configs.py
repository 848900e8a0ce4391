"""Full-size GPU parity at the two BASELINE configs no other test runs at their
workload shape:

- ppi SAGE-Mean (BASELINE configs[2], README.md:45): node-sampled batch of
  B = 30,000 from the 44,906-node synthetic ppi graph, M = 4,096 codewords,
  layer 1 at F = 52 (50 features zero-padded, nb = 13; utils/misc.py:212-222)
  and layer 2 at F = 256 (nb = 64), D^-1 A weights (utils/misc.py:21-25) and
  the host fc_sage (models.py:203-204);
- arxiv GAT (configs[4], convs.py:165-266, models.py:176-189): the full
  84,670-row arxiv batch, M = 1,024, C = F + 1 = 129;
- arxiv GCN, the headline (configs[1]): M = 256, the full batch, through
  bench.py's own update sequence (feature_update warm-up, update(defer=True)
  + finish_update(), feature_update, and dead codewords).

Bounds: codeword indices and BatchNorm state bit-exact against the oracle
(vq_ref, pinned to the reference's vq.py by the golden fixtures) on a spread
of branches; EMA state within 1e-5 (scale-relative); aggregation outputs
within 1e-5 of the sum of |terms| of an fp64 restatement on 1,024 sampled
rows plus the longest ones (north_star: fp32 messages within 1e-5 relative);
GAT coefficients within 2e-6 of the oracle's reference-order fp32 chain."""
import numpy as np
import pytest
import torch

from helpers import sequential_argmin, tie_aware_mismatch
from oracle import conv_ref, vq_ref
from vq_gnn_amd import graph, kernels
from vq_gnn_amd.convs_gat import OurGATConv
from vq_gnn_amd.models import LowRankGNNLayer
from vq_gnn_amd.vq import VQBank

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
D = 4


@pytest.fixture(scope="module")
def ppi():
    g, _, b = graph.make_batch(graph.CONFIGS["ppi_sage"])
    return g, b


@pytest.fixture(scope="module")
def arxiv_gat():
    g, _, b = graph.make_batch(graph.CONFIGS["arxiv_gat"])
    return g, b


def _features(B, F, seed):
    gen = torch.Generator().manual_seed(seed)
    X = torch.randn(B, F, generator=gen)
    if F == 52:                        # ppi's 50 features zero-padded (misc.py:212-222)
        X[:, 50:] = 0
    G = torch.randn(B, F, generator=gen) * 1e-3
    return X, G


def _bank_and_states(nb, M, sample, seed):
    torch.manual_seed(seed)
    bank = VQBank(nb, M, D, warm_up_flag=True)
    for b in range(nb):
        bank.init_branch(b)
    states = []
    for b in sample:
        st = vq_ref.new_state(M, D, warm_up=True)
        for k, src in (("embedding", bank.emb), ("ema_w", bank.ema_w),
                       ("embedding_output", bank.emb_out), ("ema_cluster_size", bank.cs)):
            st[k] = src[b].clone()
        states.append(st)
    return bank.to(DEV), states


def _check_state(bank, st, b, tag, skip=None):
    """BatchNorm state bit-identical, EMA state within 1e-5; ``skip``: codewords
    left out of the EMA check (those of adjudicated near-tie rows)."""
    for k, mine in (("rm_f", bank.rm_f), ("rv_f", bank.rv_f), ("rm_g", bank.rm_g),
                    ("rv_g", bank.rv_g)):
        assert torch.equal(mine[b].cpu(), st[k]), f"{tag} branch {b} {k}"
    keep = None
    if skip is not None and len(skip):
        keep = torch.ones(st["embedding"].shape[0], dtype=torch.bool)
        keep[torch.as_tensor(sorted(skip))] = False
    for k, mine in (("embedding", bank.emb), ("embedding_output", bank.emb_out),
                    ("ema_cluster_size", bank.cs), ("ema_w", bank.ema_w)):
        a, r = mine[b].cpu(), st[k]
        if keep is not None:
            a, r = a[keep], r[keep]
        scale = 1.0 + (r.abs().amax(dim=-1, keepdim=True) if r.dim() == 2 else r.abs())
        err = ((a - r).abs() / scale).max().item()
        assert err < 1e-5, f"{tag} branch {b} {k}: rel err {err:.2e}"


def _vq_update_vs_oracle(g, b, F, M, seed):
    B, nb = b.B, F // D
    X, G = _features(B, F, seed)
    sample = sorted(set([0, 1, nb // 2, nb - 1]))
    bank, states = _bank_and_states(nb, M, sample, seed)
    bidx = torch.from_numpy(b.batch_idx).to(DEV)
    codes = torch.zeros(g.N, nb, dtype=torch.int16, device=DEV)
    idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
    bank.update(X.to(DEV), G.to(DEV), 0, nb, True, idx_out=idx, codes=codes, batch_idx=bidx)
    torch.cuda.synchronize()
    idx_c = idx.cpu()
    assert torch.equal(codes[bidx].long().cpu(), idx_c.T)
    for st, br in zip(states, sample):
        ref, _, _ = vq_ref.update(st, X[:, br * D:(br + 1) * D], G[:, br * D:(br + 1) * D])
        n_mis = int((idx_c[br] != ref[:, 0]).sum())
        assert n_mis == 0, f"F={F} M={M} branch {br}: {n_mis} index mismatches"
        _check_state(bank, st, br, f"F={F} M={M}")


@pytest.mark.parametrize("F", [52, 256])
def test_ppi_vq_update_vs_oracle(ppi, F):
    """update() for all nb branches of a ppi layer on the full 30,000-row
    batch at M = 4,096 (codebook staged in LDS chunks, EMA statistics in the
    split kernel)."""
    g, b = ppi
    assert b.B == 30_000
    _vq_update_vs_oracle(g, b, F, 4096, seed=F)


def test_arxiv_gat_vq_update_vs_oracle(arxiv_gat):
    """update() for the 32 branches of the arxiv GAT layer (M = 1,024) on the
    full 84,670-row batch."""
    g, b = arxiv_gat
    _vq_update_vs_oracle(g, b, 128, 1024, seed=5)


@pytest.fixture(scope="module")
def arxiv_gcn():
    g, _, b = graph.make_batch(graph.CONFIGS["arxiv_gcn"])
    return g, b


def _normalised(st, xb, gb=None):
    """The oracle's normalised rows of one call (training: batch statistics,
    so the running-stat clones are left untouched) and the codebook its
    argmin reads -- taken before the call mutates the state."""
    bn = torch.nn.functional.batch_norm
    xn = bn(xb, st["rm_f"].clone(), st["rv_f"].clone(), None, None, True, 0.1, 1e-5)
    if gb is None:
        return xn, st["embedding"][:, :D].clone()
    gn = bn(gb, st["rm_g"].clone(), st["rv_g"].clone(), None, None, True, st["momentum"],
            st["epsilon"]) * st["grad_scale"][0]
    return torch.cat([xn, gn], 1), st["embedding"].clone()


def _compare_branches(idx, codes, bidx, states, sample, ref_call, bank, tag, inputs, emb_pre):
    """Indices against vq_ref on the sampled branches.  The first call sees
    identical codebooks and must match bit for bit.  After an EMA update the
    codebooks agree to 1e-5, not bitwise (the device sums the statistics
    exactly in int64, the reference in fp32 matmuls), so a
    row whose two best codewords are closer than that rounding may pick
    either: such a row must equal the pinned sequential fp32 arithmetic
    (helpers.sequential_argmin, vq.py:166-171) on the device's own codebook
    and be a tie within 1e-5 under the oracle's distances
    (helpers.tie_aware_mismatch); at most 4 per branch.  Their two codewords
    leave the EMA comparison of this call, and every oracle state is then
    re-based on the device's EMA state, so each call starts from identical
    codebooks."""
    torch.cuda.synchronize()
    idx_c = idx.cpu()
    assert torch.equal(codes[bidx].long().cpu(), idx_c.T), f"{tag}: codes != indices"
    for st, br in zip(states, sample):
        xn, emb_ref = _normalised(st, *inputs(br))
        ref = ref_call(st, br)
        bad = torch.nonzero(idx_c[br] != ref[:, 0]).view(-1)
        if bad.numel():
            assert emb_pre is not None, f"{tag} branch {br}: {bad.numel()} index mismatches"
            assert bad.numel() <= 4, f"{tag} branch {br}: {bad.numel()} index mismatches"
            W = xn.shape[1]
            pinned = torch.from_numpy(sequential_argmin(xn[bad].numpy(),
                                                        emb_pre[br][:, :W].numpy()))
            assert torch.equal(idx_c[br][bad], pinned), \
                f"{tag} branch {br}: rows {bad.tolist()} differ from the pinned arithmetic"
            dist = vq_ref.distances(xn[bad], emb_ref)
            n_mis, n_bad = tie_aware_mismatch(idx_c[br][bad], ref[bad, 0], dist)
            assert n_bad == 0, f"{tag} branch {br}: rows {bad.tolist()} are not near-ties"
        skip = set(idx_c[br][bad].tolist()) | set(ref[bad, 0].tolist())
        _check_state(bank, st, br, tag, skip)
        for k, mine in (("embedding", bank.emb), ("embedding_output", bank.emb_out),
                        ("ema_cluster_size", bank.cs), ("ema_w", bank.ema_w)):
            st[k] = mine[br].cpu().clone()


def test_arxiv_gcn_headline_vq_vs_oracle(arxiv_gcn):
    """The headline config (BASELINE configs[1]: arxiv GCN, M = 256, D = 4, the
    full 84,670-row cluster batch, nb = 32) through bench.py's exact sequence:
    the warm-up feature_update (W = 4) on the fresh codebook, then the timed
    step's update(defer=True) (W = 8) with the codeword gather queued before
    finish_update(), then feature_update (W = 4) on the warm codebook.  At
    M <= 512 the filter stages an f32 candidate copy in LDS and packs 3-bit
    pair indices (a path no other full-size test takes).  Indices of 6 spread
    branches bit-exact against vq_ref (vq.py:160-279), BatchNorm state
    bit-identical, EMA state within 1e-5."""
    g, b = arxiv_gcn
    F, M = 128, 256
    nb, B = F // D, b.B
    assert B == 84_670
    X = torch.randn(B, F, generator=torch.Generator().manual_seed(1))        # bench.py inputs
    G = torch.randn(B, F, generator=torch.Generator().manual_seed(2)) * 1e-3
    sample = [0, 5, 11, 17, 23, 31]
    bank, states = _bank_and_states(nb, M, sample, seed=0)
    bidx = torch.from_numpy(b.batch_idx).to(DEV)
    _, subset, _ = graph.batch_to_device(b, DEV)
    codes = torch.randint(0, M, (g.N, nb), dtype=torch.int16,
                          generator=torch.Generator().manual_seed(5)).to(DEV)
    Xd, Gd = X.to(DEV), G.to(DEV)
    idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
    cols = lambda t, br: t[:, br * D:(br + 1) * D]      # noqa: E731 (strided slices, models.py:162)

    bank.feature_update(Xd, 0, nb, True, idx_out=idx, codes=codes, batch_idx=bidx)
    fu_in = lambda br: (cols(X, br),)                    # noqa: E731
    up_in = lambda br: (cols(X, br), cols(G, br))        # noqa: E731
    _compare_branches(idx, codes, bidx, states, sample,
                      lambda st, br: vq_ref.feature_update(st, cols(X, br)), bank, "warm-up W=4",
                      fu_in, None)                      # identical codebooks: bit-exact
    emb_pre = bank.emb.cpu()
    bank.update(Xd, Gd, 0, nb, True, idx_out=idx, codes=codes, batch_idx=bidx, defer=True)
    kernels.gather_codewords(subset, B, codes, bank.emb_out, D)   # queued as in the bench step
    bank.finish_update()
    _compare_branches(idx, codes, bidx, states, sample,
                      lambda st, br: vq_ref.update(st, cols(X, br), cols(G, br))[0], bank,
                      "update W=8", up_in, emb_pre)
    emb_pre = bank.emb.cpu()

    bank.feature_update(Xd, 0, nb, True, idx_out=idx, codes=codes, batch_idx=bidx)
    _compare_branches(idx, codes, bidx, states, sample,
                      lambda st, br: vq_ref.feature_update(st, cols(X, br)), bank,
                      "warm feature_update W=4", fu_in, emb_pre)

    # dead codewords (a trained codebook's unused ones reach |e|^2 ~ 1e10:
    # scored +inf by the filter, the range path of DESIGN.md §4.1), injected
    # alike into the bank and the oracle states, then the bench step again
    dead = torch.arange(3, M, 17)
    for st, br in zip(states, sample):
        st["embedding"][dead] *= 1e5
    bank.emb[:, dead] *= 1e5
    assert int((bank.emb[:, :, :D].pow(2).sum(-1) >= 2 ** 15).sum()) >= nb * dead.numel()
    emb_pre = bank.emb.cpu()
    bank.update(Xd, Gd, 0, nb, True, idx_out=idx, codes=codes, batch_idx=bidx, defer=True)
    kernels.gather_codewords(subset, B, codes, bank.emb_out, D)
    bank.finish_update()
    _compare_branches(idx, codes, bidx, states, sample,
                      lambda st, br: vq_ref.update(st, cols(X, br), cols(G, br))[0], bank,
                      "update W=8, dead codewords", up_in, emb_pre)


def _sampled_rows(rowptr, n_rows, k, seed, longest=16):
    lens = np.diff(rowptr[:n_rows + 1])
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([rng.integers(0, n_rows, k),
                                     np.argsort(lens)[-longest:]]))


def _edges_of(rowptr, col, val, rows):
    seg = np.repeat(np.arange(rows.size), np.diff(rowptr)[rows])
    e = np.concatenate([np.arange(rowptr[r], rowptr[r + 1]) for r in rows])
    return seg, col[e].astype(np.int64), val[e].astype(np.float64), e


@pytest.mark.parametrize("F_in", [52, 256])
def test_ppi_sage_layer_vs_fp64(ppi, F_in):
    """The SAGE layer (models.py:144-231) at the ppi shape: init (feature_update
    of all branches) + codeword gather + the D^-1 A aggregation + gnn_transform
    + fc_sage.  Sampled branches' codes equal the oracle's; the layer output
    on sampled batch rows (and the hub rows) is within 1e-5 of the fp64
    restatement's sum of |terms|."""
    g, b = ppi
    M, F_out = 4096, 256
    nb = F_in // D
    torch.manual_seed(11)
    layer = LowRankGNNLayer(F_in, F_out, 0.0, M, D, g.N, 0, 'vq', False, True, 10, True, True,
                            False, 0, False, False, 0.5, [1, 1], True, False, True, 0.1,
                            "SAGE", False)
    sample = sorted(set([0, nb // 2, nb - 1]))
    states = []
    for br in sample:
        st = vq_ref.new_state(M, D, warm_up=True)
        for k, src in (("embedding", layer._bank.emb), ("ema_w", layer._bank.ema_w),
                       ("embedding_output", layer._bank.emb_out),
                       ("ema_cluster_size", layer._bank.cs)):
            st[k] = src[br].clone()
        states.append(st)
    layer = layer.to(DEV).train()
    X, _ = _features(b.B, F_in, seed=F_in + 1)
    batch_A = graph.batch_to_device(b, DEV)
    with torch.no_grad():
        out, *_ = layer(X.to(DEV), batch_A, 1.0, False)
    torch.cuda.synchronize()
    codes = layer._codes.cpu()
    for st, br in zip(states, sample):
        ref = vq_ref.feature_update(st, X[:, br * D:(br + 1) * D])
        got = codes[torch.from_numpy(b.batch_idx), br].long()
        assert int((got != ref[:, 0]).sum()) == 0, f"F={F_in} branch {br}: index mismatch"
    # fp64 restatement on sampled batch rows, from the GPU's own codes/codebook
    emb_out = layer._bank.emb_out.cpu().numpy()
    rows = _sampled_rows(b.rowptr, b.B, 1024, F_in)
    seg, cols, w, _ = _edges_of(b.rowptr, b.col, b.val, rows)
    xin = conv_ref.gather_input(X, b.subset, b.B, codes.numpy(), emb_out, D).numpy().astype(
        np.float64)
    agg = np.zeros((rows.size, F_in))
    aabs = np.zeros((rows.size, F_in))
    np.add.at(agg, seg, w[:, None] * xin[cols])
    np.add.at(aabs, seg, np.abs(w[:, None] * xin[cols]))
    Wt = layer.gnn_transform.weight.detach().double().cpu().numpy()
    bt = layer.gnn_transform.bias.detach().double().cpu().numpy()
    Ws = layer.fc_sage.weight.detach().double().cpu().numpy()
    bs = layer.fc_sage.bias.detach().double().cpu().numpy()
    x64 = X.double().numpy()[rows]
    ref = agg @ Wt.T + bt + x64 @ Ws.T + bs
    scale = aabs @ np.abs(Wt).T + np.abs(bt) + np.abs(x64) @ np.abs(Ws).T + np.abs(bs)
    err = np.abs(out.cpu().double().numpy()[rows] - ref)
    assert (err <= 1e-5 * scale + 1e-30).all(), \
        f"F={F_in}: max error / magnitude {(err / (scale + 1e-30)).max():.2e}"


def test_arxiv_gat_full_batch_vs_oracle(arxiv_gat):
    """OurGATConv's fused path on the full arxiv batch (C = 129, x_first
    gathered from an M = 1,024 codebook): per-edge coefficients of sampled
    rows against the oracle's reference-order fp32 chain (2e-6), and the
    normalised outputs of sampled batch rows and of sampled out-of-batch rows
    within 1e-5 of the fp64 chain's sum of |terms|."""
    g, b = arxiv_gat
    F, M = 128, 1024
    nb = F // D
    rng = np.random.default_rng(4)
    X = rng.standard_normal((b.B, F)).astype(np.float32)
    emb_out = rng.standard_normal((nb, M, 2 * D)).astype(np.float32)
    codes = rng.integers(0, M, size=(g.N, nb)).astype(np.int16)
    bidx, subset, adj = graph.batch_to_device(b, DEV)
    xf_d, _ = kernels.gather_codewords(subset, b.B, torch.from_numpy(codes).to(DEV),
                                       torch.from_numpy(emb_out).to(DEV), D)
    torch.manual_seed(4)
    conv = OurGATConv(F + 1, F + 1, bias=False, add_self_loops=False).to(DEV)
    x_d = torch.from_numpy(X).to(DEV)
    _, _, _, als, ars = kernels.gat_alpha(x_d, conv.att_l.view(-1), conv.att_r.view(-1), F,
                                          X2=xf_d, B=b.B, ones=True)
    plan = adj.plan(F)
    out, den, coef = kernels.gat_spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, x_d, F, als,
                                      ars, plan, adj.rows(), X2=xf_d, B=b.B, norm_B=b.B,
                                      want_den=True, want_coef=True)
    layer_out = conv.fused_forward(x_d, adj, xf_d, b.B)
    torch.cuda.synchronize()
    assert torch.equal(layer_out, out)
    xin = np.concatenate([np.concatenate([X, xf_d.cpu().numpy()]),
                          np.ones((b.n, 1), np.float32)], 1)
    att_l = conv.att_l.detach().cpu().numpy()
    att_r = conv.att_r.detach().cpu().numpy()
    # coefficients: the reference's fp32 op order (PyG message + vq_softmax)
    _, coef_ref = conv_ref.gat_forward(xin, att_l, att_r, b.rowptr, b.col, b.val)
    rows = np.concatenate([_sampled_rows(b.rowptr, b.B, 768, 1),
                           b.B + _sampled_rows(b.rowptr[b.B:] - b.rowptr[b.B], b.n - b.B,
                                               256, 2, longest=4)])
    seg, cols, w, e = _edges_of(b.rowptr, b.col, b.val, rows)
    c_got = coef.cpu().numpy()[e]
    c_ref = coef_ref.numpy()[e]
    np.testing.assert_allclose(c_got, c_ref, rtol=2e-6, atol=1e-7)
    # outputs against the fp64 chain
    x64 = xin.astype(np.float64)
    al64 = x64 @ att_l.reshape(-1).astype(np.float64)
    ar64 = x64 @ att_r.reshape(-1).astype(np.float64)
    s64 = np.sqrt(al64.max() ** 2 + 1) * np.sqrt(ar64.max() ** 2 + 1)
    row_of = rows[seg]
    a = al64[cols] / s64 + ar64[row_of] / s64
    c64 = np.exp(np.where(a > 0, a, 0.2 * a)) * w
    num = np.zeros((rows.size, F))
    mag = np.zeros((rows.size, F))
    den64 = np.zeros(rows.size)
    np.add.at(num, seg, c64[:, None] * x64[cols, :F])
    np.add.at(mag, seg, np.abs(c64[:, None] * x64[cols, :F]))
    np.add.at(den64, seg, c64)
    inb = rows < b.B
    num[inb] /= den64[inb, None] + 1e-16
    mag[inb] /= den64[inb, None] + 1e-16
    err = np.abs(out.cpu().double().numpy()[rows] - num)
    assert (err <= 1e-5 * mag + 1e-30).all(), \
        f"max error / magnitude {(err / (mag + 1e-30)).max():.2e}"
