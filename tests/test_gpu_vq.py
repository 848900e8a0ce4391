"""GPU parity of the VQ kernels (HIP, via the C-ABI) against the oracle and the
reference's golden vectors."""
import pytest
import torch

import numpy as np

from helpers import (STATE_KEYS, as_layout, golden_cases, load_case, oracle_state_from,
                     sequential_argmin, tie_aware_mismatch, torch_threads)
from oracle import vq_ref
from vq_gnn_amd import kernels
from vq_gnn_amd.vq import VQBank, VectorQuantizerEMA

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _coef_tensor(alpha_f, beta_f, alpha_g=None, beta_g=None):
    F = alpha_f.numel()
    c = torch.zeros(6, F)
    c[0], c[1] = alpha_f, beta_f
    if alpha_g is not None:
        c[2], c[3] = alpha_g, beta_g
    return c.to(DEV)


@pytest.mark.parametrize("M,D,W,B,tie", [
    (256, 4, 8, 3000, False), (256, 4, 4, 3000, False), (37, 4, 8, 1000, False),
    (1030, 4, 8, 2100, False), (4096, 4, 8, 1500, False), (64, 4, 8, 999, True),
    (128, 2, 4, 777, False), (64, 2, 2, 513, False), (16, 8, 16, 300, False),
    (5000, 4, 4, 700, False)])
def test_assign_bit_exact_given_coefficients(M, D, W, B, tie):
    """Same normalisation coefficients -> the codeword index is bit-exact
    (ATen fma BN, sequential |x|^2, MKL K<=8 sgemm == MFMA fma chain)."""
    g = torch.Generator().manual_seed(M * 7 + B)
    X = torch.randn(B, D, generator=g) * 2 + 0.5
    G = torch.randn(B, D, generator=g) * 1e-3
    emb = torch.randn(M, 2 * D, generator=g)
    if tie:
        emb[M // 2:] = emb[: M - M // 2]
    rmf, rvf = torch.zeros(D), torch.ones(D)
    af, bf = vq_ref.bn_coefficients(X, True, rmf, rvf, 1e-5)
    ag, bg = vq_ref.bn_coefficients(G, True, torch.zeros(D), torch.ones(D), 1e-24)
    scale = 0.75
    idx_ref, _ = vq_ref.assign_with_coef(X, G if W == 2 * D else None, af, bf, ag, bg, scale, emb)
    coef = _coef_tensor(af, bf, ag, bg)
    idx = torch.empty(1, B, dtype=torch.long, device=DEV)
    stats = kernels.vq_assign(X.to(DEV), G.to(DEV) if W == 2 * D else None, coef, scale,
                              emb.view(1, M, 2 * D).to(DEV), D, W, idx_out=idx, want_stats=True)
    assert torch.equal(idx.cpu()[0], idx_ref)
    # EMA statistics: int64 fixed point -> exact counts; sums within the
    # quantisation (half a unit of 2^-shift per row) of the fp64 sums
    assert stats.dtype == torch.int64
    xn = torch.cat([X * af + bf, ((G * ag + bg) * scale)], 1)[:, :W]
    cnt = torch.bincount(idx_ref, minlength=M).double()
    dw = torch.zeros(M, W, dtype=torch.float64).index_add_(0, idx_ref, xn.double())
    st = kernels.decode_stats(stats.sum(0), D, B, scale).cpu()[0]
    assert torch.equal(st[:, 0], cnt)
    sf, sg = kernels.stat_shifts(B, scale)
    unit = torch.tensor([2.0 ** -sf] * D + [2.0 ** -sg] * (W - D), dtype=torch.float64)
    absw = torch.zeros(M, W, dtype=torch.float64).index_add_(0, idx_ref, xn.double().abs())
    tol = cnt[:, None] * unit * 0.5 + 1e-6 * absw   # + fp32 rounding of xn itself
    assert ((st[:, 1:] - dw).abs() <= tol + 1e-7).all()


@pytest.mark.parametrize("M,B", [(1024, 2100), (1030, 2100), (4096, 1500)])
def test_assign_repeat_launches_identical(M, B):
    """The same assign launched 12 times gives the oracle's indices every
    time.  Guards the sweep's MFMA/VALU schedule: a software-pipelined sweep
    (round 5, removed) picked a near-best codeword for a few rows of some
    launches and not others ("Pipelined sweep")."""
    D, W = 4, 8
    g = torch.Generator().manual_seed(M * 7 + B)
    X = torch.randn(B, D, generator=g) * 2 + 0.5
    G = torch.randn(B, D, generator=g) * 1e-3
    emb = torch.randn(M, 2 * D, generator=g)
    af, bf = vq_ref.bn_coefficients(X, True, torch.zeros(D), torch.ones(D), 1e-5)
    ag, bg = vq_ref.bn_coefficients(G, True, torch.zeros(D), torch.ones(D), 1e-24)
    idx_ref, _ = vq_ref.assign_with_coef(X, G, af, bf, ag, bg, 0.75, emb)
    coef = _coef_tensor(af, bf, ag, bg)
    Xd, Gd, Ed = X.to(DEV), G.to(DEV), emb.view(1, M, 2 * D).to(DEV)
    bad = []
    for rep in range(12):
        idx = torch.empty(1, B, dtype=torch.long, device=DEV)
        kernels.vq_assign(Xd, Gd, coef, 0.75, Ed, D, W, idx_out=idx)
        n = int((idx.cpu()[0] != idx_ref).sum())
        if n:
            bad.append((rep, n))
    assert not bad, f"(launch, mismatching rows): {bad}"


@pytest.mark.parametrize("M,nb,D", [(256, 32, 4), (1024, 32, 4), (4096, 13, 4), (1024, 32, 2),
                                    (256, 32, 2)])
def test_assign_repeat_launches_many_branches(M, nb, D):
    """The shapes where round 5's packed-f32 resolve variant returned different
    indices on repeated launches (13-32 branches x 30,000 rows, M = 256 /
    1,024 / 4,096; profiles/r05_pipe_packed_determinism.txt, DESIGN.md 4.1
    "Nondeterminism"): every one of 4 launches of the shipped assign equals
    the oracle, branch by branch.  D = 2 runs the general filter instance
    (WM 0), whose resolve the compiler used to pack (v_pk_fma_f32 over two
    candidates) until the library was built without SLP vectorization."""
    W, B = 2 * D, 30_000
    g = torch.Generator().manual_seed(M + nb)
    X = torch.randn(B, nb * D, generator=g)
    G = torch.randn(B, nb * D, generator=g) * 1e-3
    emb = torch.rand(nb, M, 2 * D, generator=g) * 2 - 1
    af, bf = torch.ones(nb * D), torch.zeros(nb * D)
    ag, bg = torch.full((nb * D,), 1000.0), torch.zeros(nb * D)
    ref = torch.empty(nb, B, dtype=torch.long)
    for b in range(nb):
        cs = slice(b * D, (b + 1) * D)
        for r0 in range(0, B, 5000):
            rs = slice(r0, r0 + 5000)
            ref[b, rs], _ = vq_ref.assign_with_coef(X[rs, cs], G[rs, cs], af[cs], bf[cs], ag[cs],
                                                    bg[cs], 0.75, emb[b])
    coef = _coef_tensor(af, bf, ag, bg)
    Xd, Gd, Ed = X.to(DEV), G.to(DEV), emb.to(DEV)
    bad = []
    for rep in range(4):
        idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
        kernels.vq_assign(Xd, Gd, coef, 0.75, Ed, D, W, idx_out=idx)
        diff = idx.cpu() != ref
        if diff.any():
            bad.append((rep, int(diff.sum()), diff.any(0).nonzero().flatten()[:6].tolist()))
    assert not bad, f"(launch, mismatching entries, first rows): {bad}"


@pytest.mark.parametrize("M,W", [(256, 8), (256, 4), (1024, 8), (4096, 8), (40, 8)])
def test_assign_near_ties_resolved_exactly(M, W):
    """The filtered sweep (f16-split scores on the MFMA) sends rows whose
    minimum is within its error bound of another codeword's score to the
    exact near-tie sweep.  Crafted ties: exact duplicate codewords, codewords one
    or two ulps apart, and rows placed on the bisector of two codewords --
    every index equals the pinned sequential arithmetic's (first index on
    exact ties; helpers.sequential_argmin -- at the ulp level the box's MKL
    is not that arithmetic for every shape), in every branch, with the EMA
    counts and the scattered codes consistent."""
    D, nb, B, N = 4, 5, 4000, 9000
    g = torch.Generator().manual_seed(M + W)
    emb = torch.randn(nb, M, 2 * D, generator=g) * 0.7
    emb[0, 1::2] = emb[0, 0::2][: M // 2]                       # exact duplicates
    emb[1, 1::2] = torch.nextafter(emb[1, 0::2][: M // 2], torch.tensor(10.0))  # 1 ulp apart
    emb[2, 1::2] = torch.nextafter(torch.nextafter(emb[2, 0::2][: M // 2], torch.tensor(-9.0)),
                                   torch.tensor(-9.0))
    X = torch.randn(B, nb * D, generator=g)
    G = torch.randn(B, nb * D, generator=g) * 1e-3
    # branch 3: rows on the bisector of codewords (2c, 2c+1) in normalised
    # space (identity coefficients below), up to fp32 rounding
    c = torch.randint(0, M // 2, (B,), generator=g)
    mid = 0.5 * (emb[3, 2 * c] + emb[3, 2 * c + 1])
    X[:, 3 * D:4 * D] = mid[:, :D]
    G[:, 3 * D:4 * D] = mid[:, D:]
    coef = torch.zeros(6, nb * D)
    coef[0] = coef[2] = 1.0                          # x -> x (grad half scaled below)
    scale = 1.0
    batch_idx = torch.randperm(N, generator=g)[:B]
    codes = torch.full((N, nb), -1, dtype=torch.int16, device=DEV)
    idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
    stats = kernels.vq_assign(X.to(DEV), G.to(DEV) if W == 2 * D else None, coef.to(DEV), scale,
                              emb.to(DEV), D, W, idx_out=idx, codes=codes,
                              batch_idx=batch_idx.to(DEV), want_stats=True)
    st = kernels.vq_ema_reduce(stats)[0].cpu()
    for b in range(nb):
        xb, gb = X[:, b * D:(b + 1) * D], G[:, b * D:(b + 1) * D]
        xn = torch.cat([xb, gb], 1)[:, :W]              # identity coefficients
        r = torch.from_numpy(sequential_argmin(xn.numpy(), emb[b].numpy()))
        n_mis = int((idx.cpu()[b] != r).sum())
        assert n_mis == 0, f"M={M} W={W} branch {b}: {n_mis} index mismatches"
        assert torch.equal(codes.cpu()[batch_idx, b].long(), r)
        assert torch.equal(st[b, :, 0], torch.bincount(r, minlength=M))


@pytest.mark.parametrize("W", [8, 4])
def test_assign_out_of_range_codewords_and_rows(W):
    """The filter's range limits: codewords with |e|^2 >=
    2^15 are scored +inf and admitted only through the per-workgroup norm
    test, rows with |x|^2 >= 2^16 take the exact sweep.  Branch 0: dead
    codewords with huge norms (|e|^2 up to 10^10, as a trained codebook's
    unused entries reach); branch 1: codewords just past the range with half
    of the rows placed next to them (they must win); branch 2: every 7th row
    scaled past |x|^2 = 2^16, and codewords of the same scale.  Indices equal
    the pinned sequential arithmetic's, EMA counts agree."""
    D, nb, B, N, M = 4, 3, 3000, 6000, 256
    g = torch.Generator().manual_seed(77 + W)
    emb = torch.randn(nb, M, 2 * D, generator=g) * 0.7
    emb[0, 5] *= 1e5
    emb[0, 77] *= 3e4
    emb[0, 200] = 1e4
    big = torch.randn(16, 2 * D, generator=g)
    big = big / big[:, :W].norm(dim=1, keepdim=True) * 190.0        # |e|^2 ~ 36100 > 2^15
    emb[1, 100:116] = big
    emb[2, 40:60] *= 300.0
    X = torch.randn(B, nb * D, generator=g)
    G = torch.randn(B, nb * D, generator=g) * 1e-3
    c = torch.randint(0, 16, (B // 2,), generator=g)
    near = big[c] + 0.01 * torch.randn(B // 2, 2 * D, generator=g)
    X[: B // 2, D:2 * D] = near[:, :D]
    G[: B // 2, D:2 * D] = near[:, D:]
    X[::7, 2 * D:3 * D] *= 300.0
    G[::7, 2 * D:3 * D] = X[::7, 2 * D:3 * D] * 0.5
    coef = torch.zeros(6, nb * D)
    coef[0] = coef[2] = 1.0
    batch_idx = torch.randperm(N, generator=g)[:B]
    codes = torch.full((N, nb), -1, dtype=torch.int16, device=DEV)
    idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
    stats = kernels.vq_assign(X.to(DEV), G.to(DEV) if W == 2 * D else None, coef.to(DEV), 1.0,
                              emb.to(DEV), D, W, idx_out=idx, codes=codes,
                              batch_idx=batch_idx.to(DEV), want_stats=True)
    st = kernels.vq_ema_reduce(stats)[0].cpu()
    for b in range(nb):
        xn = torch.cat([X[:, b * D:(b + 1) * D], G[:, b * D:(b + 1) * D]], 1)[:, :W]
        r = torch.from_numpy(sequential_argmin(xn.numpy(), emb[b].numpy()))
        n_mis = int((idx.cpu()[b] != r).sum())
        assert n_mis == 0, f"W={W} branch {b}: {n_mis} index mismatches"
        assert torch.equal(codes.cpu()[batch_idx, b].long(), r)
        assert torch.equal(st[b, :, 0], torch.bincount(r, minlength=M))
        if b == 1:                          # the out-of-range codewords do win their rows
            assert (r[: B // 2] >= 100).float().mean() > 0.9


def test_assign_multibranch_strided_views_and_codes():
    nb, D, M, B, N = 6, 4, 96, 1200, 5000
    g = torch.Generator().manual_seed(3)
    X = torch.randn(B, nb * D + 3, generator=g)[:, 1:1 + nb * D]     # strided view
    emb = torch.randn(nb, M, 2 * D, generator=g)
    coef = torch.zeros(6, nb * D)
    coef[0], coef[1] = 1.3, -0.2
    batch_idx = torch.randperm(N, generator=g)[:B]
    codes = torch.full((N, nb + 2), -7, dtype=torch.int16)
    Xd = X.to(DEV)
    codes_d = codes.to(DEV)
    idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
    kernels.vq_assign(Xd, None, coef.to(DEV), 1.0, emb.to(DEV), D, D, idx_out=idx,
                      codes=codes_d[:, :nb], batch_idx=batch_idx.to(DEV))
    for b in range(nb):
        xb = X[:, b * D:(b + 1) * D]
        r, _ = vq_ref.assign_with_coef(xb, None, coef[0, :D], coef[1, :D], None, None, 1.0,
                                       emb[b])
        assert torch.equal(idx.cpu()[b], r)
        assert torch.equal(codes_d.cpu()[batch_idx, b].long(), r)
    assert int((codes_d.cpu()[:, nb:] != -7).sum()) == 0


def _bank_from_pre(meta, pre, bn_inited):
    D, M = meta["D"], meta["M"]
    bank = VQBank(1, M, D, grad_normalize_scale=list(meta["grad_scale"]),
                  warm_up_flag=meta["warm_up"], momentum=meta["momentum"]).to(DEV)
    bank.emb[0].copy_(pre["embedding"])
    bank.emb_out[0].copy_(pre["embedding_output"])
    bank.cs[0].copy_(pre["ema_cluster_size"])
    bank.ema_w[0].copy_(pre["ema_w"])
    bank.rm_f[0].copy_(pre["rm_f"])
    bank.rv_f[0].copy_(pre["rv_f"])
    bank.rm_g[0].copy_(pre["rm_g"])
    bank.rv_g[0].copy_(pre["rv_g"])
    bank.bn_inited = [bn_inited]
    return bank


def _bank_state(bank):
    return dict(embedding=bank.emb[0], embedding_output=bank.emb_out[0],
                ema_cluster_size=bank.cs[0], ema_w=bank.ema_w[0], rm_f=bank.rm_f[0],
                rv_f=bank.rv_f[0], rm_g=bank.rm_g[0], rv_g=bank.rv_g[0])


@pytest.mark.parametrize("name", golden_cases())
def test_vq_step_vs_reference_golden(name):
    """Full feature_update / update on the GPU vs the reference's outputs, with
    the inputs in the reference's layout (strided slice or contiguous) and its
    thread count: indices and BatchNorm running stats bit-exact, the logging
    stash bit-exact, the EMA codebook state within 1e-5."""
    meta, calls = load_case(name)
    D, M = meta["D"], meta["M"]
    strided = meta.get("strided", False)
    for c, rec in enumerate(calls):
        bank = _bank_from_pre(meta, rec["pre"], rec["bn_inited_pre"])
        bank.ref_threads = meta.get("threads", 8)
        B = rec["X"].shape[0]
        X = as_layout(rec["X"], strided, DEV)
        G = as_layout(rec["G"], strided, DEV)
        idx = torch.empty(1, B, dtype=torch.long, device=DEV)
        err = ""
        try:
            if meta["op"] == "feature_update":
                bank.feature_update(X, 0, 1, meta["training"], idx_out=idx)
            else:
                bank.update(X, G, 0, 1, meta["training"], idx_out=idx)
        except ValueError as e:
            err = str(e)
        assert err == rec["error"]
        if err:
            return
        got = idx.cpu()[0]
        if not torch.equal(got, rec["idx"]):
            # diagnostics only: how far from a tie are the mismatched rows?
            st = oracle_state_from(meta, rec["pre"], rec["bn_inited_pre"])
            with torch_threads(meta.get("threads", 8)):
                Xc, Gc = as_layout(rec["X"], strided), as_layout(rec["G"], strided)
                if meta["op"] == "feature_update":
                    xn = torch.nn.functional.batch_norm(Xc, st["rm_f"].clone(),
                                                        st["rv_f"].clone(), None, None,
                                                        meta["training"], 0.1, 1e-5)
                    dist = vq_ref.distances(xn, rec["pre"]["embedding"][:, :D])
                else:
                    dist = vq_ref.update(st, Xc, Gc, meta["training"])[2]["distances"]
            n_mis, n_bad = tie_aware_mismatch(got, rec["idx"], dist)
            raise AssertionError(f"{name} call {c}: {n_mis} index mismatches "
                                 f"({n_mis - n_bad} within 1e-5 of a tie)")
        post = _bank_state(bank)
        for k in ("rm_f", "rv_f", "rm_g", "rv_g"):
            assert torch.equal(post[k].cpu(), rec["post"][k]), f"{name} call {c} {k}"
        for k in ("embedding", "embedding_output", "ema_cluster_size", "ema_w"):
            a, b = post[k].cpu(), rec["post"][k]
            # relative to the row scale: EMA sums are exact here and fp32 MKL
            # sums in the reference
            scale = 1.0 + b.abs().amax(dim=-1, keepdim=True) if b.dim() == 2 else 1.0 + b.abs()
            err_rel = ((a - b).abs() / scale).max().item()
            assert err_rel < 1e-5, f"{name} call {c} {k}: max rel err {err_rel:.2e}"
        if meta["op"] == "update":
            # logging stash (vq.py:208-211): torch.mean / torch.var of the
            # [B, 2D] concatenation take ATen's interleaved row_sum / Welford
            # reductions (vector-width dependent); the stash comes from the
            # BN statistics -- equal up to a few ulps of the column scale
            std_ref = rec["logs"]["std"][0]
            got_std = torch.cat([bank.last_batch[1], bank.last_batch[3]]).cpu()
            got_mean = torch.cat([bank.last_batch[0], bank.last_batch[2]]).cpu()
            torch.testing.assert_close(got_std, std_ref, rtol=1e-6, atol=0)
            assert ((got_mean - rec["logs"]["mean"][0]).abs() <= 1e-6 * std_ref).all()


BN_SHAPES = [(2, 1), (3, 2), (17, 3), (40, 8), (700, 8), (1031, 5), (4096, 4), (4113, 8),
             (20000, 7), (65537, 8), (84670, 16), (600001, 8)]


@pytest.mark.parametrize("B,T", BN_SHAPES)
@pytest.mark.parametrize("strided", [True, False])
def test_bn_coefficients_bit_exact(B, T, strided):
    """vqgnn_bn_stats_finalize in the ATen arithmetic of each layout against
    oracle/bn_ref.py (itself pinned to ATen): normalised values, running stats
    (train, init, eval) and the logging stash, bit for bit."""
    from oracle import bn_ref
    if not strided and B > 70000:
        pytest.skip("contiguous restatement loops in Python")
    rng = np.random.default_rng(B + 7 * T)
    D = 4
    X = torch.from_numpy((rng.standard_normal((B, D)) * rng.uniform(0.05, 5)
                          + rng.uniform(-3, 3)).astype(np.float32))
    Gt = torch.from_numpy((rng.standard_normal((B, D)) * 1e-3).astype(np.float32))
    rm = torch.from_numpy(rng.standard_normal(D).astype(np.float32))
    rv = torch.from_numpy(rng.uniform(0.3, 2, D).astype(np.float32))
    ar = kernels.BN_STRIDED if strided else kernels.BN_CONTIG
    Xd, Gd = as_layout(X, strided, DEV), as_layout(Gt, strided, DEV)
    for mode in (kernels.BN_TRAIN, kernels.BN_TRAIN_INIT, kernels.BN_EVAL, kernels.BN_EVAL_INIT):
        if B < 2 and mode != kernels.BN_EVAL:
            continue
        rmf, rvf, rmg, rvg = (t.clone().to(DEV) for t in (rm, rv, rm * 0.1, rv))
        coef, batch, _ = kernels.bn_stats_finalize(
            Xd, Gd, D, mode, 0.1, 1e-5, 0.3, 1e-24, 1e-24, rmf, rvf, rmg, rvg,
            want_batch=True, arith_x=ar, arith_g=ar, ref_threads=T)
        coef, batch = coef.cpu(), batch.cpu()
        for half, (Z, r0, v0, mom, eps, rmo, rvo) in enumerate(
                ((X, rm, rv, 0.1, 1e-5, rmf, rvf), (Gt, rm * 0.1, rv, 0.3, 1e-24, rmg, rvg))):
            Zn = Z.numpy()
            r1, v1 = r0.numpy(), v0.numpy()
            if mode in (kernels.BN_TRAIN_INIT, kernels.BN_EVAL_INIT):
                r1, v1 = bn_ref.torch_mean(Zn), bn_ref.torch_var(Zn)
            if mode in (kernels.BN_TRAIN, kernels.BN_TRAIN_INIT):
                out, r2, v2, *_ = bn_ref.bn_train(Zn, r1, v1, mom, eps, not strided, T)
            else:
                out, *_ = bn_ref.bn_eval(Zn, r1, v1, eps, not strided)
                r2, v2 = r1, v1
            a, b_, sh = coef[2 * half], coef[2 * half + 1], coef[4 + half]
            got = ((Z - sh).double() * a.double() + b_.double()).float()   # fma(x-sh, a, b)
            np.testing.assert_array_equal(got.numpy(), out, err_msg=f"mode {mode} half {half}")
            np.testing.assert_array_equal(rmo.cpu().numpy(), r2)
            np.testing.assert_array_equal(rvo.cpu().numpy(), v2)
            np.testing.assert_array_equal(batch[2 * half].numpy(), bn_ref.torch_mean(Zn))
            std = np.sqrt((bn_ref.torch_var(Zn) + np.float32(1e-24)).astype(np.float32))
            np.testing.assert_array_equal(batch[2 * half + 1].numpy(), std)


def test_module_api_update_and_state_dict():
    torch.manual_seed(0)
    m = VectorQuantizerEMA(64, 4, grad_normalize_scale=[1, 1], warm_up_flag=True).to(DEV)
    X = torch.randn(500, 4, device=DEV)
    G = torch.randn(500, 4, device=DEV) * 1e-3
    m.train()
    idx = m.feature_update(X)
    assert idx.shape == (500, 1) and idx.dtype == torch.long
    idx2, enc = m.update(X, G)
    assert enc.shape == (500, 64)
    assert torch.equal(enc.to_dense().argmax(1).cpu(), idx2[:, 0].cpu())
    assert m.bn_inited and m.mean.shape == (1, 8) and m.std.shape == (1, 8)
    assert m.running_std.shape == (1, 8)
    assert 0 <= float(m.feat_zero_rate) <= 1
    sd = m.state_dict()
    for k in ("_embedding", "_embedding_output", "_ema_cluster_size", "_ema_w",
              "batch_norm_feat.running_mean", "batch_norm_feat.running_var",
              "batch_norm_grad.running_mean", "batch_norm_grad.num_batches_tracked"):
        assert k in sd, k
    assert m.get().shape == (64, 8) and m.get_codebook().shape == (64, 4)


def test_bad_init_raises_on_gpu():
    meta, calls = load_case("fu_bad_init")
    rec = calls[0]
    bank = _bank_from_pre(meta, rec["pre"], False)
    with pytest.raises(ValueError, match="Bad Init!"):
        bank.feature_update(rec["X"].to(DEV), 0, 1, True)


def test_update_eval_mode_stashes_batch_stats():
    """vq.py:208-211: update() records the batch mean / std in every mode,
    including eval after the running statistics were initialised."""
    torch.manual_seed(3)
    m = VectorQuantizerEMA(64, 4, grad_normalize_scale=[1, 1], warm_up_flag=True).to(DEV)
    m.train()
    m.update(torch.randn(400, 4, device=DEV), torch.randn(400, 4, device=DEV) * 1e-3)
    m.eval()
    X = torch.randn(300, 4, device=DEV) * 2 + 1
    G = torch.randn(300, 4, device=DEV) * 1e-3
    rm = m.batch_norm_feat.running_mean.clone()
    m.update(X, G)
    inputs = torch.cat([X, G], 1)
    torch.testing.assert_close(m.mean, inputs.mean(0, keepdim=True), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m.std, torch.sqrt(inputs.var(0, keepdim=True) + 1e-24),
                               rtol=1e-5, atol=1e-7)
    assert torch.equal(m.batch_norm_feat.running_mean, rm)      # eval: running stats untouched


@pytest.mark.parametrize("M,W,nb,B", [(4096, 8, 3, 5000), (5000, 4, 2, 3001), (4096, 8, 1, 700)])
def test_split_ema_statistics_equal_global(M, W, nb, B, monkeypatch):
    """Codebooks whose int64 EMA slab exceeds the LDS (ppi: M = 4096, W = 8)
    accumulate per codeword range in LDS (vq_ema_split_kernel); the slab is
    integer, so it must equal the global-atomics path exactly, and its counts
    the bincount of the indices."""
    from vq_gnn_amd import kernels
    D = 4
    F = nb * D
    g = torch.Generator().manual_seed(M + B)
    X = (torch.randn(B, F, generator=g) * 2).to(DEV)
    G = (torch.randn(B, F, generator=g) * 1e-3).to(DEV)
    emb = torch.randn(nb, M, 2 * D, generator=g).to(DEV)
    coef = torch.zeros(6, F)
    coef[0] = coef[2] = 1.0
    coef = coef.to(DEV)
    out = {}
    for mode in ("split", "global"):
        if mode == "global":
            monkeypatch.setenv("VQGNN_EMA_GLOBAL", "1")
        idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
        st = kernels.vq_assign(X, G if W == 2 * D else None, coef, 1.0, emb, D, W, idx_out=idx,
                               want_stats=True, stat_count=B)
        out[mode] = (idx.clone(), kernels.vq_ema_reduce(st).clone())
    monkeypatch.delenv("VQGNN_EMA_GLOBAL", raising=False)
    torch.cuda.synchronize()
    assert torch.equal(out["split"][0], out["global"][0])
    assert torch.equal(out["split"][1], out["global"][1])
    stats = out["split"][1].view(nb, M, W + 1)
    for b in range(nb):
        assert torch.equal(stats[b, :, 0].cpu(),
                           torch.bincount(out["split"][0][b].cpu(), minlength=M)), b
