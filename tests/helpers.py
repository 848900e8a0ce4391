"""Shared test helpers (golden loading, tie-aware index comparison)."""
import ast
import glob
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

STATE_KEYS = ("embedding", "embedding_output", "ema_cluster_size", "ema_w",
              "rm_f", "rv_f", "rm_g", "rv_g")


def golden_cases():
    return sorted(os.path.basename(p)[3:-4] for p in glob.glob(os.path.join(GOLDEN, "vq_*.npz")))


def load_case(name):
    z = np.load(os.path.join(GOLDEN, f"vq_{name}.npz"), allow_pickle=False)
    meta = ast.literal_eval(str(z["meta"]))
    calls = []
    for c in range(meta["calls"]):
        p = f"c{c}_"
        if p + "X" not in z:
            break
        rec = dict(X=torch.from_numpy(z[p + "X"]), G=torch.from_numpy(z[p + "G"]),
                   idx=torch.from_numpy(z[p + "idx"]), error=str(z[p + "error"]),
                   bn_inited_pre=bool(z[p + "bn_inited_pre"]),
                   pre={k: torch.from_numpy(z[p + "pre_" + k]) for k in STATE_KEYS},
                   post={k: torch.from_numpy(z[p + "post_" + k]) for k in STATE_KEYS})
        logs = {k[len(p) + 4:]: torch.from_numpy(z[k]) for k in z.files if k.startswith(p + "log_")}
        rec["logs"] = logs
        calls.append(rec)
    return meta, calls


def oracle_state_from(meta, pre, bn_inited):
    st = dict(M=meta["M"], D=meta["D"], decay=0.99, epsilon=1e-24,
              grad_scale=list(meta["grad_scale"]), warm_up=meta["warm_up"],
              momentum=meta["momentum"], bn_inited=bn_inited)
    for k in STATE_KEYS:
        st[k] = pre[k].clone()
    return st


def tie_aware_mismatch(idx_a, idx_b, dist, rel=1e-5):
    """Rows where idx_a != idx_b; returns (n_mismatch, n_unexplained) where a
    mismatch is explained when the two candidates' distances (under the
    oracle's own distances ``dist`` [B, M]) are within rel of the scale."""
    idx_a = torch.as_tensor(idx_a).long().view(-1)
    idx_b = torch.as_tensor(idx_b).long().view(-1)
    bad = torch.nonzero(idx_a != idx_b).view(-1)
    if bad.numel() == 0:
        return 0, 0
    da = dist[bad, idx_a[bad]].double()
    db = dist[bad, idx_b[bad]].double()
    scale = 1.0 + dist[bad].abs().max(dim=1).values.double()
    unexplained = int(((da - db).abs() > rel * scale).sum())
    return int(bad.numel()), unexplained


def as_layout(t, strided, device=None):
    """``t`` [B, D] as the reference received it: a column slice of a wider
    row-major matrix when ``strided`` (ATen's non-contiguous BatchNorm path,
    as the layers' x[:, D*i:D*(i+1)]), else a contiguous tensor."""
    t = t.to(device) if device is not None else t
    if not strided:
        return t.contiguous()
    B, D = t.shape
    wide = torch.zeros(B, 3 * D, dtype=t.dtype, device=t.device)
    wide[:, D:2 * D] = t
    return wide[:, D:2 * D]


class torch_threads:
    """Context manager: torch.set_num_threads(n), restored on exit (the
    reference's contiguous-input BatchNorm depends on the thread count)."""

    def __init__(self, n):
        self.n = n

    def __enter__(self):
        self.old = torch.get_num_threads()
        torch.set_num_threads(self.n)

    def __exit__(self, *a):
        torch.set_num_threads(self.old)


def sequential_argmin(xn, emb, window=1e-3):
    """argmin_m of the distance in the arithmetic the golden fixtures pin
    (vq.py:166-171 as restated in oracle/vq_ref.py): |x|^2 and |e|^2 summed
    sequentially in fp32, x.e as a k-ordered fp32 fma chain from fl(e0 x0),
    d = fl(fl(|x|^2 + |e|^2) - 2 x.e), first index on ties -- evaluated
    exactly (Fraction arithmetic) for every codeword within ``window`` of the
    fp64 minimum.  The fixtures were generated on this container's CPU; the
    GPU box's MKL picks other sgemm kernels for some shapes, whose last-ulp
    rounding differs, so ulp-level near-ties are checked against this model.
    xn [B, W] float32, emb [M, >= W] float32 -> int64 [B]."""
    from fractions import Fraction

    xn = np.asarray(xn, np.float32)
    W = xn.shape[1]
    e = np.asarray(emb, np.float32)[:, :W]
    d64 = ((xn.astype(np.float64) ** 2).sum(1)[:, None] + (e.astype(np.float64) ** 2).sum(1)[None]
           - 2 * xn.astype(np.float64) @ e.astype(np.float64).T)
    lo = d64.min(1)

    def f32(v):
        return np.float32(float(v))

    def seqsq(v):
        s = f32(Fraction(float(v[0])) * Fraction(float(v[0])))
        for k in range(1, len(v)):
            s = f32(Fraction(float(s)) + Fraction(float(f32(Fraction(float(v[k])) ** 2))))
        return s

    se_cache = {}
    out = np.empty(xn.shape[0], np.int64)
    for i in range(xn.shape[0]):
        x = xn[i]
        sx = seqsq(x)
        best, bm = None, -1
        for m in np.nonzero(d64[i] <= lo[i] + window)[0]:
            if m not in se_cache:
                se_cache[m] = seqsq(e[m])
            dot = f32(Fraction(float(e[m, 0])) * Fraction(float(x[0])))
            for k in range(1, W):
                dot = f32(Fraction(float(e[m, k])) * Fraction(float(x[k])) + Fraction(float(dot)))
            S = f32(Fraction(float(sx)) + Fraction(float(se_cache[m])))
            d = f32(Fraction(float(S)) - 2 * Fraction(float(dot)))
            if best is None or d < best:
                best, bm = d, m
        out[i] = bm
    return out
