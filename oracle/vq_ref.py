"""Oracle for VectorQuantizerEMA (reference: vq_gnn_v2/vq.py:60-279).

Op-for-op restatement with torch CPU ops, on an explicit state dict, so a test
can feed the same pre-state to the HIP path and compare post-states.  Every
line cites the reference line it restates.  TEST INFRASTRUCTURE ONLY.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def new_state(M, D, grad_scale=(1.0, 1.0), warm_up=False, momentum=0.1, decay=0.99,
              epsilon=1e-24, generator=None):
    """vq.py:61-100 (add_flag=False)."""
    W = 2 * D
    st = dict(M=M, D=D, decay=decay, epsilon=epsilon, grad_scale=list(grad_scale),
              warm_up=warm_up, momentum=momentum, bn_inited=False)
    st["embedding"] = torch.randn(M, W, generator=generator)                     # :73
    st["embedding_output"] = torch.zeros(M, W)                                    # :74
    st["ema_cluster_size"] = torch.zeros(M)                                       # :76
    st["ema_w"] = torch.zeros(M, W)                                               # :77
    if warm_up:
        st["ema_w"].normal_(generator=generator)                                  # :79-80
    st["rm_f"], st["rv_f"] = torch.zeros(D), torch.ones(D)                        # :86
    st["rm_g"], st["rv_g"] = torch.zeros(D), torch.ones(D)                        # :87-88
    st["embedding"][:, D:2 * D] *= st["grad_scale"][0]                            # :93
    st["ema_w"][:, D:2 * D] *= st["grad_scale"][0]                                # :94
    return st


def clone_state(st):
    return {k: (v.clone() if isinstance(v, torch.Tensor) else
                (list(v) if isinstance(v, list) else v)) for k, v in st.items()}


def _bn(x, rm, rv, training, momentum, eps):
    # nn.BatchNorm1d(affine=False).forward == F.batch_norm with the running stats
    return F.batch_norm(x, rm, rv, None, None, training, momentum, eps)


def distances(xn, emb):
    """vq.py:166-168 / :230-232 (same expression, same op order)."""
    return (torch.sum(xn ** 2, dim=1, keepdim=True)
            + torch.sum(emb ** 2, dim=1)
            - 2 * torch.matmul(xn, emb.t()))


def feature_update(st, X_B, training=True):
    """vq.py:160-202.  Mutates st; returns encoding_indices [B, 1] (int64)."""
    D, M = st["D"], st["M"]
    xn = _bn(X_B, st["rm_f"], st["rv_f"], training, 0.1, 1e-5)                  # :162
    emb = st["embedding"][:, :D]                                                 # :163
    d = distances(xn, emb)                                                       # :166-168
    idx = torch.argmin(d, dim=1).unsqueeze(1)                                    # :171
    enc = torch.zeros(idx.shape[0], M)                                           # :172
    enc.scatter_(1, idx, 1)                                                      # :173
    if training:
        decay = st["decay"]
        st["ema_cluster_size"] = st["ema_cluster_size"] * decay + \
            (1 - decay) * torch.sum(enc, 0)                                      # :177-178
        if st["warm_up"]:
            n = torch.sum(st["ema_cluster_size"])                                # :183
            st["ema_cluster_size"] = ((st["ema_cluster_size"] + 1e-5)
                                      / (n + M * 1e-5) * n)                      # :184-186
        if torch.count_nonzero(st["ema_cluster_size"]) != M:                     # :188
            raise ValueError('Bad Init!')
        dw = torch.matmul(enc.t(), xn)                                           # :191
        st["ema_w"][:, :D] = st["ema_w"][:, :D] * decay + (1 - decay) * dw       # :193-194
        st["embedding"][:, :D] = st["ema_w"][:, :D] / st["ema_cluster_size"].unsqueeze(1)  # :195-196
        rstd = torch.sqrt(st["rv_f"] + 1e-5).unsqueeze(0)                        # :198
        rmean = st["rm_f"].unsqueeze(0)                                          # :199
        st["embedding_output"][:, :D] = st["embedding"][:, :D] * rstd + rmean    # :200
    return idx


def update(st, X_B, grad, training=True):
    """vq.py:204-279.  Mutates st; returns (encoding_indices, encodings, logs)."""
    D, M, eps = st["D"], st["M"], st["epsilon"]
    inputs = torch.cat([X_B, grad], dim=1)                                       # :206
    mean = torch.mean(inputs, dim=0, keepdim=True)                               # :208
    std = torch.sqrt(torch.var(inputs, dim=0, keepdim=True) + eps)               # :209
    logs = dict(mean=mean, std=std,
                feat_zero_rate=torch.sum(torch.abs(inputs[:, 0]) < std[0][0] * 1e-5) / X_B.shape[0],
                grad_zero_rate=torch.sum(inputs[:, D] < std[0][D] * 1e-5) / X_B.shape[0])  # :213-214
    if not st["bn_inited"]:                                                      # :216-221
        st["rm_f"] = torch.mean(X_B, dim=0)
        st["rv_f"] = torch.var(X_B, dim=0)
        st["rm_g"] = torch.mean(grad, dim=0)
        st["rv_g"] = torch.var(grad, dim=0)
        st["bn_inited"] = True
    xn = torch.cat([_bn(X_B, st["rm_f"], st["rv_f"], training, 0.1, 1e-5),
                    _bn(grad, st["rm_g"], st["rv_g"], training, st["momentum"], eps)], dim=1)  # :223
    xn[:, D:2 * D] *= st["grad_scale"][0]                                        # :224
    d = distances(xn, st["embedding"])                                           # :230-232
    logs["distances"] = d          # (oracle extra: what argmin ran on, for diagnostics)
    idx = torch.argmin(d, dim=1).unsqueeze(1)                                    # :236
    enc = torch.zeros(idx.shape[0], M)                                           # :237
    enc.scatter_(1, idx, 1)                                                      # :238
    if training:
        decay = st["decay"]
        st["ema_cluster_size"] = st["ema_cluster_size"] * decay + \
            (1 - decay) * torch.sum(enc, 0)                                      # :242-243
        if st["warm_up"]:
            n = torch.sum(st["ema_cluster_size"])                                # :248
            st["ema_cluster_size"] = ((st["ema_cluster_size"] + 1e-5)
                                      / (n + M * 1e-5) * n)                      # :249-251
        if torch.count_nonzero(st["ema_cluster_size"]) != M:                     # :253
            raise ValueError('Bad Init!')
        dw = torch.matmul(enc.t(), xn)                                           # :256
        st["ema_w"] = st["ema_w"] * decay + (1 - decay) * dw                     # :258
        st["embedding"] = st["ema_w"] / st["ema_cluster_size"].unsqueeze(1)      # :259
        out = st["embedding"].detach().clone()                                   # :261
        out[:, D:2 * D] /= st["grad_scale"][0] + eps                             # :263
        rv = torch.cat([st["rv_f"] + 1e-5, st["rv_g"] + eps])                    # :267
        rstd = torch.sqrt(rv).unsqueeze(0)                                       # :268
        rmean = torch.cat([st["rm_f"], st["rm_g"]]).unsqueeze(0)                 # :270-271
        st["embedding_output"] = out * rstd + rmean                              # :272
        if st["grad_scale"][0] == 0:                                             # :274-275
            st["embedding_output"][:, D:] *= 0
        logs["running_mean"], logs["running_std"] = rmean, rstd                  # :276-277
    return idx, enc, logs


def bn_coefficients(X, training, rm, rv, eps):
    """The (alpha, beta) ATen's CPU batch_norm applies: y = fma(x, alpha, beta)
    with alpha = invstd, beta = -(mean * invstd).  Used to feed identical
    coefficients to the HIP assign kernel for bit-exact index tests."""
    if training:
        _, save_mean, save_invstd = torch.native_batch_norm(
            X, None, None, rm.clone(), rv.clone(), True, 0.1, eps)
        alpha = save_invstd
        beta = -(save_mean * save_invstd)
    else:
        alpha = 1.0 / torch.sqrt(rv + eps)
        beta = -(rm * alpha)
    return alpha.float(), beta.float()


def assign_with_coef(X, G, alpha_f, beta_f, alpha_g, beta_g, scale, emb):
    """Nearest codeword given explicit normalisation coefficients, in ATen's
    arithmetic (fma BN, sequential sums, MKL sgemm == sequential fma).
    Returns (idx [B] int64, distances [B, M])."""
    import numpy as np
    xf = X.double() * alpha_f.double() + beta_f.double()      # exact product + 1 rounding = fma
    parts = [xf.float()]
    if G is not None:
        xg = (G.double() * alpha_g.double() + beta_g.double()).float() * scale
        parts.append(xg)
    xn = torch.cat(parts, dim=1)
    W = xn.shape[1]
    d = distances(xn, emb[:, :W])
    return torch.argmin(d, dim=1), d
