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
