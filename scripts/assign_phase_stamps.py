"""Per-iteration phase times of the assign's row loop from s_memtime stamps
(a variant library built with the stamps: VQGNN_LIB=vq-gnn_amd/lib/ab_vqtime.so,
exporting vqgnn_dbg_vq_times).  Wave 0 of workgroups 0..255, first 16 row
iterations: t0 top | t1 rows normalised, split, B fragments built | t2
sweep done | t3 resolve done | t4 outputs + EMA statistics issued.
Config as bench.py's arxiv step (B = 84,670, nb = 32, M = 256 or M=<env>)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd._lib import lib  # noqa: E402

DEV = torch.device("cuda:0")
B, nb, D = 84670, 32, 4
M = int(os.environ.get("M", "256"))
F, W = nb * D, 8
torch.manual_seed(0)
X = torch.randn(B, F, device=DEV)
G = torch.randn(B, F, device=DEV) * 1e-3
emb = torch.randn(nb, M, 2 * D, device=DEV)
rm, rv = torch.zeros(F, device=DEV), torch.ones(F, device=DEV)
coef, _, _ = kernels.bn_stats_finalize(X, G, F, kernels.BN_TRAIN, 0.1, 1e-5, 0.1, 1e-24, 1e-24,
                                       rm, rv, rm.clone(), rv.clone())
codes = torch.zeros(200000, nb, dtype=torch.int16, device=DEV)
bidx = torch.randperm(200000, device=DEV)[:B]
slab = torch.zeros(1, nb, M, W + 1, dtype=torch.int64, device=DEV)
L = lib()
L.vqgnn_dbg_vq_times.restype = ctypes.c_int
L.vqgnn_dbg_vq_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
n = 256 * 16 * 8
for rep in range(5):
    slab.zero_()
    kernels.vq_assign(X, G, coef, 1.0, emb, D, W, codes=codes, batch_idx=bidx, want_stats=True,
                      stat_count=B, stats_out=slab)
torch.cuda.synchronize()
buf = np.zeros(n, dtype=np.uint64)
assert L.vqgnn_dbg_vq_times(buf.ctypes.data, n) == 0
t = buf.reshape(256, 16, 8)[:, :, :5].astype(np.int64)
valid = (t[:, :, 0] > 0) & (t[:, :, 4] > t[:, :, 0])
ph = np.diff(t, axis=2)                       # [wg, it, 4]
names = ["rows+split+B frags", "sweep", "resolve", "outputs+EMA"]
print(f"M={M}: {int(valid.sum())} stamped iterations (wave 0, {valid.any(1).sum()} workgroups)")
for k, nm in enumerate(names):
    v = ph[:, :, k][valid]
    print(f"  {nm:22s} mean {v.mean():8.0f}  median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f} cycles")
it_total = (t[:, :, 4] - t[:, :, 0])[valid]
print(f"  {'iteration':22s} mean {it_total.mean():8.0f}  median {np.median(it_total):8.0f}")
# gap between iterations (t0 of it+1 minus t4 of it): the next row's load wait etc.
g = (t[:, 1:, 0] - t[:, :-1, 4])[valid[:, 1:] & valid[:, :-1]]
print(f"  {'between iterations':22s} mean {g.mean():8.0f}  median {np.median(g):8.0f}")
