"""Timeline of the SpMM wave kernel from s_memtime stamps (VQGNN_SPMM_DEBUG=4)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["VQGNN_SPMM_DEBUG"] = os.environ.get("VQGNN_SPMM_DEBUG", "4")
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels, _lib  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402

dev = torch.device("cuda:0")
cfg = CONFIGS["arxiv_gcn"]
g, _, b = make_batch(cfg)
bidx, subset, adj = batch_to_device(b, dev)
Xn = torch.randn(b.n, 128, device=dev)
for _ in range(3):
    kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, Xn, 128)
torch.cuda.synchronize()
L = _lib.lib()
f = L.vqgnn_debug_spmm_stamps
f.restype = ctypes.c_int64
f.argtypes = [ctypes.c_void_p, ctypes.c_int64]
n = f(None, 0)
buf = np.zeros(n, dtype=np.uint64)
f(buf.ctypes.data, n)
st = buf.reshape(-1, 4).astype(np.int64)
st = st[st[:, 3] > 0]
t0 = st[:, 0].min()
start, search, end = st[:, 0] - t0, st[:, 1] - st[:, 0], st[:, 2] - st[:, 1]
# s_memtime ticks (100 MHz on gfx9 ref clock? report raw and scaled)
print("waves", len(st), "span ticks", (st[:, 2].max() - t0))
for name, v in (("start offset", start), ("head (kernarg+search)", search), ("chunks", end)):
    print(f"{name:24s} median {np.median(v):10.0f}  p10 {np.percentile(v, 10):10.0f}  "
          f"p90 {np.percentile(v, 90):10.0f}  max {v.max():10.0f}")
lifetime = st[:, 2] - st[:, 0]
print(f"{'lifetime':24s} median {np.median(lifetime):10.0f}  mean {lifetime.mean():10.0f}")
# concurrency: average resident waves = sum(lifetime) / span
print("mean resident waves", lifetime.sum() / (st[:, 2].max() - t0))
