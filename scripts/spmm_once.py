"""Run the default SpMM of the arxiv bench batch N times (for rocprofv3
kernel-trace comparisons of plan / kernel variants set through VQGNN_* env)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402

dev = torch.device("cuda:0")
cfg = dict(CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "arxiv_gcn"])
n_rep = int(sys.argv[2]) if len(sys.argv) > 2 else 20
g, _, b = make_batch(cfg)
F = cfg["F"]
bidx, subset, adj = batch_to_device(b, dev)
X = torch.randn(b.B, F, device=dev)
X2 = torch.randn(b.n - b.B, F, device=dev)
out = torch.empty(b.n, F, device=dev)
plan = adj.plan(F, B=b.B)
for _ in range(n_rep):
    kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=X2, B=b.B, out=out, plan=plan)
torch.cuda.synchronize()
print("done", type(plan).__name__)
