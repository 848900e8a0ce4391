"""Time the GAT backward kernels (edge grad, att grad) on the arxiv batch."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vqgnn_pkg
vqgnn_pkg.load()
from vq_gnn_amd import kernels
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch

DEV = torch.device("cuda:0")
g, _, b = make_batch(CONFIGS["arxiv_gat"])
bidx, subset, adj = batch_to_device(b, DEV)
n, B, F = b.n, b.B, 128
x = torch.randn(B, F, device=DEV)
xf = torch.randn(n - B, F, device=DEV)
att_l = torch.randn(F + 1, device=DEV) * 0.1
att_r = torch.randn(F + 1, device=DEV) * 0.1
al, ar, params = kernels.gat_alpha(x, att_l, att_r, F, X2=xf, B=B, ones=True)
coef, den = kernels.gat_coef(adj.rowptr, adj.col, adj.value, n, adj.nnz(), al, ar, params)
dy = torch.randn(n, F, device=DEV)
dden = torch.randn(n, device=DEV)
for dbg in ("0",):
    f = lambda: kernels.gat_edge_grad(adj.rows(), adj.col, coef, adj.nnz(), x, F, dy, dden, al, ar, params, X2=xf, B=B)  # noqa: E731
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        f()
    e1.record()
    torch.cuda.synchronize()
    print(f"dbg={dbg}: {e0.elapsed_time(e1) / 5 * 1e3:.1f} us (incl. 3 zero-fills)", flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    kernels.gat_att_grad(x, F, al, ar, X2=xf, B=B, ones=True)
e1.record()
torch.cuda.synchronize()
print(f"att_grad: {e0.elapsed_time(e1) / 5 * 1e3:.1f} us", flush=True)
