"""Debug (GPU): undecided-row counts of the filtered assign path (switched on
here with vqgnn_assign_filter(1)), determinism, and agreement with an fp64
argmin on the microbench data."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd._lib import lib, ptr, stream_ptr, check  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
B, nb, M, D = int(os.environ.get("FD_B", 84670)), 32, 256, 4
F = nb * D
X = torch.randn(B, F, device=dev)
G = torch.randn(B, F, device=dev) * 1e-3
emb = torch.randn(nb, M, 2 * D, device=dev)
coef = torch.zeros(6, F, device=dev)
coef[0] = 1.0
coef[2] = 1.0
L = lib()
L.vqgnn_assign_filter(1)
W = 2 * D
for trial in range(2):
    ws = torch.zeros(L.vqgnn_vq_assign_workspace(B, nb, M, W) // 4 + 64, dtype=torch.int32,
                     device=dev)
    idx = torch.empty(nb, B, dtype=torch.int64, device=dev)
    check(L.vqgnn_vq_assign(ptr(X), X.stride(0), ptr(G), G.stride(0), B, nb, D, M, W, ptr(coef),
                            1.0, ptr(emb), 2 * D, emb.stride(0), ptr(idx), None, 0, None, None, 0,
                            B, ptr(ws), stream_ptr()), "assign")
    torch.cuda.synchronize()
    cnt = ws[:nb].cpu()
    print("trial", trial, "fallback rows per branch:", cnt.tolist()[:8], "total", int(cnt.sum()),
          f"({int(cnt.sum()) / (B * nb):.3%})")
    if trial == 0:
        first = idx.clone()
    else:
        print("deterministic:", bool(torch.equal(first, idx)))
# exact reference: squared distances in fp64 argmin (tie-free random data)
xs = X.view(B, nb, D)
gs = G.view(B, nb, D)
xx = torch.cat([xs, gs], 2).double()          # BN coef = identity, grad scale 1
e = emb.double()
d = (xx * xx).sum(2)[:, :, None] + (e * e).sum(2)[None] - 2 * torch.einsum("bnk,nmk->bnm", xx, e)
ref = d.argmin(2).T
print("mismatch vs fp64 argmin:", int((ref != first).sum()))
