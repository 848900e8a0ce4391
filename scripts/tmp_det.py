"""Repeat-launch determinism of the assign over many branches (diagnostic)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vqgnn_pkg
vqgnn_pkg.load()
from vq_gnn_amd import kernels
DEV = torch.device("cuda:0")
D, W = 4, 8
for (M, nb, B) in ((4096, 13, 30000), (1024, 32, 30000), (256, 32, 30000)):
    g = torch.Generator().manual_seed(M + nb)
    X = torch.randn(B, nb * D, generator=g).to(DEV)
    G = (torch.randn(B, nb * D, generator=g) * 1e-3).to(DEV)
    emb = (torch.rand(nb, M, 2 * D, generator=g) * 2 - 1).to(DEV)
    coef = torch.zeros(6, nb * D)
    coef[0] = 1.0; coef[2] = 1000.0
    coef = coef.to(DEV)
    ref = None
    for rep in range(int(os.environ.get("REPS", "8"))):
        idx = torch.empty(nb, B, dtype=torch.long, device=DEV)
        kernels.vq_assign(X, G, coef, 0.75, emb, D, W, idx_out=idx)
        torch.cuda.synchronize()
        if ref is None:
            ref = idx.clone()
            continue
        diff = (idx != ref)
        n = int(diff.sum())
        if n:
            rows = diff.any(0).nonzero().flatten()[:6].tolist()
            print(M, nb, B, "rep", rep, "differs from launch 0 in", n, "entries; rows", rows, flush=True)
    print(M, nb, B, "done", flush=True)
