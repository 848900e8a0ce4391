"""Debug the filtered assign on one small case: mismatching rows, their exact
distances and the rank of the GPU's pick."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vqgnn_pkg
vqgnn_pkg.load()
from vq_gnn_amd import kernels
from oracle import vq_ref
DEV = torch.device("cuda:0")
for (M, D, W, B) in [(64, 4, 8, 512), (256, 4, 8, 3000), (256, 4, 4, 3000)]:
    g = torch.Generator().manual_seed(M * 7 + B)
    X = torch.randn(B, D, generator=g) * 2 + 0.5
    G = torch.randn(B, D, generator=g) * 1e-3
    emb = torch.randn(M, 2 * D, generator=g)
    af, bf = vq_ref.bn_coefficients(X, True, torch.zeros(D), torch.ones(D), 1e-5)
    ag, bg = vq_ref.bn_coefficients(G, True, torch.zeros(D), torch.ones(D), 1e-24)
    scale = 0.75
    idx_ref, _ = vq_ref.assign_with_coef(X, G if W == 2 * D else None, af, bf, ag, bg, scale, emb)
    coef = torch.zeros(6, D)
    coef[0], coef[1], coef[2], coef[3] = af, bf, ag, bg
    idx = torch.empty(1, B, dtype=torch.long, device=DEV)
    kernels.vq_assign(X.to(DEV), G.to(DEV) if W == 2 * D else None, coef.to(DEV), scale,
                      emb.view(1, M, 2 * D).to(DEV), D, W, idx_out=idx)
    torch.cuda.synchronize()
    gi = idx.cpu()[0]
    xn = X * af + bf
    gn = (G * ag + bg) * scale
    z = torch.cat([xn, gn], 1)[:, :W].double()
    e = emb[:, :W].double()
    d = (z * z).sum(1, keepdim=True) + (e * e).sum(1)[None] - 2 * z @ e.T
    bad = (gi != idx_ref).nonzero().flatten()
    print(f"M={M} D={D} W={W} B={B}: {len(bad)} mismatches")
    for r in bad[:8].tolist():
        rank = int((d[r] < d[r, gi[r]]).sum())
        print(f"  row {r}: gpu {int(gi[r])} ref {int(idx_ref[r])} d_gpu {d[r, gi[r]]:.6f} "
              f"d_ref {d[r, idx_ref[r]]:.6f} rank {rank} |x|^2 {float((z[r]**2).sum()):.3f} "
              f"gpu%32 {int(gi[r]) % 32} ref%32 {int(idx_ref[r]) % 32}")
