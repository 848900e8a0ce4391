"""Near-tie statistics of the filtered assign on the bench configurations:
the fraction of (row, branch) pairs whose top-2 distance gap lies within the
filter's bound Delta, duplicate codewords, max |e|^2."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vqgnn_pkg
vqgnn_pkg.load()
from vq_gnn_amd.vq import VQBank
from vq_gnn_amd.graph import CONFIGS
dev = torch.device("cuda:0")
for name in sys.argv[1:] or ["arxiv_gcn", "arxiv_gat"]:
    cfg = CONFIGS[name]
    F, M, D = cfg["F"], cfg["M"], 4
    nb = F // D
    B = 20000
    X = torch.randn(B, F, generator=torch.Generator().manual_seed(1))
    torch.manual_seed(0)
    bank = VQBank(nb, M, D, warm_up_flag=True)
    for b in range(nb):
        bank.init_branch(b)
    bank = bank.to(dev)
    codes = torch.zeros(B, nb, dtype=torch.int16, device=dev)
    bidx = torch.arange(B, device=dev)
    bank.feature_update(X.to(dev), 0, nb, True, codes=codes, batch_idx=bidx)
    torch.cuda.synchronize()
    emb = bank.emb.double().cpu()
    x = X.double()
    z = (x - x.mean(0)) / torch.sqrt(x.var(0, unbiased=False) + 1e-5)
    tot = near = 0
    dup = 0
    semax = 0.0
    for b in range(min(nb, 8)):
        e = emb[b][:, :D]
        zb = z[:, b * D:(b + 1) * D]
        se = (e * e).sum(1)
        semax = max(semax, float(se.max()))
        dup += int(M - torch.unique(e, dim=0).shape[0])
        sx = (zb * zb).sum(1)
        d = sx[:, None] + se[None] - 2 * zb @ e.T
        top2 = torch.topk(d, 2, largest=False).values
        gap = top2[:, 1] - top2[:, 0]
        tmin = top2[:, 0] - sx
        delta = (978 * sx + 390 * tmin.abs() + 489) * 2.0 ** -24
        near += int((gap <= delta).sum())
        tot += B
        if b == 0:
            print(name, "gap quantiles", [f"{float(v):.2e}" for v in torch.quantile(gap, torch.tensor([0.001, 0.01, 0.1, 0.5], dtype=torch.float64))],
                  "delta median", f"{float(delta.median()):.2e}")
    print(name, f"M={M} near-tie fraction {near / tot:.4%} duplicates {dup} max|e|^2 {semax:.1f}")
