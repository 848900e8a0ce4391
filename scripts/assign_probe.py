"""Time vq_assign_kernel pieces on the arxiv batch shapes (B = 84,670,
nb = 32, M = 256, W = 8): with / without the code scatter and the fused EMA
statistics.  VQGNN_ASSIGN_MSWEEP (set before start) shortens the sweep;
M=<codewords> (default 256; arxiv_gat: 1024)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vqgnn_pkg
vqgnn_pkg.load()
from vq_gnn_amd import kernels

DEV = torch.device("cuda:0")
B, nb, D = 84670, 32, 4
M = int(os.environ.get("M", "256"))
F = nb * D
W = int(os.environ.get("W", "8"))
torch.manual_seed(0)
X = torch.randn(B, F, device=DEV)
G = torch.randn(B, F, device=DEV) * 1e-3
emb = torch.randn(nb, M, 2 * D, device=DEV)
rm = torch.zeros(F, device=DEV)
rv = torch.ones(F, device=DEV)
coef, _, _ = kernels.bn_stats_finalize(X, G if W == 8 else None, F, kernels.BN_TRAIN, 0.1, 1e-5,
                                       0.1, 1e-24, 1e-24, rm, rv, rm.clone(), rv.clone())
codes = torch.zeros(200000, nb, dtype=torch.int16, device=DEV)
bidx = torch.randperm(200000, device=DEV)[:B]
slab = torch.zeros(1, nb, M, W + 1, dtype=torch.int64, device=DEV)
Gx = G if W == 8 else None


def run(want_codes, want_stats):
    if want_stats:
        slab.zero_()
    kernels.vq_assign(X, Gx, coef, 1.0, emb, D, W, codes=codes if want_codes else None,
                      batch_idx=bidx if want_codes else None, want_stats=want_stats,
                      stat_count=B, stats_out=slab if want_stats else None)


for wc, ws in ((True, True), (False, True), (True, False), (False, False)):
    run(wc, ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run(wc, ws)
    e1.record()
    torch.cuda.synchronize()
    print(f"M={M} W={W} msweep={os.environ.get('VQGNN_ASSIGN_MSWEEP', 'all')} codes={wc} stats={ws}: "
          f"{e0.elapsed_time(e1) / 10 * 1e3:.1f} us (stats: + a slab memset)", flush=True)
