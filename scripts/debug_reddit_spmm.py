"""Debug: per-row SpMM error on the reddit batch (task kernel vs chunk kernel vs fp64)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vqgnn_pkg
vqgnn_pkg.load()
from vq_gnn_amd import kernels
from vq_gnn_amd.graph import CONFIGS, make_batch_device

DEV = torch.device("cuda:0")
cfg = dict(CONFIGS["reddit_gcn"])
if len(sys.argv) > 1:
    cfg["edges"] = int(sys.argv[1])
graph, (bidx, subset, adj) = make_batch_device(cfg, device=DEV)
B, n = bidx.numel(), subset.numel()
F = 128
X = torch.randn(B, F, device=DEV)
x_first = torch.randn(n - B, F, device=DEV)
rp, cl, vl = adj.rowptr, adj.col, adj.value
print("B", B, "n", n, "nnz", adj.nnz(), "rp dtype", rp.dtype, cl.dtype, flush=True)
plan = adj.plan(F, B=B)
print("plan", type(plan).__name__, getattr(plan, "K", None), plan.n_jobs, plan.n_empty, flush=True)
out = kernels.spmm(rp, cl, vl, n, adj.nnz(), X, F, X2=x_first, B=B, plan=plan)
cplan = adj.plan(F, B=B, kind="chunk")
out_c = kernels.spmm(rp, cl, vl, n, adj.nnz(), X, F, X2=x_first, B=B, plan=cplan)
torch.cuda.synchronize()
xin = torch.cat([X, x_first])
lens = (rp[1:] - rp[:-1]).long()
rows = torch.randint(0, n, (256,), device=DEV)
bad = []
for r in rows.tolist():
    s, e = int(rp[r]), int(rp[r + 1])
    ref = (vl[s:e].double()[:, None] * xin[cl[s:e].long()].double()).sum(0)
    mag = (vl[s:e].double()[:, None] * xin[cl[s:e].long()].double()).abs().sum(0)
    et = ((out[r].double() - ref).abs() / (mag + 1e-30)).max().item()
    ec = ((out_c[r].double() - ref).abs() / (mag + 1e-30)).max().item()
    if et > 1e-5 or ec > 1e-5:
        bad.append((r, s, e, e - s, et, ec))
print("bad rows", len(bad), "of", rows.numel())
K = plan.K
for b in bad[:20]:
    r, s, e, l, et, ec = b
    print(f"row {r} edges [{s},{e}) len {l} tasks {s // K}..{(e - 1) // K} err task {et:.2e} chunk {ec:.2e}")
print("col max", int(cl.max()), "n", n)
