"""Codebook source at M = 1,024 on the arxiv GAT batch:
times, interleaved in one process, (a) gather_codewords + the two-source task
SpMM, (b) the codebook-source SpMM (narrow column tiles: 8 lanes per task at
M = 1,024), (c) the fused GAT aggregation with gathered rows (alpha +
coefficients + SpMM + normalise), all on the same batch and codebook.  (b)
vs (a) bounds what a codebook-source GAT walker could gain: its per-edge
coefficient work would repeat per column tile like (b)'s walk does.
Usage: python scripts/cb_m1024_probe.py [reps] [config]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd.convs_gat import OurGATConv  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402
from vq_gnn_amd.vq import VQBank  # noqa: E402

dev = torch.device("cuda:0")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "arxiv_gat"]
F, M, D = cfg["F"], cfg["M"], 4
nb = F // D
g, _, b = make_batch(cfg)
bidx, subset, adj = batch_to_device(b, dev)
gen = torch.Generator().manual_seed(5)
X = torch.randn(b.B, F, generator=gen).to(dev)
codes = torch.randint(0, M, (g.N, nb), dtype=torch.int16, generator=gen).to(dev)
torch.manual_seed(6)
bank = VQBank(nb, M, D, warm_up_flag=True)
for i in range(nb):
    bank.init_branch(i)
bank = bank.to(dev)
assert kernels.codebook_source_ok(X, F, M, D, codes=codes, n_rows=b.n, n_branches=nb)
print("cb lds bytes", kernels.lib().vqgnn_spmm_task_cb_lds(M))
plan = adj.plan(F, B=b.B)
plan_cb = adj.plan_codebook(b.B, subset, g.N)
torch.manual_seed(4)
gat = OurGATConv(F + 1, F + 1, bias=False, add_self_loops=False).to(dev)


def two_source():
    xt, _ = kernels.gather_codewords(subset, b.B, codes, bank.emb_out, D)
    return kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=xt, B=b.B, plan=plan)


def cb():
    return kernels.spmm_codebook(adj.rowptr, b.n, b.nnz, X, F, b.B, codes, bank.emb_out, D, plan_cb)


def gat_agg():
    xt, _ = kernels.gather_codewords(subset, b.B, codes, bank.emb_out, D)
    with torch.no_grad():
        return gat.fused_forward(X, adj, xt, b.B)


ref = two_source()
out = cb()
torch.cuda.synchronize()
print("cb == gather + two-source:", bool(torch.equal(ref, out)))
forms = {"gather+two_source": two_source, "codebook_source": cb, "gat_gathered": gat_agg}
for f in forms.values():
    for _ in range(3):
        f()
torch.cuda.synchronize()
times = {k: [] for k in forms}
for r in range(reps):
    for k, f in forms.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) * 1e3)
for k, t in times.items():
    t = sorted(t)
    print(f"{k:20s} median {t[len(t) // 2]:8.1f} us  min {t[0]:8.1f}  max {t[-1]:8.1f}")
