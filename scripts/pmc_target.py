"""Run one hot-path kernel a few times on a bench config's batch (PMC target).
CONFIG=<bench config> (reddit configs build graph and batch on the device);
argv[1]: step | vq | spmm | gat (the fused GAT aggregation of the bench);
GATHER_ROWS=1: the two-source SpMM over gathered rows instead of the
codebook-source SpMM the bench runs for GCN configs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402
from vq_gnn_amd.vq import VQBank  # noqa: E402
import vq_gnn_amd.vq as vqmod  # noqa: E402

vqmod.STRICT_BAD_INIT = False
dev = torch.device("cuda:0")
what = sys.argv[1] if len(sys.argv) > 1 else "step"
reps = int(os.environ.get("REPS", "5"))
cfg = CONFIGS[os.environ.get("CONFIG", "arxiv_gcn")]
if cfg.get("device_build"):
    from types import SimpleNamespace
    from vq_gnn_amd.graph import make_batch_device
    dg, (bidx, subset, adj) = make_batch_device(cfg, device=dev)
    g = SimpleNamespace(N=dg.N)
    b = SimpleNamespace(B=int(bidx.numel()), n=int(subset.numel()), nnz=adj.nnz())
    del dg
else:
    g, _, b = make_batch(cfg)
    bidx, subset, adj = batch_to_device(b, dev)
F, M, D = cfg["F"], cfg["M"], 4
nb = F // D
X = torch.randn(b.B, F, device=dev)
G = torch.randn(b.B, F, device=dev) * 1e-3
codes = torch.randint(0, M, (g.N, nb), dtype=torch.int16, device=dev)
bank = VQBank(nb, M, D, warm_up_flag=True)
for i in range(nb):
    bank.init_branch(i)
bank = bank.to(dev)
bank.feature_update(X, 0, nb, True, codes=codes, batch_idx=bidx)
xt, _ = kernels.gather_codewords(subset, b.B, codes, bank.emb_out, D)
plan = adj.plan(F, B=b.B)
# the bench's aggregation: out-of-batch rows from the codebook where it applies
use_cb = (what != "gat" and os.environ.get("GATHER_ROWS", "0") == "0" and
          kernels.codebook_source_ok(X, F, M, D))
plan_cb = adj.plan_codebook(b.B, subset, g.N) if use_cb else None
gat = None
if what == "gat":
    from vq_gnn_amd.convs_gat import OurGATConv
    torch.manual_seed(4)
    gat = OurGATConv(F + 1, F + 1, bias=False, add_self_loops=False).to(dev)
torch.cuda.synchronize()
for _ in range(reps):
    if gat is not None:
        with torch.no_grad():
            gat.fused_forward(X, adj, xt, b.B)
    if what in ("vq", "step"):
        bank.update(X, G, 0, nb, True, codes=codes, batch_idx=bidx)
    if what in ("spmm", "step") and use_cb:
        kernels.spmm_codebook(adj.rowptr, b.n, b.nnz, X, F, b.B, codes, bank.emb_out, D, plan_cb)
    elif what in ("spmm", "step"):
        xt, _ = kernels.gather_codewords(subset, b.B, codes, bank.emb_out, D)
        kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=xt, B=b.B, plan=plan)
torch.cuda.synchronize()
print("done", what, "B", b.B, "n", b.n, "nnz", b.nnz)
