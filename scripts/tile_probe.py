"""Time the tiled SpMM pieces on the reddit batch (VQGNN_TILE_DBG variants)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vqgnn_pkg
vqgnn_pkg.load()
from vq_gnn_amd import kernels
from vq_gnn_amd._lib import lib
from vq_gnn_amd.graph import CONFIGS, make_batch_device

DEV = torch.device("cuda:0")
F = int(sys.argv[1]) if len(sys.argv) > 1 else 604
graph, (bidx, subset, adj) = make_batch_device(CONFIGS["reddit_gcn_l1"], device=DEV)
B, n = bidx.numel(), subset.numel()
X = torch.randn(B, F, device=DEV)
X2 = torch.randn(n - B, F, device=DEV)
plan = adj.plan(F, B=B)
print("plan", type(plan).__name__, "dense blocks", plan.n_dense, "dense edges", plan.dense_edges,
      "sparse", plan.s_nnz, "records", int(plan.boff[-1]), flush=True)
out = torch.empty(n, F, device=DEV)
L = lib()


def tile():
    L.vqgnn_spmm_tile(n, n, B, X.data_ptr(), F, X2.data_ptr(), F, F, out.data_ptr(), F,
                      plan.blocks.data_ptr(), plan.n_dense, plan.rowptr_b.data_ptr(),
                      plan.boff.data_ptr(), plan.drec.data_ptr(), torch.cuda.current_stream().cuda_stream)


for dbg in ("0", "1", "2", "3"):
    os.environ["VQGNN_TILE_DBG"] = dbg
    tile()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        tile()
    e1.record()
    torch.cuda.synchronize()
    print(f"F={F} dbg={dbg}: {e0.elapsed_time(e1) / 3:.3f} ms", flush=True)
