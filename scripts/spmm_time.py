"""Time the default SpMM (task kernel + fix-up) of a config's bench batch
with the library VQGNN_LIB selects (A/B of library builds: scripts/ab_spmm.sh).
Usage: python scripts/spmm_time.py [config] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch, make_batch_device  # noqa: E402

dev = torch.device("cuda:0")
name = sys.argv[1] if len(sys.argv) > 1 else "arxiv_gcn"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
cfg = dict(CONFIGS[name])
F = cfg["F"]
if cfg.get("device_build"):
    _, (bidx, subset, adj) = make_batch_device(cfg, device=dev)
    B, n, nnz = int(bidx.numel()), int(subset.numel()), adj.nnz()
else:
    g, _, b = make_batch(cfg)
    bidx, subset, adj = batch_to_device(b, dev)
    B, n, nnz = b.B, b.n, b.nnz
X = torch.randn(B, F, device=dev)
X2 = torch.randn(n - B, F, device=dev)
out = torch.empty(n, F, device=dev)
plan = adj.plan(F, B=B)
fn = lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, X, F,  # noqa: E731
                          X2=X2, B=B, out=out, plan=plan)
for _ in range(3):
    fn()
torch.cuda.synchronize()
ts = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / reps * 1e3)
alg = 4 * (n + 1) + 8 * nnz + 8 * n * F
print(f"{name} {os.path.basename(os.environ.get('VQGNN_LIB', 'libvqgnn.so'))}: "
      f"{min(ts):8.1f} us  frac {alg / min(ts) / 8e6:.3f}  ({', '.join(f'{t:.1f}' for t in ts)})"
      f"  checksum {float(out.double().sum()):.6e}",
      flush=True)
