"""Time the codebook-source aggregation (spmm_codebook: walk + fix-up) of a
config's bench batch with the library VQGNN_LIB selects (A/B of library
builds).  Usage: python scripts/cb_time.py [config] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402

dev = torch.device("cuda:0")
name = sys.argv[1] if len(sys.argv) > 1 else "arxiv_gcn"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
cfg = dict(CONFIGS[name])
F, M, D = cfg["F"], cfg["M"], 4
nb = F // D
g, _, b = make_batch(cfg)
bidx, subset, adj = batch_to_device(b, dev)
B, n, nnz, N = b.B, b.n, b.nnz, cfg["N"]
gen = torch.Generator(device="cpu").manual_seed(3)
X = torch.randn(B, F, generator=gen).to(dev)
codes = torch.randint(0, M, (N, nb), dtype=torch.int16, generator=gen).to(dev)
emb_out = torch.randn(nb, M, 2 * D, generator=gen).to(dev)
out = torch.empty(n, F, device=dev)
pcb = adj.plan_codebook(B, subset, N)
fn = lambda: kernels.spmm_codebook(adj.rowptr, n, nnz, X, F, B, codes, emb_out, D, pcb,  # noqa
                                   out=out)
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
print(f"{name} cb {os.path.basename(os.environ.get('VQGNN_LIB', 'libvqgnn.so'))}: "
      f"{min(ts):8.1f} us  ({', '.join(f'{t:.1f}' for t in ts)})  checksum {float(out.double().sum()):.6e}",
      flush=True)
