"""Time the codeword gather (x_first_order, include/vqgnn.h) on a config's
bench batch with the library VQGNN_LIB selects.  Usage: gather_time.py [config]"""
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
cfg = CONFIGS[name]
g, _, b = make_batch(cfg)
bidx, subset, adj = batch_to_device(b, dev)
nb, M, D = cfg["F"] // 4, cfg["M"], 4
codes = torch.randint(0, M, (g.N, nb), dtype=torch.int16, device=dev)
emb = torch.randn(nb, M, 2 * D, device=dev)
ref, _ = kernels.gather_codewords(subset, b.B, codes, emb, D)
c = codes[subset[b.B:]].long()
want = emb[torch.arange(nb, device=dev)[None, :], c, :D].reshape(b.n - b.B, nb * D)
assert torch.equal(ref, want), "gather mismatch"
fn = lambda: kernels.gather_codewords(subset, b.B, codes, emb, D)  # noqa: E731
for _ in range(3):
    fn()
torch.cuda.synchronize()
ts = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 50 * 1e3)
print(f"{name} gather {os.path.basename(os.environ.get('VQGNN_LIB', 'libvqgnn.so'))}: {min(ts):.1f} us "
      f"(B'={b.n - b.B}, {(b.n - b.B) * nb * D * 4 / 1e6:.1f} MB written)", flush=True)
