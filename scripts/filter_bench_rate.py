"""Measurement (GPU): share of undecided rows of the filtered assign path on
bench.py's data (random-init codebook after one warm-up feature_update pass,
BN-normalised rows, update semantics) against scripts/filter_debug.py's random
codebook.  Captures the assign workspace to read the per-branch counters."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd._lib import lib  # noqa: E402
from vq_gnn_amd.vq import VQBank  # noqa: E402
import vq_gnn_amd.vq as vqmod  # noqa: E402

vqmod.STRICT_BAD_INIT = False
dev = torch.device("cuda:0")
B, F, M, D = 84670, 128, 256, 4
nb = F // D
X = torch.randn(B, F, generator=torch.Generator().manual_seed(1)).to(dev)
G = (torch.randn(B, F, generator=torch.Generator().manual_seed(2)) * 1e-3).to(dev)
N = 169343
codes = torch.randint(0, M, (N, nb), dtype=torch.int16,
                      generator=torch.Generator().manual_seed(5)).to(dev)
bidx = torch.randperm(N, generator=torch.Generator().manual_seed(6))[:B].to(dev)
torch.manual_seed(0)
bank = VQBank(nb, M, D, warm_up_flag=True)
for b in range(nb):
    bank.init_branch(b)
bank = bank.to(dev)
bank.feature_update(X, 0, nb, True, codes=codes, batch_idx=bidx)

captured = []
orig = kernels.workspace


def grab(nbytes, device):
    t = orig(nbytes, device)
    captured.append(t)
    return t


kernels.workspace = grab
lib().vqgnn_assign_filter(1)
for step in range(3):
    captured.clear()
    bank.update(X, G, 0, nb, True, codes=codes, batch_idx=bidx)
    torch.cuda.synchronize()
    want = max(int(lib().vqgnn_vq_assign_workspace(B, nb, M, 2 * D)), 256)
    ws = [t for t in captured if t.numel() == want]
    assert len(ws) == 1, [t.numel() for t in captured]
    cnt = ws[0][: nb * 4].view(torch.int32).cpu()
    print(f"step {step}: undecided rows {int(cnt.sum())} of {B * nb} "
          f"({int(cnt.sum()) / (B * nb):.2%}), per branch min {int(cnt.min())} max {int(cnt.max())}",
          flush=True)
lib().vqgnn_assign_filter(-1)
