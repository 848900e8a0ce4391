"""Probe: how much of the task SpMM's time is its global gathers?  Some steps
of every block read a 512-byte row from LDS instead of a global gather (the
probe library ab_hotprobe.so; results invalid, timing only):
  DBG=2 every other step, DBG=4 three steps in four, +8: the step loads
  nothing at all.  Near (32-bit buffer) and far (64-bit) source paths.
Usage: VQGNN_LIB=vq-gnn_amd/lib/ab_hotprobe.so python scripts/spmm_hot_probe.py [config]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, reps=30, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


name = sys.argv[1] if len(sys.argv) > 1 else "arxiv_gcn"
cfg = dict(CONFIGS[name])
g, _, b = make_batch(cfg)
F = cfg["F"]
bidx, subset, adj = batch_to_device(b, dev)
X = torch.randn(b.B, F, device=dev)
X2 = torch.randn(b.n - b.B, F, device=dev)
out = torch.empty(b.n, F, device=dev)
plan = adj.plan(F, B=b.B)
fn = lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F,  # noqa: E731
                          X2=X2, B=b.B, out=out, plan=plan)
res = {}
for rep in range(3):
    for far in ("0", "1"):
        for dbg in ("0", "2", "4", "10", "12"):
            os.environ["VQGNN_SPMM_FAR"], os.environ["VQGNN_TASK_DBG"] = far, dbg
            res.setdefault((far, dbg), []).append(timeit(fn))
for (far, dbg), ts in res.items():
    print(f"{name} far={far} dbg={dbg:>2}: {min(ts):7.1f} us (min of 3; {', '.join(f'{t:.1f}' for t in ts)})",
          flush=True)
