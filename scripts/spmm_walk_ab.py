"""A/B of the codebook-source SpMM walkers in one process (VQGNN_CB_WALK:
2 = the pipelined walk, 1 = the stream walker, 0 = the round-4 walk) on a
config's bench batch: both checked bit-identical to gather_codewords + the
two-source task SpMM, then timed interleaved (HIP events, min of 3 x reps).
Usage: python scripts/spmm_walk_ab.py [reps] [config]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402

dev = torch.device("cuda:0")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
name = sys.argv[2] if len(sys.argv) > 2 else "arxiv_gcn"
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
plan = adj.plan(F, B=B)
pcb = adj.plan_codebook(B, subset, N)
out = torch.empty(n, F, device=dev)


def ref():
    xf, _ = kernels.gather_codewords(subset, B, codes, emb_out, D)
    return kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, X, F, X2=xf, B=B, plan=plan)


def walk(w):
    os.environ["VQGNN_CB_WALK"] = str(w)
    return kernels.spmm_codebook(adj.rowptr, n, nnz, X, F, B, codes, emb_out, D, pcb, out=out)


r = ref().clone()
for w in (2, 1, 0):
    o = walk(w).clone()
    torch.cuda.synchronize()
    print(f"{name} walk={w}: bit-identical to gather+task {torch.equal(o, r)}, "
          f"max |diff| {(o - r).abs().max().item():.3e}", flush=True)


def timeit(fn):
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
    return min(ts), ts


for rep in range(2):
    for nm, fn in (("pipelined walk", lambda: walk(2)), ("stream walker", lambda: walk(1)),
                   ("round-4 walker", lambda: walk(0)), ("gather+task", ref)):
        t, ts = timeit(fn)
        print(f"{name} {nm:15s} {t:8.1f} us ({', '.join(f'{x:.1f}' for x in ts)})", flush=True)
os.environ["VQGNN_CB_WALK"] = "2"
