"""SpMM kernel comparison on the bench batches (GPU): the task-split kernel
(include/vqgnn.h §6) at several K / G / U settings, with the algorithmic-byte
roofline fraction of SURVEY §8(d), and bound probes (same plan shape,
columns rewritten).
Usage: python scripts/bench_spmm.py [arxiv_gcn|reddit_gcn|ppi_sage ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def run(name, F=None):
    cfg = dict(CONFIGS[name])
    g, _, b = make_batch(cfg)
    F = F or cfg["F"]
    bidx, subset, adj = batch_to_device(b, dev)
    X = torch.randn(b.B, F, device=dev)
    X2 = torch.randn(b.n - b.B, F, device=dev)
    out = torch.empty(b.n, F, device=dev)
    alg = 4 * (b.n + 1) + 8 * b.nnz + 8 * b.n * F
    deg = np.diff(b.rowptr)
    print(f"{name}: F={F} B={b.B} n={b.n} nnz={b.nnz} mean deg {deg.mean():.1f} "
          f"max {deg.max()}  alg bytes {alg / 1e6:.1f} MB", flush=True)

    def line(tag, t):
        print(f"  {tag:28s} {t:9.1f} us  {alg / t / 1e3:7.1f} GB/s alg  frac {alg / t / 8e6:.3f}"
              f"  {b.nnz * 4 * F / t / 1e6:6.2f} TB/s gathered", flush=True)

    plans = {K: kernels.spmm_task_plan(adj.rowptr, adj.col, adj.value, b.n, b.nnz, K)
             for K in (32, 64, 128)}
    os.environ["VQGNN_TASK_SNAP"] = "0"     # fixed K-edge tasks (rows cut anywhere)
    plans.update({-K: kernels.spmm_task_plan(adj.rowptr, adj.col, adj.value, b.n, b.nnz, K)
                  for K in (64, 128)})
    del os.environ["VQGNN_TASK_SNAP"]
    variants = [
        (f"task K={K} G={G} U={U}" + (" fixed" if K < 0 else ""), K, G, U)
        for (K, G, U) in ((64, 32, 8), (-64, 32, 8), (64, 32, 4), (64, 32, 16), (128, 32, 8),
                          (128, 32, 16), (32, 32, 8), (64, 16, 8), (64, 16, 16))]
    res = {v[0]: [] for v in variants}
    for rep in range(3):              # interleaved repeats: box drift hits every variant alike
        for tag, K, G, U in variants:
            os.environ["VQGNN_TASK_U"], os.environ["VQGNN_TASK_G"] = str(U), str(G)
            pl = plans[K]
            fn = lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F,  # noqa
                                      X2=X2, B=b.B, out=out, plan=pl)
            res[tag].append(timeit(fn))
    for tag, ts in res.items():
        line(tag + " (min of 3)", min(ts))
    os.environ.pop("VQGNN_TASK_U", None)
    os.environ.pop("VQGNN_TASK_G", None)
    tp = timeit(lambda: kernels.spmm_task_plan(adj.rowptr, adj.col, adj.value, b.n, b.nnz, 64))
    print(f"  task plan build            {tp:9.1f} us", flush=True)
    # bound probes: same CSR shape and task split, columns rewritten
    Xn = torch.randn(b.n, F, device=dev)
    rows = torch.repeat_interleave(torch.arange(b.n, device=dev),
                                   torch.from_numpy(deg).to(dev))
    ar = torch.arange(b.nnz, device=dev)
    for tag, colv in (("hot set 1024 rows (L2)", ar % 1024),
                      ("hot set 64 rows (L1)", ar % 64),
                      ("col = row (stream)", rows),
                      ("uniform random", torch.randint(0, b.n, (b.nnz,), device=dev))):
        c32 = colv.to(torch.int32).contiguous()
        pl = kernels.spmm_task_plan(adj.rowptr, c32, adj.value, b.n, b.nnz, 64)
        t = timeit(lambda: kernels.spmm(adj.rowptr, c32, adj.value, b.n, b.nnz, Xn, F,
                                        out=out, plan=pl))
        line("probe " + tag, t)


if __name__ == "__main__":
    for n in (sys.argv[1:] or ["arxiv_gcn"]):
        run(n)
