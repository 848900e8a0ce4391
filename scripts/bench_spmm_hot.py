"""Hot-column tile SpMM (include/vqgnn.h §6h) against the task kernel (§6) on
the bench batches, interleaved repeats on one box: µs per product, the
algorithmic-byte roofline fraction of SURVEY §8(d), the plan's hot coverage
(edges read from LDS) and the plan build time, over a few (Et, C) settings.
Usage: python scripts/bench_spmm_hot.py [arxiv_gcn|reddit_gcn|...] (reddit
configs build the graph on the device)."""
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


def coverage(plan):
    rec = plan.records[:plan.nnz].cpu().numpy()
    return float(((rec & 0xFFFFFFFF) >> 25 & 1).mean())


def run(name, settings, dbgs=()):
    cfg = dict(CONFIGS[name])
    if cfg.get("device_build"):
        from vq_gnn_amd.graph import make_batch_device
        _, (bidx, subset, adj) = make_batch_device(cfg, device=dev)
        B, n, nnz = int(bidx.numel()), int(subset.numel()), adj.nnz()
    else:
        _, _, b = make_batch(cfg)
        bidx, subset, adj = batch_to_device(b, dev)
        B, n, nnz = b.B, b.n, b.nnz
    F = cfg["F"]
    X = torch.randn(B, F, device=dev)
    X2 = torch.randn(n - B, F, device=dev)
    out = torch.empty(n, F, device=dev)
    alg = 4 * (n + 1) + 8 * nnz + 8 * n * F
    print(f"{name}: F={F} B={B} n={n} nnz={nnz} alg bytes {alg / 1e6:.1f} MB", flush=True)
    plans = {"task": kernels.spmm_task_plan(adj.rowptr, adj.col, adj.value, n, nnz)}
    for Et, C in settings:
        plans[f"hot Et={Et} C={C}"] = kernels.spmm_hot_plan(adj.rowptr, adj.col, adj.value, n,
                                                            nnz, n_cols=n, Et=Et, C=C)
    # VQGNN_HOT_DBG experiments on the first hot plan (results invalid but 4)
    variants = [(k, pl, "0") for k, pl in plans.items()]
    first = next(k for k in plans if k != "task")
    variants += [(f"{first} dbg={d}", plans[first], d) for d in dbgs]
    res = {v[0]: [] for v in variants}
    for _ in range(3):
        for k, pl, d in variants:
            os.environ["VQGNN_HOT_DBG"] = d
            res[k].append(timeit(lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, X,
                                                      F, X2=X2, B=B, out=out, plan=pl)))
    os.environ["VQGNN_HOT_DBG"] = "0"
    ref = kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, X, F, X2=X2, B=B,
                       plan=plans["task"])
    for k, ts in res.items():
        t = min(ts)
        extra = ""
        if k in plans and k != "task":
            got = kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, X, F, X2=X2, B=B,
                               plan=plans[k])
            d = (got - ref).abs().max().item()
            tb = timeit(lambda: kernels.spmm_hot_plan(adj.rowptr, adj.col, adj.value, n, nnz,
                                                      n_cols=n, Et=plans[k].Et, C=plans[k].C),
                        reps=3, warm=1)
            extra = f"  hot edges {coverage(plans[k]):.3f}  plan {tb:7.1f} us  max|hot-task| {d:.2e}"
        print(f"  {k:24s} {t:9.1f} us (min of 3: {', '.join(f'{x:.1f}' for x in ts)})  "
              f"{alg / t / 1e3:7.1f} GB/s  frac {alg / t / 8e6:.3f}{extra}", flush=True)


if __name__ == "__main__":
    names = sys.argv[1:] or ["arxiv_gcn"]
    sets = [tuple(int(v) for v in x.split(",")) for x in
            os.environ.get("HOT_SETS", "16384,1024 8192,1024 16384,512 16384,0").split()]
    dbgs = os.environ.get("HOT_DBG", "").split()
    for nm in names:
        run(nm, sets, dbgs)
