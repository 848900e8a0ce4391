"""Probe (GPU): one arxiv_gcn layer step serial vs with the SpMM on a second
stream beside the VQ update.  Order of the overlapped step: codeword gather
(reads the codebook as of the step start) -> fork -> {update on the main
stream, SpMM on the side stream} -> join.  Usage: python scripts/overlap_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch, synthetic_graph  # noqa: E402
from vq_gnn_amd.vq import VQBank  # noqa: E402
import vq_gnn_amd.vq as vqmod  # noqa: E402

vqmod.STRICT_BAD_INIT = False
dev = torch.device("cuda:0")
cfg = CONFIGS["arxiv_gcn"]
g = synthetic_graph(cfg["N"], cfg["parts"], cfg["edges"], seed=cfg.get("seed", 0))
_, _, batch = make_batch(cfg, rank=0, graph=g)
B, n, nnz = batch.B, batch.n, batch.nnz
F, M, D = cfg["F"], cfg["M"], 4
nb = F // D
X = torch.randn(B, F, device=dev)
G = torch.randn(B, F, device=dev) * 1e-3
codes = torch.randint(0, M, (g.N, nb), dtype=torch.int16, device=dev)
torch.manual_seed(0)
bank = VQBank(nb, M, D, warm_up_flag=True)
for b in range(nb):
    bank.init_branch(b)
bank = bank.to(dev)
bidx, subset, adj = batch_to_device(batch, dev)
plan = adj.plan(F)
bank.feature_update(X, 0, nb, True, codes=codes, batch_idx=bidx)
prio = int(os.environ.get("OV_PRIO", "0"))
side = torch.cuda.Stream(priority=prio)
main = torch.cuda.current_stream()
out_buf = {}


def serial():
    bank.update(X, G, 0, nb, True, codes=codes, batch_idx=bidx)
    xf, _ = kernels.gather_codewords(subset, B, codes, bank.emb_out, D)
    out_buf["o"] = kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, X, F, X2=xf, B=B,
                                plan=plan)


def overlapped():
    xf, _ = kernels.gather_codewords(subset, B, codes, bank.emb_out, D)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out_buf["o"] = kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, X, F, X2=xf, B=B,
                                    plan=plan)
    bank.update(X, G, 0, nb, True, codes=codes, batch_idx=bidx)
    main.wait_stream(side)


def spmm_only():
    kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, X, F, X2=out_buf["xf"], B=B, plan=plan)


def update_only():
    bank.update(X, G, 0, nb, True, codes=codes, batch_idx=bidx)


def timeit(fn, reps=40, warm=5):
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


out_buf["xf"], _ = kernels.gather_codewords(subset, B, codes, bank.emb_out, D)
if os.environ.get("OV_HOST"):
    import time
    for fn in (serial, serial):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(40):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"[host] issue {(t1 - t0) / 40 * 1e6:8.1f} us/step, wall {(t2 - t0) / 40 * 1e6:8.1f} "
              f"us/step", flush=True)
    # the step captured once in a HIP graph, replayed
    torch.cuda.synchronize()
    gs = torch.cuda.Stream()
    gs.wait_stream(main)
    with torch.cuda.stream(gs):
        for _ in range(3):
            serial()
    main.wait_stream(gs)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        serial()
    torch.cuda.synchronize()
    for _ in range(2):
        t0 = time.perf_counter()
        for _ in range(40):
            graph.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"[graph] issue {(t1 - t0) / 40 * 1e6:8.1f} us/step, wall {(t2 - t0) / 40 * 1e6:8.1f} "
              f"us/step", flush=True)
    print(f"[graph] event-timed {timeit(graph.replay):8.1f} us", flush=True)
    sys.exit(0)
tag = os.environ.get("VQGNN_ASG_TARGET", "auto")
for name, fn in [("update only", update_only), ("spmm only", spmm_only), ("serial step", serial),
                 ("overlapped step", overlapped), ("serial step", serial),
                 ("overlapped step", overlapped)]:
    print(f"[target={tag} prio={prio}] {name:16s} {timeit(fn):8.1f} us", flush=True)
