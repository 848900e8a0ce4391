"""Kernel-level microbenchmarks (GPU): isolate the costs inside the VQ assign
and SpMM kernels.  Usage: python scripts/microbench.py [vq|spmm|all]"""
import os
import sys
import time

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


def bench_vq(B=84670, nb=32, M=256, D=4):
    F = nb * D
    X = torch.randn(B, F, device=dev)
    G = torch.randn(B, F, device=dev) * 1e-3
    emb = torch.randn(nb, M, 2 * D, device=dev)
    coef = torch.zeros(6, F, device=dev)
    coef[0] = 1.0
    coef[2] = 1.0
    N = 169343
    codes = torch.zeros(N, nb, dtype=torch.int16, device=dev)
    bidx = torch.randperm(N, device=dev)[:B]
    bidx_sorted = torch.arange(B, device=dev)
    flops = 2.0 * B * M * 2 * D * nb
    for name, kw in [
        ("assign only W=8", dict()),
        ("+ EMA", dict(want_stats=True)),
        ("+ codes(random rows)", dict(codes=codes, batch_idx=bidx)),
        ("+ codes(contig rows)", dict(codes=codes, batch_idx=bidx_sorted)),
        ("+ EMA + codes(contig)", dict(want_stats=True, codes=codes, batch_idx=bidx_sorted)),
    ]:
        t = timeit(lambda: kernels.vq_assign(X, G, coef, 1.0, emb, D, 2 * D, **kw))
        print(f"vq_assign {name:28s} {t:8.1f} us  {flops / t / 1e6:6.1f} TFLOP/s", flush=True)
    t = timeit(lambda: kernels.vq_assign(X, None, coef, 1.0, emb, D, D))
    print(f"vq_assign W=4 assign only          {t:8.1f} us  {flops / 2 / t / 1e6:6.1f} TFLOP/s")
    t = timeit(lambda: kernels.bn_stats(X, G, F))
    print(f"bn_stats X+G                       {t:8.1f} us  {2 * X.numel() * 4 / t / 1e3:6.1f} GB/s")


def bench_spmm():
    cfg = CONFIGS["arxiv_gcn"]
    g, _, b = make_batch(cfg)
    bidx, subset, adj = batch_to_device(b, dev)
    F, D, M = 128, 4, 256
    nb = F // D
    X = torch.randn(b.B, F, device=dev)
    Xn = torch.randn(b.n, F, device=dev)
    emb_out = torch.randn(nb, M, 2 * D, device=dev)
    codes = torch.randint(0, M, (g.N, nb), dtype=torch.int16, device=dev)
    xt, _ = kernels.gather_codewords(subset, b.B, codes, emb_out, D)
    by = 4 * (b.n + 1) + 8 * b.nnz + 8 * b.n * F
    deg = np.diff(b.rowptr)
    print(f"batch B={b.B} n={b.n} nnz={b.nnz} maxdeg={deg.max()} rows>128: {(deg > 128).sum()}")
    pl = adj.plan(F) if os.environ.get("MB_PLAN", "1") == "1" else None
    t = timeit(lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=xt,
                                    B=b.B, plan=pl))
    print(f"spmm two-source     {t:8.1f} us  {by / t / 1e3:7.1f} GB/s alg  "
          f"{b.nnz * 512 / t / 1e6:6.2f} TB/s gathered")
    t = timeit(lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, Xn, F, plan=pl))
    print(f"spmm dense n rows   {t:8.1f} us  {b.nnz * 512 / t / 1e6:6.2f} TB/s gathered")
    t = timeit(lambda: kernels.gather_codewords(subset, b.B, codes, emb_out, D))
    print(f"gather_codewords    {t:8.1f} us  {(b.n - b.B) * F * 4 / t / 1e3:7.1f} GB/s written")
    # bound probes: same CSR shape, columns rewritten
    rows = torch.repeat_interleave(torch.arange(b.n, device=dev),
                                   torch.from_numpy(deg).to(dev))
    for name, colv in (("hot set (1024 rows)", (torch.arange(b.nnz, device=dev) % 1024)),
                       ("col = row (stream)", rows),
                       ("col = row+k (local)", (rows + torch.arange(b.nnz, device=dev) % 16)
                        .clamp(max=b.n - 1))):
        c32 = colv.to(torch.int32).contiguous()
        t = timeit(lambda: kernels.spmm(adj.rowptr, c32, adj.value, b.n, b.nnz, Xn, F, plan=pl))
        print(f"probe {name:22s} {t:8.1f} us  {b.nnz * 512 / t / 1e6:6.2f} TB/s gathered")


def bench_codes():
    """Code-source SpMM against the two-source SpMM, plus structure probes:
    all-X (B = n) isolates the persistent/occupancy structure, all-codes
    (B = 0) the LDS codeword path."""
    cfg = CONFIGS["arxiv_gcn"]
    g, _, b = make_batch(cfg)
    bidx, subset, adj = batch_to_device(b, dev)
    F, D, M = 128, 4, 256
    nb = F // D
    X = torch.randn(b.B, F, device=dev)
    Xn = torch.randn(b.n, F, device=dev)
    emb_out = torch.randn(nb, M, 2 * D, device=dev)
    codes = torch.randint(0, M, (g.N, nb), dtype=torch.int16, device=dev)
    xt, lc = kernels.gather_codewords(subset, b.B, codes, emb_out, D, want_codes=True)
    lc_all = torch.randint(0, M, (b.n, nb), dtype=torch.int16, device=dev)
    pl = adj.plan(F)
    res = {}
    res["rows two-source"] = timeit(lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n,
                                                         b.nnz, X, F, X2=xt, B=b.B, plan=pl))
    res["rows all-X"] = timeit(lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz,
                                                    Xn, F, plan=pl))
    res["codes fused"] = timeit(lambda: kernels.spmm_codes(adj.rowptr, adj.col, adj.value, b.n,
                                                           b.nnz, X, F, lc, emb_out, D, b.B,
                                                           plan=pl))
    res["codes all-X (B=n)"] = timeit(lambda: kernels.spmm_codes(
        adj.rowptr, adj.col, adj.value, b.n, b.nnz, Xn, F, lc[:0], emb_out, D, b.n, plan=pl))
    res["codes all-codes (B=0)"] = timeit(lambda: kernels.spmm_codes(
        adj.rowptr, adj.col, adj.value, b.n, b.nnz, X[:0], F, lc_all, emb_out, D, 0, plan=pl))
    for k, v in res.items():
        print(f"{k:24s} {v:8.1f} us", flush=True)
    # parity of the variants against the two-source result (bit-identical)
    ref = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=xt, B=b.B, plan=pl)
    fz = kernels.spmm_codes(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, lc, emb_out, D,
                            b.B, plan=pl)
    print("codes == two-source:", bool(torch.equal(ref, fz)), flush=True)


def bench_pair():
    """Segment-pair SpMM (dwordx4, two segments per wave) against the chunk
    wave kernel: time, plan build time, and bit-identity of the outputs."""
    cfg = CONFIGS["arxiv_gcn"]
    g, _, b = make_batch(cfg)
    bidx, subset, adj = batch_to_device(b, dev)
    F = 128
    X = torch.randn(b.B, F, device=dev)
    xt = torch.randn(b.n - b.B, F, device=dev)
    Xn = torch.randn(b.n, F, device=dev)
    pl = adj.plan(F)
    tp = timeit(lambda: kernels.spmm_pair_plan(adj.rowptr, b.n, b.nnz, F, b.B), reps=5, warm=1)
    pp = kernels.spmm_pair_plan(adj.rowptr, b.n, b.nnz, F, b.B)
    hdr = pp.buf[:16].cpu().tolist()
    print(f"pair plan: {tp:8.1f} us  segs={hdr[0]} long={hdr[1]} xcd_begin={hdr[2:11]}", flush=True)
    res = {}
    res["wave two-source"] = timeit(lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n,
                                                         b.nnz, X, F, X2=xt, B=b.B, plan=pl))
    res["pair two-source"] = timeit(lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n,
                                                         b.nnz, X, F, X2=xt, B=b.B, plan=pp))
    res["wave all-X"] = timeit(lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz,
                                                    Xn, F, plan=pl))
    res["pair all-X"] = timeit(lambda: kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz,
                                                    Xn, F, plan=pp))
    deg = np.diff(b.rowptr)
    rows = torch.repeat_interleave(torch.arange(b.n, device=dev), torch.from_numpy(deg).to(dev))
    hot = (torch.arange(b.nnz, device=dev) % 1024).to(torch.int32)
    res["wave hot set"] = timeit(lambda: kernels.spmm(adj.rowptr, hot, adj.value, b.n, b.nnz, Xn,
                                                      F, plan=pl))
    res["pair hot set"] = timeit(lambda: kernels.spmm(adj.rowptr, hot, adj.value, b.n, b.nnz, Xn,
                                                      F, plan=pp))
    for k, v in res.items():
        print(f"{k:24s} {v:8.1f} us  {b.nnz * 512 / v / 1e6:6.2f} TB/s gathered", flush=True)
    ref = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=xt, B=b.B, plan=pl)
    got = kernels.spmm(adj.rowptr, adj.col, adj.value, b.n, b.nnz, X, F, X2=xt, B=b.B, plan=pp)
    print("pair == wave:", bool(torch.equal(ref, got)),
          "max|d| =", float((ref - got).abs().max()), flush=True)
    del rows


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("vq", "all"):
        bench_vq()
    if what == "codes":
        bench_codes()
    if what == "pair":
        bench_pair()
    if what in ("spmm", "all"):
        for s_ in os.environ.get("SPMM_S_LIST", "").split(","):
            pass
        bench_spmm()
