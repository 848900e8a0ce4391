"""Codebook-source SpMM probe (a library variant with vqgnn_spmm_task_cb,
selected by VQGNN_LIB): on the arxiv bench batch, the out-of-batch rows read
their codewords from an LDS image of the codebook instead of a gathered
x_first row.  Checks the output against gather_codewords + the two-source
task SpMM (same fma chain: bit-identical expected) and times both.
Usage: VQGNN_LIB=... python scripts/spmm_cb_probe.py [reps] [config] [entry]
(entry: vqgnn_spmm_task_cb, or a variant's entry with the same arguments)"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import kernels  # noqa: E402
from vq_gnn_amd._lib import lib  # noqa: E402
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402

dev = torch.device("cuda:0")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
name = sys.argv[2] if len(sys.argv) > 2 else "arxiv_gcn"
entry = sys.argv[3] if len(sys.argv) > 3 else "vqgnn_spmm_task_cb"
cfg = dict(CONFIGS[name])
F, M, D = cfg["F"], cfg["M"], 4
nb = F // D
if cfg.get("device_build"):
    from vq_gnn_amd.graph import make_batch_device
    dg, (bidx, subset, adj) = make_batch_device(cfg, device=dev)
    N = dg.N
    del dg
    B, n, nnz = int(bidx.numel()), int(subset.numel()), adj.nnz()
else:
    g, _, b = make_batch(cfg)
    bidx, subset, adj = batch_to_device(b, dev)
    B, n, nnz = b.B, b.n, b.nnz
    N = cfg["N"]
gen = torch.Generator(device="cpu").manual_seed(3)
X = torch.randn(B, F, generator=gen).to(dev)
codes = torch.randint(0, M, (N, nb), dtype=torch.int16, generator=gen).to(dev)
emb_out = torch.randn(nb, M, 2 * D, generator=gen).to(dev)
out_ref = torch.empty(n, F, device=dev)
out_cb = torch.empty(n, F, device=dev)
plan = adj.plan(F, B=B)

L = lib()
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
L.vqgnn_spmm_task_records_cb.restype = ctypes.c_int
L.vqgnn_spmm_task_records_cb.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                         ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                         ctypes.c_void_p]
fcb = getattr(L, entry)
fcb.restype = ctypes.c_int
fcb.argtypes = ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                  ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                  ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                  ctypes.c_void_p])
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
rec_cb = plan.records.clone()
rc = L.vqgnn_spmm_task_records_cb(p(rec_cb), nnz, B, p(subset), n, N, stream)
assert rc == 0, L.vqgnn_last_error()
ws = torch.empty(L.vqgnn_spmm_task_workspace(nnz, plan.K, F) // 4 + 64, device=dev)


def ref():
    xf, _ = kernels.gather_codewords(subset, B, codes, emb_out, D)
    kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, X, F, X2=xf, B=B, out=out_ref,
                 plan=plan)


def cb():
    rc = fcb(p(adj.rowptr), n, nnz, B, p(X), F, F, p(codes), nb, N,
                              p(emb_out), emb_out.stride(1), emb_out.stride(0), nb, M, D,
                              p(out_cb), F, p(plan.plan), p(rec_cb), plan.K, plan.n_jobs,
                              plan.n_empty, p(ws), stream)
    assert rc == 0, L.vqgnn_last_error()


ref()
cb()
torch.cuda.synchronize()
diff = (out_ref - out_cb).abs().max().item()
same = torch.equal(out_ref, out_cb)
print(f"cb vs gather+task: bit-identical {same}, max |diff| {diff:.3e}", flush=True)


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


u = os.environ.get("VQGNN_TASK_CB_U", "8")
tag = entry.replace("vqgnn_spmm_task_", "")
for nm, fn in (("gather+task", ref), (f"{tag} U={u}", cb), ("gather+task", ref), (f"{tag} U={u}", cb)):
    t, ts = timeit(fn)
    print(f"{name} {nm:12s} {t:8.1f} us ({', '.join(f'{x:.1f}' for x in ts)})", flush=True)
