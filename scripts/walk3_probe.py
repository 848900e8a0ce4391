"""Round-6 probe: the split-pass codebook-source walk (scripts/probes/walk3.hip)
against the shipped vqgnn_spmm_task_cb on the arxiv bench batch.

The plan is built here in numpy (probe only): tasks of at most R rows and
about K edges (rows cost max(len, K/R); rows longer than K cut into K-edge
chunks summed by a fix-up), each task's edges split into an X stream and a
codebook stream in row order.  Checks the result against the fp64 product
(|got - ref| <= 1e-5 * sum|w x| per element) and times both kernels
interleaved.  Usage: python scripts/walk3_probe.py [--cpu] [reps] [U] [R] [K]
(--cpu: build the plan and check its emulation against fp64, no GPU)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build_plan(rowptr, col, val, B, node_of, ldxb, ldcb, K=64, R=8, align=8, pad=32):
    """-> meta [T,16] u32, xrec [.,2] i32, crec [.,2] i32, jobs [J,3] i32."""
    n = rowptr.shape[0] - 1
    lens = np.diff(rowptr)
    cmin = -(-K // R)
    tasks = []            # (r0, nrows, e_lo of first row, e_hi of last row, head, open)
    r, cur_r0, cur_cost = 0, None, 0
    cut_jobs = []
    for r in range(n):
        L = int(lens[r])
        if L > K:
            if cur_r0 is not None:
                tasks.append((cur_r0, r - cur_r0, None, None, False, False))
                cur_r0, cur_cost = None, 0
            t_first = len(tasks)
            e0 = int(rowptr[r])
            for c0 in range(0, L, K):
                c1 = min(L, c0 + K)
                tasks.append((r, 1, e0 + c0, e0 + c1, c0 > 0, c1 < L))
            cut_jobs.append((r, t_first, len(tasks) - 1))
            continue
        c = max(L, cmin)
        if cur_r0 is not None and cur_cost + c > K:
            tasks.append((cur_r0, r - cur_r0, None, None, False, False))
            cur_r0, cur_cost = None, 0
        if cur_r0 is None:
            cur_r0 = r
        cur_cost += c
    if cur_r0 is not None:
        tasks.append((cur_r0, n - cur_r0, None, None, False, False))
    T = len(tasks)
    meta = np.zeros((T, 16), dtype=np.uint32)
    xrec, crec = [], []
    xlen = clen = 0
    isx = col < B
    for t, (r0, nr, elo, ehi, head, opn) in enumerate(tasks):
        assert nr <= R
        xr, cr = [], []
        xm = cm = 0
        xsl = csl = 0
        kx = kc = 0
        for s in range(nr):
            rr = r0 + s
            a0, a1 = (elo, ehi) if elo is not None else (int(rowptr[rr]), int(rowptr[rr + 1]))
            es = np.arange(a0, a1)
            ex = es[isx[a0:a1]]
            ec = es[~isx[a0:a1]]
            if ex.size:
                for e in ex:
                    xr.append((int(col[e]) * ldxb, val[e]))
                xm |= 1 << (len(xr) - 1)
                xsl |= s << (4 * kx)
                kx += 1
            if ec.size:
                for e in ec:
                    cr.append((int(node_of[col[e]]) * ldcb, val[e]))
                cm |= 1 << (len(cr) - 1)
                csl |= s << (4 * kc)
                kc += 1
        assert len(xr) <= 64 and len(cr) <= 64 and kx <= 8 and kc <= 8
        meta[t, 0], meta[t, 1] = xlen, len(xr)
        meta[t, 2], meta[t, 3] = clen, len(cr)
        meta[t, 4], meta[t, 5] = xm & 0xFFFFFFFF, xm >> 32
        meta[t, 6], meta[t, 7] = cm & 0xFFFFFFFF, cm >> 32
        meta[t, 8], meta[t, 9] = xsl, csl
        meta[t, 10], meta[t, 11] = r0, nr
        meta[t, 12] = (1 if head else 0) | (2 if opn else 0)
        xr += [(0, np.float32(0))] * ((-len(xr)) % align)
        cr += [(0, np.float32(0))] * ((-len(cr)) % align)
        xrec += xr
        crec += cr
        xlen += len(xr)
        clen += len(cr)
    xrec += [(0, np.float32(0))] * pad
    crec += [(0, np.float32(0))] * pad

    def pack(lst):
        a = np.zeros((len(lst), 2), dtype=np.int32)
        a[:, 0] = np.array([p[0] for p in lst], dtype=np.int64).astype(np.int32)
        a[:, 1] = np.array([p[1] for p in lst], dtype=np.float32).view(np.int32)
        return a

    jobs = np.array(cut_jobs, dtype=np.int32).reshape(-1, 3)
    return meta, pack(xrec), pack(crec), jobs, tasks


def emulate(meta, xrec, crec, jobs, X, xf, ldxb, ldcb, n, F):
    """fp32 emulation of the kernel's order (non-fused multiply-add)."""
    out = np.zeros((n, F), dtype=np.float32)
    carry = np.zeros((meta.shape[0], 2, F), dtype=np.float32)
    for t in range(meta.shape[0]):
        xs, nx, cs, nc = (int(v) for v in meta[t, :4])
        xm = int(meta[t, 4]) | (int(meta[t, 5]) << 32)
        cm = int(meta[t, 6]) | (int(meta[t, 7]) << 32)
        xsl, csl, r0, nr, fl = (int(v) for v in meta[t, 8:13])
        sl = np.zeros((8, F), np.float32)
        sc = np.zeros((8, F), np.float32)
        acc = np.zeros(F, np.float32)
        k = 0
        for i in range(nx):
            j = xrec[xs + i, 0] // ldxb
            w = xrec[xs + i, 1:2].view(np.float32)[0]
            acc = (acc + w * X[j]).astype(np.float32)
            if (xm >> i) & 1:
                sl[(xsl >> 4 * k) & 15] = acc
                acc[:] = 0
                k += 1
        k = 0
        for i in range(nc):
            node = crec[cs + i, 0] // ldcb
            w = crec[cs + i, 1:2].view(np.float32)[0]
            acc = (acc + w * xf[node]).astype(np.float32)
            if (cm >> i) & 1:
                sc[(csl >> 4 * k) & 15] = acc
                acc[:] = 0
                k += 1
        for s in range(nr):
            v = sl[s] + sc[s]
            if s == nr - 1 and (fl & 2):
                carry[t, 1] = v
            elif s == 0 and (fl & 1):
                carry[t, 0] = v
            else:
                out[r0 + s] = v
    for r, ts, te in jobs:
        s = carry[ts, 1].copy()
        for u in range(ts + 1, te):
            s += carry[u, 1]
        s += carry[te, 0]
        out[r] = s
    return out


def main():
    cpu = "--cpu" in sys.argv
    args = [a for a in sys.argv[1:] if a != "--cpu"]
    reps = int(args[0]) if len(args) > 0 else 30
    Us = [int(u) for u in (args[1] if len(args) > 1 else "16").split(",")]
    U = Us[0]
    R = int(args[2]) if len(args) > 2 else 8
    K = int(args[3]) if len(args) > 3 else 64
    import torch
    import vqgnn_pkg
    vqgnn_pkg.load()
    from vq_gnn_amd.graph import CONFIGS, make_batch
    cfg = dict(CONFIGS["arxiv_gcn"])
    F, M, D = cfg["F"], cfg["M"], 4
    nb = F // D
    t0 = time.time()
    g, _, b = make_batch(cfg)
    B, n, nnz, N = b.B, b.n, b.nnz, cfg["N"]
    print(f"batch B={B} n={n} nnz={nnz} ({time.time() - t0:.1f}s)", flush=True)
    gen = torch.Generator(device="cpu").manual_seed(3)
    X = torch.randn(B, F, generator=gen)
    codes = torch.randint(0, M, (N, nb), dtype=torch.int16, generator=gen)
    emb_out = torch.randn(nb, M, 2 * D, generator=gen)
    ldxb, ldcb = F * 4, nb * 2
    t0 = time.time()
    meta, xrec, crec, jobs, tasks = build_plan(b.rowptr, b.col, b.val, B, b.subset, ldxb, ldcb,
                                               K=K, R=R)
    print(f"plan: {meta.shape[0]} tasks, {jobs.shape[0]} cut rows, X stream {xrec.shape[0]}, "
          f"CB stream {crec.shape[0]} ({time.time() - t0:.1f}s)", flush=True)
    # x_first rows of every node: the codeword feature halves by code
    feat = emb_out[:, :, :D]                       # [nb, M, D]
    xf_node = feat[torch.arange(nb)[None, :], codes.long()].reshape(N, F).numpy()
    rowptr, col, val = b.rowptr, b.col, b.val
    xin = np.concatenate([X.numpy(), xf_node[b.subset[B:]]]).astype(np.float64)
    ref = np.zeros((n, F))
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    np.add.at(ref, rows, val[:, None].astype(np.float64) * xin[col])
    mag = np.zeros((n, F))
    np.add.at(mag, rows, np.abs(val[:, None].astype(np.float64) * xin[col]))
    if cpu:
        emu = emulate(meta, xrec, crec, jobs, X.numpy(), xf_node, ldxb, ldcb, n, F)
        bad = np.abs(emu - ref) > 1e-5 * mag + 1e-30
        print(f"emulation vs fp64: {int(bad.sum())} elements off (max rel "
              f"{(np.abs(emu - ref) / (mag + 1e-30)).max():.2e})", flush=True)
        return
    from vq_gnn_amd import kernels
    from vq_gnn_amd.graph import batch_to_device
    dev = torch.device("cuda:0")
    bidx, subset, adj = batch_to_device(b, dev)
    Xd, codes_d, emb_d = X.to(dev), codes.to(dev), emb_out.to(dev)
    plan = adj.plan(F, B=B)
    plan_cb = plan.with_codebook_source(B, subset, N)
    out_ship = torch.empty(n, F, device=dev)
    out_w3 = torch.empty(n, F, device=dev)
    so = ctypes.CDLL(os.path.join(ROOT, "vq-gnn_amd", "lib", "probe_walk3.so"))
    so.walk3_run.restype = ctypes.c_int
    P = ctypes.c_void_p
    so.walk3_run.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int, ctypes.c_uint32,
                             ctypes.c_uint32, P, ctypes.c_uint32,
                             P, ctypes.c_uint32, P, ctypes.c_longlong, ctypes.c_longlong,
                             ctypes.c_int, ctypes.c_int, P, ctypes.c_uint32, P, ctypes.c_int,
                             ctypes.c_int, P, ctypes.c_int, P]
    meta_d = torch.from_numpy(meta.view(np.int32)).to(dev)
    xrec_d = torch.from_numpy(xrec).to(dev)
    crec_d = torch.from_numpy(crec).to(dev)
    jobs_d = torch.from_numpy(jobs if jobs.size else np.zeros((1, 3), np.int32)).to(dev)
    T = meta.shape[0]
    cf = F + 4
    carry = torch.zeros(T * 2 * cf + 64, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def ship():
        kernels.spmm_codebook(adj.rowptr, n, nnz, Xd, F, B, codes_d, emb_d, D, plan_cb, out=out_ship)

    def w3(U=U):
        rc = so.walk3_run(U, R, p(meta_d), p(xrec_d), p(crec_d), T, xrec.shape[0] - 32,
                          crec.shape[0] - 32, p(Xd), B * F * 4, p(codes_d),
                          N * nb * 2, p(emb_d), emb_d.stride(1), emb_d.stride(0), M, D, p(out_w3),
                          F * 4, p(carry), cf, F, p(jobs_d), int(jobs.shape[0]),
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc

    ship()
    torch.cuda.synchronize()
    got = out_ship.cpu().numpy().astype(np.float64)
    bad = np.abs(got - ref) > 1e-5 * mag + 1e-30
    print(f"shipped: {int(bad.sum())} elements off fp64 (max rel "
          f"{(np.abs(got - ref) / (mag + 1e-30)).max():.2e})", flush=True)
    for u in Us:
        out_w3.fill_(float("nan"))
        w3(u)
        torch.cuda.synchronize()
        got = out_w3.cpu().numpy().astype(np.float64)
        bad = ~(np.abs(got - ref) <= 1e-5 * mag + 1e-30)
        print(f"walk variant {u}: {int(bad.sum())} elements off fp64 (max rel "
              f"{np.nanmax(np.abs(got - ref) / (mag + 1e-30)):.2e})", flush=True)

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

    for _ in range(2):
        for nm, fn in [("shipped", ship)] + [(f"walk variant {u} R={R} K={K}", (lambda u=u: w3(u)))
                                             for u in Us]:
            t, ts = timeit(fn)
            print(f"{nm:28s} {t:8.1f} us ({', '.join(f'{x:.1f}' for x in ts)})", flush=True)


if __name__ == "__main__":
    main()
