"""CPU baseline leg of bench.py — the reference algorithm on the host cores.

One "layer step" exactly as the reference runs it on a CPU-only torch
(SURVEY.md §8d): for each of the nb branches VectorQuantizerEMA.update
(vq.py:204-279, op for op incl. the dense [B, M] one-hot — oracle/vq_ref.py),
the per-branch codebook gather + torch.cat (models.py:157-174), and the
aggregation A @ x_input (GCN/SAGE, convs.py:95) or, for GAT, the attention
coefficients exp(leaky(alpha_l[j]/s + alpha_r[i]/s)) * w and the weighted sum
with the ones column and the row normalisation of rows < B (convs.py:189-266,
vq_softmax.py:33-57, models.py:187-189).  torch_sparse / torch_scatter are
not installed, so torch's CSR matmul stands in for their spmm_sum /
segment_csr (row-parallel on all threads).
TEST/BASELINE INFRASTRUCTURE ONLY.

Bounded samples (bench.py keeps the default run within minutes): the VQ
update may run on a sample of the branches (the time scaled by nb / sampled,
every branch does the same work) and the aggregation on a leading block of
rows holding about ``edge_sample`` edges (the time scaled by nnz / edges in
the block: the CSR product is linear in the edges at fixed F).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from . import vq_ref


def _row_block(rowptr: np.ndarray, edge_sample):
    """Leading rows [0, r1) holding about edge_sample edges (all rows if None)."""
    n = rowptr.shape[0] - 1
    if edge_sample is None or edge_sample >= rowptr[-1]:
        return n
    return int(max(1, min(n, np.searchsorted(rowptr, edge_sample, side="right"))))


def layer_step_timer(X, G, batch, codes, M, D, threads, max_seconds=12.0, min_steps=5,
                     branch_sample=None, edge_sample=None, gat=None):
    """-> (seconds per full layer step, timed steps, description of the sample).

    batch: anything with batch_idx, subset, rowptr, col, val (numpy) and n.
    gat: None, or (att_l [F+1], att_r [F+1]) float32 for the GAT aggregation.
    The estimate per step is t_vq * nb / branches + t_gather + t_agg * nnz /
    edges_in_block, the median over the timed steps."""
    torch.set_num_threads(threads)
    B, F = X.shape
    nb = F // D
    nbs = nb if branch_sample is None else max(1, min(nb, int(branch_sample)))
    states = [vq_ref.new_state(M, D, warm_up=True) for _ in range(nbs)]
    for b, st in enumerate(states):   # one feature_update warm pass (as the GPU leg)
        vq_ref.feature_update(st, X[:, b * D:(b + 1) * D])
    rowptr = np.asarray(batch.rowptr, dtype=np.int64)
    nnz = int(rowptr[-1])
    r1 = _row_block(rowptr, edge_sample)
    e1 = int(rowptr[r1])
    A = torch.sparse_csr_tensor(torch.from_numpy(rowptr[:r1 + 1].copy()),
                                torch.from_numpy(np.asarray(batch.col[:e1], dtype=np.int64)),
                                torch.from_numpy(np.asarray(batch.val[:e1], dtype=np.float32)),
                                (r1, batch.n))
    bidx = torch.from_numpy(np.asarray(batch.batch_idx, dtype=np.int64))
    first = torch.from_numpy(np.asarray(batch.subset[B:], dtype=np.int64))
    codes = codes.clone()
    if gat is not None:
        att_l, att_r = (torch.as_tensor(np.asarray(a, dtype=np.float32)).view(-1) for a in gat)
        row = torch.repeat_interleave(torch.arange(r1), torch.from_numpy(np.diff(rowptr[:r1 + 1])))
        colb = A.col_indices()
        wb = A.values()

    def step():
        t0 = time.perf_counter()
        for b, st in enumerate(states):
            idx, _, _ = vq_ref.update(st, X[:, b * D:(b + 1) * D], G[:, b * D:(b + 1) * D])
            codes[bidx, b] = idx[:, 0].to(torch.int16)
        t1 = time.perf_counter()
        parts = [states[b % nbs]["embedding_output"][codes[first, b].long()][:, :D]
                 for b in range(nb)]
        x_input = torch.cat([X, torch.cat(parts, dim=1)])
        t2 = time.perf_counter()
        if gat is None:
            _ = A @ x_input
        else:
            xin = torch.cat([x_input, torch.ones(x_input.shape[0], 1)], 1)
            al = (xin * att_l).sum(-1)
            ar = (xin * att_r).sum(-1)
            s = torch.sqrt(torch.max(al) ** 2 + 1) * torch.sqrt(torch.max(ar) ** 2 + 1)
            al, ar = al / s, ar / s
            coef = torch.nn.functional.leaky_relu(al[colb] + ar[row], 0.2).exp() * wb
            Ac = torch.sparse_csr_tensor(A.crow_indices(), colb, coef, (r1, batch.n))
            out = Ac @ xin
            nB = min(B, r1)
            out[:nB, :-1] /= out[:nB, -1:] + 1e-16
        t3 = time.perf_counter()
        return (t1 - t0) * nb / nbs + (t2 - t1) + (t3 - t2) * nnz / max(e1, 1)

    step()  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < min_steps or (time.perf_counter() - t_start) < max_seconds:
        times.append(step())
        if len(times) >= 50:
            break
    if nbs == nb and e1 == nnz:
        desc = "full layer step"
    else:
        desc = (f"VQ update on {nbs} of {nb} branches (x {nb / nbs:.3g}), aggregation on the "
                f"first {r1} rows = {e1} of {nnz} edges (x {nnz / max(e1, 1):.3g})")
    return float(np.median(times)), len(times), desc


def host_topology() -> dict:
    """CPU model, logical CPUs of the machine, this process's affinity set and
    the physical core / socket counts from /proc/cpuinfo."""
    import os
    info = dict(logical_cpus=os.cpu_count(), affinity=len(os.sched_getaffinity(0)))
    try:
        model, phys, cores = None, set(), set()
        pid = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "physical id":
                pid = v
                phys.add(v)
            elif k == "core id":
                cores.add((pid, v))
        info.update(model=model, sockets=len(phys) or None, physical_cores=len(cores) or None)
    except OSError:
        pass
    return info
