"""CPU baseline leg of bench.py — the reference algorithm on the host cores.

One "layer step" exactly as the reference runs it on a CPU-only torch
(SURVEY.md §8d): for each of the nb branches VectorQuantizerEMA.update
(vq.py:204-279, op for op incl. the dense [B, M] one-hot — oracle/vq_ref.py),
the per-branch codebook gather + torch.cat (models.py:157-174), and the
aggregation A @ x_input.  torch_sparse is not installed, so torch's CSR
matmul stands in for torch_sparse spmm_sum (row-parallel on all threads).
TEST/BASELINE INFRASTRUCTURE ONLY.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from . import vq_ref


def layer_step_timer(X, G, batch, codes, M, D, threads, max_seconds=12.0, min_steps=2):
    torch.set_num_threads(threads)
    B, F = X.shape
    nb = F // D
    states = [vq_ref.new_state(M, D, warm_up=True) for _ in range(nb)]
    for b, st in enumerate(states):   # one feature_update warm pass (as the GPU leg)
        vq_ref.feature_update(st, X[:, b * D:(b + 1) * D])
    A = torch.sparse_csr_tensor(torch.from_numpy(batch.rowptr), torch.from_numpy(batch.col),
                                torch.from_numpy(batch.val), (batch.n, batch.n))
    bidx = torch.from_numpy(batch.batch_idx)
    first = torch.from_numpy(batch.subset[B:])
    codes = codes.clone()

    def step():
        for b, st in enumerate(states):
            idx, _, _ = vq_ref.update(st, X[:, b * D:(b + 1) * D], G[:, b * D:(b + 1) * D])
            codes[bidx, b] = idx[:, 0].to(torch.int16)
        parts = [states[b]["embedding_output"][codes[first, b].long()][:, :D] for b in range(nb)]
        x_input = torch.cat([X, torch.cat(parts, dim=1)])
        return A @ x_input

    step()  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < min_steps or (time.perf_counter() - t_start) < max_seconds:
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
        if len(times) >= 50:
            break
    return float(np.median(times)), len(times)
