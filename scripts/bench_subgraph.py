"""Batch construction on the arxiv-shaped config: the device
path (DeviceGraph.batch: k-hop subset + CSR, include/vqgnn.h §9) against the
CPU restatement of the reference path (_k_hop_subgraph + SparseTensor build,
oracle/subgraph_ref.py, torch CPU).  Prints one JSON line.

usage: python scripts/bench_subgraph.py [--config arxiv_gcn] [--reps 20]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import graph  # noqa: E402
from vq_gnn_amd.loader import DeviceGraph  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="arxiv_gcn")
p.add_argument("--reps", type=int, default=20)
p.add_argument("--cpu-reps", type=int, default=3)
args = p.parse_args()
cfg = graph.CONFIGS[args.config]
dev = torch.device("cuda:0")
g, (rp, cl, vl), b = graph.make_batch(cfg)
dg = DeviceGraph(torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vl), g.N, dev)
node_idx = torch.from_numpy(b.batch_idx)
node_idx_d = node_idx.to(dev)

for _ in range(3):
    dg.batch(node_idx_d)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.reps):
    _, subset, adj = dg.batch(node_idx_d)
torch.cuda.synchronize()
gpu_ms = (time.perf_counter() - t0) / args.reps * 1e3
for _ in range(3):
    dg.k_hop_subgraph(node_idx_d)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.reps):
    dg.k_hop_subgraph(node_idx_d)
torch.cuda.synchronize()
gpu_ref_ms = (time.perf_counter() - t0) / args.reps * 1e3

from oracle import subgraph_ref  # noqa: E402  (CPU baseline only)

threads = min(16, os.cpu_count() or 1)
torch.set_num_threads(threads)
rp_t, cl_t, vl_t = torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vl)
ts = []
for _ in range(args.cpu_reps + 1):
    t0 = time.perf_counter()
    s, ei, w = subgraph_ref.k_hop_subgraph(rp_t, cl_t, vl_t, g.N, node_idx)
    subgraph_ref.sparse_tensor_csr(ei[0], ei[1], w, s.numel(), s.numel())
    ts.append(time.perf_counter() - t0)
cpu_ms = float(np.median(ts[1:])) * 1e3
# algorithmic bytes: the batch rows' CSR slices + the kept entries' node_map
# lookups and the outputs (int32 col, fp32 val, int32 rowptr, int64 subset)
deg = np.diff(rp)
touched = int(deg[b.subset].sum())
alg = 8 * (b.n + 1) + touched * (4 + 4 + 4) + b.nnz * 8 + 4 * (b.n + 1) + 8 * b.n
print(json.dumps(dict(
    what="batch construction (_k_hop_subgraph + CSR), " + args.config,
    B=b.B, n=b.n, nnz=b.nnz, graph_nodes=g.N, graph_edges=int(cl.shape[0]),
    gpu_ms_csr=gpu_ms, gpu_ms_reference_order=gpu_ref_ms,
    cpu_ms_reference_restatement=cpu_ms, cpu_threads=threads,
    speedup=cpu_ms / gpu_ms, alg_bytes=alg, gpu_gbs=alg / (gpu_ms * 1e-3) / 1e9,
    note="gpu times are wall-clock per call incl. the one sizes readback; cpu = "
         "oracle/subgraph_ref.py (torch CPU) median of %d" % args.cpu_reps)))
