"""Random-walk sampling ('edge' / 'rw' / 'cont' samplers) on
the arxiv-shaped graph: the device walk (vqgnn_random_walk, include/vqgnn.h
§9b) against a vectorised numpy restatement of torch_cluster's uniform step
(the reference's SparseTensor.random_walk, dataloader.py:70-90) on one host
thread, which draws its own uniforms.  The first walkers are checked against
the oracle (oracle/subgraph_ref.py) with the device's own uniforms.
Prints one JSON line.

usage: python scripts/bench_walk.py [--roots 50000] [--walk-length 4] [--reps 20]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from oracle import subgraph_ref  # noqa: E402
from vq_gnn_amd import graph, kernels  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="arxiv_gcn")
p.add_argument("--roots", type=int, default=50000)
p.add_argument("--walk-length", type=int, default=4)
p.add_argument("--reps", type=int, default=20)
p.add_argument("--cpu-reps", type=int, default=5)
args = p.parse_args()
cfg = graph.CONFIGS[args.config]
g = graph.synthetic_graph(cfg["N"], cfg["parts"], cfg["edges"], seed=cfg.get("seed", 0))
rp = np.asarray(g.rowptr, dtype=np.int64)
cl = np.asarray(g.col, dtype=np.int64)
dev = torch.device("cuda:0")
rp_d = torch.from_numpy(rp).to(dev)
cl_d = torch.from_numpy(cl.astype(np.int32)).to(dev)
rng = np.random.default_rng(0)
start = rng.integers(0, g.N, size=args.roots)
start_d = torch.from_numpy(start).to(dev)
L = args.walk_length

# parity on the first walkers: the device's uniforms through the oracle
seed = 12345
out = kernels.random_walk(rp_d, cl_d, g.N, start_d, L, seed).cpu().numpy()
k = 300
u = subgraph_ref.walk_uniforms(seed, k, L)
ref = subgraph_ref.random_walk(rp, cl, start[:k], L, u)
assert np.array_equal(out[:k], ref), "device walk != oracle"

for _ in range(3):
    kernels.random_walk(rp_d, cl_d, g.N, start_d, L, seed)
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(args.reps):
    kernels.random_walk(rp_d, cl_d, g.N, start_d, L, seed + r)
torch.cuda.synchronize()
gpu_ms = (time.perf_counter() - t0) / args.reps * 1e3


def cpu_walk(start, L, rng):
    """torch_cluster's uniform step, vectorised over walkers (one thread)."""
    v = start.copy()
    walks = np.empty((start.shape[0], L + 1), dtype=np.int64)
    walks[:, 0] = v
    for step in range(L):
        rs, re = rp[v], rp[v + 1]
        deg = re - rs
        uu = rng.random(v.shape[0], dtype=np.float32)
        e = rs + (uu * deg.astype(np.float32)).astype(np.int64)
        nxt = cl[np.minimum(e, np.maximum(re - 1, 0))]
        v = np.where(deg > 0, nxt, v)
        walks[:, step + 1] = v
    return walks


cpu_walk(start, L, rng)
times = []
for _ in range(args.cpu_reps):
    t0 = time.perf_counter()
    cpu_walk(start, L, rng)
    times.append(time.perf_counter() - t0)
cpu_ms = float(np.median(times)) * 1e3
print(json.dumps({
    "metric": "random walks (torch_cluster uniform step), arxiv-shaped graph",
    "roots": args.roots, "walk_length": L, "N": int(g.N), "edges": int(cl.shape[0]),
    "gpu_ms": gpu_ms, "gpu_steps_per_s": args.roots * L / (gpu_ms * 1e-3),
    "cpu_ms": cpu_ms, "cpu_steps_per_s": args.roots * L / (cpu_ms * 1e-3), "cpu_threads": 1,
    "cpu": "vectorised numpy restatement (one thread), own uniforms",
    "parity": f"first {k} walkers == oracle (device uniforms)",
    "gpu_includes": "one status read per call (vqgnn_random_walk's range check)"}))
