"""Synthetic graphs and the reference's mini-batch layout (host-side harness).

The reference loads OGB/PyG datasets (network; vq_gnn_v2/utils/misc.py:144-224)
and builds batches on the CPU in ``OurDataLoader._k_hop_subgraph``
(vq_gnn_v2/dataloader.py:98-148) + ``prepare_batch_input`` (misc.py:57-75).
Neither is on the hot path (SURVEY.md §8f lists GPU batch construction as the
next row).  This module restates the batch *layout* contract in numpy so the
bench and tests feed the kernels exactly what the reference feeds its layer:

  subset = [batch nodes in loader order, then the 1-hop out-of-batch nodes in
  ascending global id]; adjacency = every edge with both ends in subset
  (train) or with its row in the batch (eval), relabelled, CSR sorted by
  (row, col), values = the normalised weights of the full graph (norm_adj).

Graph generator: contiguous "METIS-like" clusters, a fixed
fraction of intra-cluster edges, Zipf-weighted endpoints (hub nodes), no
self-edges, deduplicated, symmetrised.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class Graph:
    N: int
    rowptr: np.ndarray      # int64 [N+1], symmetric, sorted cols, no self loops
    col: np.ndarray         # int64 [nnz]
    cluster_ptr: np.ndarray  # int64 [parts+1], contiguous clusters

    @property
    def nnz(self):
        return int(self.col.shape[0])


def synthetic_graph(N, num_parts, num_undirected_edges, intra_frac=0.8, zipf_a=0.9,
                    seed=0) -> Graph:
    rng = np.random.default_rng(seed)
    sizes = np.full(num_parts, N // num_parts, dtype=np.int64)
    sizes[: N % num_parts] += 1
    cptr = np.zeros(num_parts + 1, dtype=np.int64)
    cptr[1:] = np.cumsum(sizes)
    # Zipf weight by a random rank inside each cluster
    w = np.empty(N, dtype=np.float64)
    for c in range(num_parts):
        s, e = cptr[c], cptr[c + 1]
        ranks = rng.permutation(e - s) + 1
        w[s:e] = ranks.astype(np.float64) ** (-zipf_a)
    cum = np.concatenate([[0.0], np.cumsum(w)])

    def sample_in(clusters, u):
        lo, hi = cum[cptr[clusters]], cum[cptr[clusters + 1]]
        idx = np.searchsorted(cum, lo + u * (hi - lo), side="right") - 1
        return np.clip(idx, cptr[clusters], cptr[clusters + 1] - 1)

    target = int(num_undirected_edges)
    keys = np.empty(0, dtype=np.int64)
    want = target
    while keys.shape[0] < target:
        m = int(want * 1.3) + 1024
        ca = rng.choice(num_parts, size=m, p=sizes / N)
        intra = rng.random(m) < intra_frac
        cb = np.where(intra, ca, (ca + rng.integers(1, max(num_parts, 2), size=m)) % num_parts)
        a = sample_in(ca, rng.random(m))
        b = sample_in(cb, rng.random(m))
        keep = a != b
        lo, hi = np.minimum(a[keep], b[keep]), np.maximum(a[keep], b[keep])
        keys = np.unique(np.concatenate([keys, lo * N + hi]))
        want = target - keys.shape[0]
    if keys.shape[0] > target:
        keys = np.sort(rng.choice(keys, size=target, replace=False))
    u, v = keys // N, keys % N
    r = np.concatenate([u, v])
    c = np.concatenate([v, u])
    order = np.lexsort((c, r))
    r, c = r[order], c[order]
    rowptr = np.zeros(N + 1, dtype=np.int64)
    rowptr[1:] = np.cumsum(np.bincount(r, minlength=N))
    return Graph(N, rowptr, c.astype(np.int64), cptr)


def synthetic_graph_device(N, num_parts, num_undirected_edges, intra_frac=0.8, zipf_a=0.9,
                           seed=0, device="cuda"):
    """``synthetic_graph``'s generator with torch ops on the device: the same
    distribution (contiguous clusters, intra_frac intra-cluster edges,
    Zipf-weighted endpoints, no self edges, deduplicated, symmetrised) from
    its own RNG stream, for reddit-sized graphs (57 M undirected edges) that
    take minutes in numpy.  -> loader.DeviceGraph (no edge values) and the
    cluster pointer."""
    from .loader import DeviceGraph
    dev = torch.device(device)
    gen = torch.Generator(device=dev).manual_seed(seed)
    i64 = dict(dtype=torch.int64, device=dev)
    sizes = torch.full((num_parts,), N // num_parts, **i64)
    sizes[: N % num_parts] += 1
    cptr = torch.zeros(num_parts + 1, **i64)
    cptr[1:] = torch.cumsum(sizes, 0)
    cl = torch.repeat_interleave(torch.arange(num_parts, **i64), sizes)
    # Zipf weight by a random rank inside each cluster
    key = cl.double() + 0.5 * torch.rand(N, generator=gen, device=dev, dtype=torch.float64)
    order = torch.argsort(key)
    rank = torch.empty(N, **i64)
    rank[order] = torch.arange(N, **i64) - cptr[cl[order]] + 1
    cum = torch.cat([torch.zeros(1, dtype=torch.float64, device=dev),
                     torch.cumsum(rank.double() ** (-zipf_a), 0)])

    def sample_in(c, u):
        lo, hi = cum[cptr[c]], cum[cptr[c + 1]]
        idx = torch.searchsorted(cum, lo + u * (hi - lo), right=True) - 1
        return torch.minimum(torch.maximum(idx, cptr[c]), cptr[c + 1] - 1)

    target = int(num_undirected_edges)
    keys = torch.empty(0, **i64)
    want = target
    while keys.numel() < target:
        m = int(want * 1.3) + 1024
        ca = cl[torch.randint(0, N, (m,), generator=gen, device=dev)]   # P(c) = size_c / N
        intra = torch.rand(m, generator=gen, device=dev) < intra_frac
        cb = torch.where(intra, ca, (ca + torch.randint(1, max(num_parts, 2), (m,), generator=gen,
                                                        device=dev)) % num_parts)
        a = sample_in(ca, torch.rand(m, generator=gen, device=dev, dtype=torch.float64))
        b = sample_in(cb, torch.rand(m, generator=gen, device=dev, dtype=torch.float64))
        keep = a != b
        a, b = a[keep], b[keep]
        keys = torch.unique(torch.cat([keys, torch.minimum(a, b) * N + torch.maximum(a, b)]))
        del ca, intra, cb, a, b, keep
        want = target - keys.numel()
    if keys.numel() > target:
        sel = torch.randperm(keys.numel(), generator=gen, device=dev)[:target]
        keys = torch.sort(keys[sel]).values
    u, v = keys // N, keys % N
    del keys
    k2 = torch.sort(torch.cat([u * N + v, v * N + u])).values
    del u, v
    r, c = k2 // N, k2 % N
    del k2
    rowptr = torch.zeros(N + 1, **i64)
    rowptr[1:] = torch.cumsum(torch.bincount(r, minlength=N), 0)
    g = DeviceGraph(rowptr, c.to(torch.int32), None, N, dev)
    return g, cptr


def make_batch_device(cfg: dict, rank: int = 0, device="cuda", graph=None):
    """``make_batch`` built on the device (graph: synthetic_graph_device,
    normalisation: vqgnn_norm_adj, batch: vqgnn_khop_subset/edges) for the
    reddit-sized configs.  -> (normalised DeviceGraph, (batch_idx, subset,
    CSR)); ``graph`` reuses a normalised DeviceGraph."""
    from .preprocess import norm_adj_graph
    dev = torch.device(device)
    if graph is None:
        g, cptr = synthetic_graph_device(cfg["N"], cfg["parts"], cfg["edges"],
                                         seed=cfg.get("seed", 0), device=dev)
        graph = norm_adj_graph(g, cfg["conv"], dev)
        graph.cluster_ptr = cptr
        del g
    gen = torch.Generator(device=dev).manual_seed(3 + rank)
    if "batch_clusters" in cfg:
        cptr = graph.cluster_ptr.cpu()
        perm = torch.randperm(cfg["parts"], generator=gen, device=dev).cpu()
        node_idx = torch.cat([torch.arange(int(cptr[c]), int(cptr[c + 1]))
                              for c in perm[: cfg["batch_clusters"]].tolist()]).to(dev)
    else:
        node_idx = torch.randperm(graph.N, generator=gen, device=dev)[: cfg["batch_nodes"]]
    return graph, graph.batch(node_idx)


def norm_adj(g: Graph, conv_type: str):
    """vq_gnn_v2/utils/misc.py:14-34.  Returns (rowptr, col, val) of the
    normalised full-graph adjacency (float32 values as torch_sparse keeps)."""
    N = g.N
    rowptr, col = g.rowptr, g.col
    if conv_type in ("GCN", "GAT"):  # set_diag(): add self loops
        row = np.repeat(np.arange(N), np.diff(rowptr))
        r = np.concatenate([row, np.arange(N)])
        c = np.concatenate([col, np.arange(N)])
        order = np.lexsort((c, r))
        r, c = r[order], c[order]
        rowptr = np.zeros(N + 1, dtype=np.int64)
        rowptr[1:] = np.cumsum(np.bincount(r, minlength=N))
        col = c
    deg = np.diff(rowptr).astype(np.float32)          # adj_t.sum(dim=1) of ones
    row = np.repeat(np.arange(N), np.diff(rowptr))
    ones = np.ones(col.shape[0], dtype=np.float32)
    if conv_type == "GCN":
        with np.errstate(divide="ignore"):
            dis = deg ** np.float32(-0.5)
        dis[np.isinf(dis)] = 0
        val = (dis[row] * ones) * dis[col]
    elif conv_type in ("SAGE", "GAT"):
        with np.errstate(divide="ignore"):
            di = deg ** np.float32(-1)
        di[np.isinf(di)] = 0
        val = di[row] * ones
    else:
        raise ValueError('GNN conv type not supported')
    return rowptr, col, val.astype(np.float32)


@dataclass
class Batch:
    batch_idx: np.ndarray   # int64 [B]
    subset: np.ndarray      # int64 [n]
    rowptr: np.ndarray      # int64 [n+1] local CSR sorted by (row, col)
    col: np.ndarray         # int64 [nnz]
    val: np.ndarray         # float32 [nnz]

    @property
    def B(self):
        return int(self.batch_idx.shape[0])

    @property
    def n(self):
        return int(self.subset.shape[0])

    @property
    def nnz(self):
        return int(self.col.shape[0])


def k_hop_batch(rowptr, col, val, N, node_idx, train_flag=True) -> Batch:
    """dataloader.py:98-148 (num_hops=1, relabel) + misc.py:73 CSR sort."""
    node_idx = np.asarray(node_idx, dtype=np.int64)
    deg = np.diff(rowptr)
    row_all = np.repeat(np.arange(N), deg)
    # neighbours of batch nodes: col[edge_mask] with edge_mask = node_mask[row]
    node_mask = np.zeros(N, dtype=bool)
    node_mask[node_idx] = True
    nbr = col[node_mask[row_all]]
    uniq = np.unique(np.concatenate([node_idx, nbr]))         # torch.unique (sorted)
    inv = np.searchsorted(uniq, node_idx)
    keep = np.ones(uniq.shape[0], dtype=bool)
    keep[inv] = False
    subset = np.concatenate([uniq[inv], uniq[keep]])
    assert np.array_equal(node_idx, subset[: node_idx.size])  # dataloader.py:128
    node_mask[:] = False
    if train_flag:
        node_mask[subset] = True
        emask = node_mask[row_all] & node_mask[col]
    else:
        node_mask[node_idx] = True
        emask = node_mask[row_all]
    remap = np.full(N, -1, dtype=np.int64)
    remap[subset] = np.arange(subset.shape[0])
    r, c, w = remap[row_all[emask]], remap[col[emask]], val[emask]
    n = subset.shape[0]
    order = np.lexsort((c, r))                                 # SparseTensor sorts (row, col)
    r, c, w = r[order], c[order], w[order]
    lrowptr = np.zeros(n + 1, dtype=np.int64)
    lrowptr[1:] = np.cumsum(np.bincount(r, minlength=n))
    return Batch(node_idx, subset, lrowptr, c, w.astype(np.float32))


def cluster_batch(g: Graph, clusters) -> np.ndarray:
    """__collate_cluster__ (dataloader.py:52-58): concatenated cluster ranges."""
    return np.concatenate([np.arange(g.cluster_ptr[c], g.cluster_ptr[c + 1]) for c in clusters])


# ---- canonical configs ----
CONFIGS = {
    # name: (N, parts, undirected edges, F_in, hidden, out, M, conv, batch clusters or nodes)
    "arxiv_gcn": dict(N=169_343, parts=80, edges=1_158_000, F=128, M=256, conv="GCN",
                      batch_clusters=40, seed=0),
    "arxiv_gat": dict(N=169_343, parts=80, edges=1_158_000, F=128, M=1024, conv="GAT",
                      batch_clusters=40, seed=0),
    "ppi_sage": dict(N=44_906, parts=1, edges=615_000, F=256, M=4096, conv="SAGE",
                     batch_nodes=30_000, seed=0),
    # reddit (README.md:75): 602 input features zero-padded to 604 = 151
    # branches of D = 4 in layer 1 (vq_gnn_v2/utils/misc.py:212-216), hidden
    # 128 after it; built on the device
    # (make_batch_device: 57.3 M undirected edges take minutes in numpy)
    "reddit_gcn": dict(N=232_965, parts=50, edges=57_300_000, F=128, M=1024, conv="GCN",
                       batch_nodes=10_000, seed=0, device_build=True),
    "reddit_gcn_l1": dict(N=232_965, parts=50, edges=57_300_000, F=604, M=1024, conv="GCN",
                          batch_nodes=10_000, seed=0, device_build=True),
}


def make_batch(cfg: dict, rank: int = 0, train_flag=True, graph=None):
    """Build (graph, normalised adjacency, Batch) for a config; ``rank`` picks a
    different batch of the same graph (weak scaling across GPUs)."""
    g = graph if graph is not None else synthetic_graph(cfg["N"], cfg["parts"], cfg["edges"],
                                                        seed=cfg.get("seed", 0))
    rp, cl, vl = norm_adj(g, cfg["conv"])
    rng = np.random.default_rng(3 + rank)
    if "batch_clusters" in cfg:
        perm = rng.permutation(cfg["parts"])
        node_idx = cluster_batch(g, perm[: cfg["batch_clusters"]])
    else:
        node_idx = rng.permutation(g.N)[: cfg["batch_nodes"]]
    return g, (rp, cl, vl), k_hop_batch(rp, cl, vl, g.N, node_idx, train_flag)


def batch_to_device(batch: Batch, device):
    """prepare_batch_input (misc.py:57-75) minus x: (batch_idx, subset, CSR)."""
    from .sparse import CSR
    adj = CSR(torch.from_numpy(batch.rowptr), torch.from_numpy(batch.col),
              torch.from_numpy(batch.val), (batch.n, batch.n)).to(device)
    return (torch.from_numpy(batch.batch_idx).to(device),
            torch.from_numpy(batch.subset).to(device), adj)
