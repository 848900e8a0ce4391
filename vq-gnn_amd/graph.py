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
    "reddit_gcn": dict(N=232_965, parts=50, edges=57_300_000, F=128, M=1024, conv="GCN",
                       batch_nodes=10_000, seed=0),
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
