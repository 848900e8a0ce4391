"""Mini-batch construction on the device.

Mirrors the reference's batch pipeline with the arithmetic in HIP
(include/vqgnn.h §9):

* ``DeviceGraph.k_hop_subgraph`` = ``OurDataLoader._k_hop_subgraph``
  (vq_gnn_v2/dataloader.py:98-148): same return ``(subset, edge_index,
  edge_w)``, same order; a node repeated in the batch keeps every copy in
  ``subset[:B]`` and relabels to its last copy, as the reference does.
* ``prepare_batch_input`` = vq_gnn_v2/utils/misc.py:57-75: returns
  ``(x[batch_idx], (batch_idx, subset, adj)), (num_B, num_B_prime)`` with
  ``adj`` the batch CSR sorted by (row, col), built on the device.
* ``OurDataLoader`` = vq_gnn_v2/dataloader.py:11-95 with every sampler:
  ``'node'``, ``'cluster'`` and the random-walk samplers ``'edge'``, ``'rw'``,
  ``'cont'`` (SparseTensor.random_walk -> torch_cluster's uniform walk, here
  ``vqgnn_random_walk`` with its own counter-based RNG seeded from torch's
  generator; include/vqgnn.h §9b).

Batches the loader yields carry their CSR (``SubgraphBatch.adj``), so
``prepare_batch_input`` does not rebuild it; the reference-order
``edge_index`` / ``edge_w`` are computed only if a caller indexes them.
"""
from __future__ import annotations

import torch

from . import kernels
from .sparse import CSR


class DeviceGraph:
    """The full normalised graph (``data.adj_t`` after ``norm_adj``) resident
    on the device: rowptr int64 [N+1], col int32, edge weights fp32."""

    def __init__(self, rowptr, col, value, num_nodes=None, device="cuda"):
        dev = torch.device(device)
        self.rowptr = torch.as_tensor(rowptr).to(device=dev, dtype=torch.int64).contiguous()
        self.col = torch.as_tensor(col).to(device=dev, dtype=torch.int32).contiguous()
        n_e = int(self.col.numel())
        self.has_value = value is not None       # torch_sparse adj_t without values
        if value is None:
            value = torch.ones(n_e, dtype=torch.float32)
        self.value = torch.as_tensor(value).to(device=dev, dtype=torch.float32).contiguous()
        self.N = int(num_nodes) if num_nodes is not None else int(self.rowptr.numel()) - 1
        if self.rowptr.numel() != self.N + 1:
            raise ValueError("rowptr must have num_nodes + 1 entries")
        if n_e >= 2 ** 31:
            raise ValueError("graph with >= 2^31 edges")

    @classmethod
    def from_adj(cls, adj_t, num_nodes=None, device="cuda"):
        """From a torch_sparse-like ``adj_t`` (``.csr()``), our ``CSR`` or a
        ``torch.sparse_csr`` tensor."""
        if isinstance(adj_t, torch.Tensor) and adj_t.layout == torch.sparse_csr:
            rp, cl, vl = adj_t.crow_indices(), adj_t.col_indices(), adj_t.values()
        else:
            rp, cl, vl = adj_t.csr()
        return cls(rp, cl, vl, num_nodes, device)

    @property
    def device(self):
        return self.rowptr.device

    # torch_sparse-like surface (data.adj_t)
    def csr(self):
        return self.rowptr, self.col, self.value

    def sparse_sizes(self):
        return (self.N, self.N)

    def nnz(self):
        return int(self.col.numel())

    def _run(self, node_idx, num_hops, train_flag, order):
        if isinstance(node_idx, (int, list, tuple)):          # dataloader.py:108-109
            node_idx = torch.tensor([node_idx]).flatten()
        return kernels.khop_subgraph(self.rowptr, self.col, self.value, self.N,
                                     torch.as_tensor(node_idx), num_hops, train_flag, order)

    def k_hop_subgraph(self, node_idx, num_hops=1, relabel_nodes=True, train_flag=True):
        """dataloader.py:98-148: (subset, edge_index [2, E] int64, edge_w)."""
        if not relabel_nodes:
            raise NotImplementedError("relabel_nodes=False (the loader always relabels)")
        r = self._run(node_idx, num_hops, train_flag, kernels.KHOP_ORDER_REF)
        edge_index = torch.stack([r["row"].to(torch.int64), r["col"].to(torch.int64)])
        return r["subset"], edge_index, r["val"]

    def batch(self, node_idx, num_hops=1, train_flag=True):
        """_k_hop_subgraph + the SparseTensor of prepare_batch_input (misc.py:73):
        (batch_idx, subset, CSR sorted by (row, col)) on the device."""
        node_idx = torch.as_tensor(node_idx)
        r = self._run(node_idx, num_hops, train_flag, kernels.KHOP_ORDER_CSR)
        n = r["n"]
        adj = CSR(r["rowptr"], r["col"], r["val"], (n, n))
        return node_idx.to(device=self.device, dtype=torch.int64), r["subset"], adj


class SubgraphBatch(tuple):
    """``(subset, edge_index, edge_w)`` as the reference's collate returns it
    (dataloader.py:146), holding the device CSR; edge_index / edge_w in the
    reference's order are produced on first access."""

    def __new__(cls, graph, node_idx, num_hops, train_flag):
        batch_idx, subset, adj = graph.batch(node_idx, num_hops, train_flag)
        self = super().__new__(cls, (subset, None, None))
        self.graph, self.node_idx, self.num_hops, self.train_flag = \
            graph, batch_idx, num_hops, train_flag
        self.adj = adj
        self._ref = None
        return self

    def _reference(self):
        if self._ref is None:
            self._ref = self.graph.k_hop_subgraph(self.node_idx, self.num_hops,
                                                  train_flag=self.train_flag)
        return self._ref

    def __getitem__(self, i):
        if isinstance(i, slice):
            return tuple(self[j] for j in range(*i.indices(3)))
        i = i + 3 if i < 0 else i
        if i == 0:
            return tuple.__getitem__(self, 0)
        if i in (1, 2):
            return self._reference()[i]
        raise IndexError(i)

    def __iter__(self):
        return iter((self[0], self[1], self[2]))


def prepare_batch_input(x, batch, device):
    """vq_gnn_v2/utils/misc.py:57-75 -> (x_B, (batch_idx, subset, adj)), (num_B, num_B')."""
    sub, batch_idx = batch[0], batch[-1]
    if isinstance(sub, SubgraphBatch):
        subset, adj = tuple.__getitem__(sub, 0), sub.adj
    else:
        subset, edge_index, edge_w = sub
        dim = int(subset.shape[0])
        dev = torch.device(device)
        ei = edge_index.to(dev)
        rp, cl, vl = kernels.coo_to_csr(ei[0], ei[1], edge_w.to(dev) if edge_w is not None
                                        else None, dim, dim)
        adj = CSR(rp, cl, vl, (dim, dim))
    adj = adj.to(device) if adj.device != torch.device(device) else adj
    num_B = int(batch_idx.shape[0])
    num_B_prime = int(subset.shape[0]) - num_B
    batch_idx_d = batch_idx.to(device)
    x_B = x[batch_idx_d] if x.device == batch_idx_d.device else x[batch_idx.cpu()].to(device)
    return (x_B, (batch_idx_d, subset.to(device), adj)), (num_B, num_B_prime)


class OurDataLoader(torch.utils.data.DataLoader):
    """vq_gnn_v2/dataloader.py:11-50 for sampler_type 'node' and 'cluster';
    the collate builds every batch on the device (``data.adj_t`` must be the
    normalised adjacency; a ``DeviceGraph`` may be passed as ``data``)."""

    def __init__(self, data, cluster_indices, batch_size, gnn_type='GCN', sampler_type='node',
                 walk_length=None, recovery_flag=True, train_flag=True, cont_sliding_window=1,
                 device="cuda", **kwargs):
        if sampler_type not in ('node', 'cluster', 'edge', 'rw', 'cont'):
            raise ValueError('Sampler type not supported!')
        if kwargs.get("num_workers", 0):
            raise ValueError("the collate runs HIP kernels: num_workers must be 0")
        self.sampler_type, self.gnn_type = sampler_type, gnn_type
        self.recovery_flag = True            # dataloader.py:16: always on
        self.walk_length, self.train_flag = walk_length, train_flag
        self.cont_sliding_window = cont_sliding_window
        if isinstance(data, DeviceGraph):
            self.graph = data
        else:
            self.graph = DeviceGraph.from_adj(data.adj_t, data.num_nodes, device)
        self.N = self.graph.N
        self.batch_size = batch_size
        if sampler_type == 'cluster':
            super().__init__(cluster_indices, collate_fn=self.__collate_cluster__,
                             batch_size=batch_size, **kwargs)
        else:
            # dataloader.py:40-46: seeds per batch so that the sampled batch
            # holds about batch_size nodes
            if sampler_type == 'edge':
                self.batch_size = batch_size // 2
            elif sampler_type == 'rw':
                self.batch_size = batch_size // (self.walk_length + 1)
            elif sampler_type == 'cont':
                self.batch_size = batch_size // self.cont_sliding_window
            super().__init__(range(self.N), collate_fn=self.__collate__,
                             batch_size=self.batch_size, **kwargs)

    def __collate_cluster__(self, batches):
        idx = torch.cat([torch.as_tensor(b) for b in batches], dim=0)
        return [(self._k_hop_subgraph(idx), idx)]

    def _walk(self, start, walk_length):
        """SparseTensor.random_walk(start, walk_length) on the device graph;
        the seed is drawn from torch's default CPU generator (torch.manual_seed
        makes a run reproducible, as torch.rand does for torch_cluster)."""
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        return kernels.random_walk(self.graph.rowptr, self.graph.col, self.N, start, walk_length,
                                   seed)

    def __collate__(self, idx):
        """dataloader.py:60-95: the sampler's node lists, then one
        (_k_hop_subgraph, node_idx) per list."""
        idx = torch.tensor(idx)
        dev = self.graph.device
        if self.sampler_type == 'node':
            node_idx_list = [idx]
        elif self.sampler_type == 'edge':                       # :70-71
            node_idx_list = [self._walk(idx, 1).view(-1).unique()]
        elif self.sampler_type == 'rw':                         # :73-74
            node_idx_list = [self._walk(idx, self.walk_length).view(-1).unique()]
        else:                                                   # 'cont', :76-88
            node_idx = idx.to(dev)
            node_idx_list = [node_idx]
            for _ in range(self.walk_length):
                node_idx = torch.cat([node_idx] * 3)
                node_idx = self._walk(node_idx, 1)[:, 1].unique()[:self.batch_size]
                node_idx_list.append(node_idx)
            if self.cont_sliding_window > 1:
                w = self.cont_sliding_window
                node_idx_list = [torch.cat(node_idx_list[i:i + w]).unique()
                                 for i in range(len(node_idx_list) - w + 1)]
        return [(self._k_hop_subgraph(n), n) for n in node_idx_list]

    def _k_hop_subgraph(self, node_idx, num_hops=1, relabel_nodes=True):
        if not relabel_nodes:
            raise NotImplementedError("relabel_nodes=False")
        return SubgraphBatch(self.graph, node_idx, num_hops, self.train_flag)


__all__ = ["DeviceGraph", "SubgraphBatch", "OurDataLoader", "prepare_batch_input"]


def mapper(batch, c, num_M, gnn_type, device=None):
    """VQ-GNN v1 ``mapper`` (vq_gnn_v1/utils/dataloader.py:144-192) on the
    device: ``batch = (deg_inv, A_BN, A_BB, A_NB_v, batch_idx)`` as the v1
    collate returns it (A_BN / A_BB as (row, col, value) COO triples, A_BB
    and A_NB_v may be None); ``c`` the branch's codes (int16 ``c_indices``).
    Returns the (B+M) x (B+M) adjacency as a ``CSR`` (torch_sparse
    ``SparseTensor`` surface), GCN symmetrised, as the reference does."""
    deg_inv, A_BN, A_BB, A_NB_v, batch_idx = batch
    B = int(batch_idx.shape[0])
    rowptr, col, val = kernels.mapper(A_BN, c, B, num_M, gnn_type, nb_val=A_NB_v, bb=A_BB,
                                      batch_idx=batch_idx, deg_inv=deg_inv)
    dim = B + int(num_M)
    return CSR(rowptr, col, val, (dim, dim))
