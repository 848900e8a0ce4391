"""GPU parity of the device mini-batch construction (include/vqgnn.h §9,
vq-gnn_amd/loader.py) against the oracle restatement of
vq_gnn_v2/dataloader.py:98-148 + utils/misc.py:73 (oracle/subgraph_ref.py) and
the numpy batch builder (vq-gnn_amd/graph.py).  Integer / index work: every
comparison is exact."""
import numpy as np
import pytest
import torch

from oracle import subgraph_ref
from vq_gnn_amd import graph, kernels
from vq_gnn_amd.loader import DeviceGraph, OurDataLoader, SubgraphBatch, prepare_batch_input

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _graph(N=6000, parts=8, edges=24000, conv="GCN", seed=2):
    g = graph.synthetic_graph(N, parts, edges, seed=seed)
    rp, cl, vl = graph.norm_adj(g, conv)
    return g, rp, cl, vl


def _eq(a, b):
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.array_equal(a, b)


def test_arxiv_shaped_batch_csr_exact():
    """Full-size arxiv-shaped cluster batch: subset and CSR bit-identical to the
    host builder (N = 169,343, ~2.3M directed edges, 40 of 80 clusters)."""
    cfg = graph.CONFIGS["arxiv_gcn"]
    g, (rp, cl, vl), b = graph.make_batch(cfg)
    dg = DeviceGraph(torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vl), g.N, DEV)
    bidx, subset, adj = dg.batch(torch.from_numpy(b.batch_idx))
    _eq(bidx, b.batch_idx)
    _eq(subset, b.subset)
    _eq(adj.rowptr, b.rowptr)
    _eq(adj.col, b.col)
    _eq(adj.value, b.val)
    assert adj.sparse_sizes() == (b.n, b.n)


@pytest.mark.parametrize("hops,train,sampler", [(1, True, "node"), (1, False, "node"),
                                                (2, True, "node"), (2, False, "cluster"),
                                                (1, True, "cluster")])
def test_k_hop_reference_order_vs_oracle(hops, train, sampler):
    g, rp, cl, vl = _graph()
    rng = np.random.default_rng(hops * 10 + train)
    if sampler == "node":
        node_idx = rng.permutation(g.N)[:700]                      # unsorted
    else:
        node_idx = graph.cluster_batch(g, rng.permutation(8)[:3])
    dg = DeviceGraph(torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vl), g.N, DEV)
    s, ei, w = dg.k_hop_subgraph(torch.from_numpy(node_idx), num_hops=hops, train_flag=train)
    s0, ei0, w0 = subgraph_ref.k_hop_subgraph(rp, cl, vl, g.N, node_idx, hops, train)
    _eq(s, s0)
    _eq(ei, ei0)
    _eq(w, w0)
    # the CSR form = SparseTensor(row, col, value) of the same edges
    _, subset, adj = dg.batch(torch.from_numpy(node_idx), hops, train)
    rp0, cl0, vl0 = subgraph_ref.sparse_tensor_csr(ei0[0], ei0[1], w0, s0.numel(), s0.numel())
    _eq(subset, s0)
    _eq(adj.rowptr, rp0.to(torch.int32))
    _eq(adj.col, cl0.to(torch.int32))
    _eq(adj.value, vl0)


def test_k_hop_edge_cases():
    g, rp, cl, vl = _graph(N=400, parts=2, edges=600)
    dg = DeviceGraph(torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vl), g.N, DEV)
    # repeated batch nodes: every copy in subset, relabelled to the last copy
    node_idx = np.array([5, 17, 5, 200, 17, 3])
    for train in (True, False):
        s, ei, w = dg.k_hop_subgraph(torch.from_numpy(node_idx), train_flag=train)
        s0, ei0, w0 = subgraph_ref.k_hop_subgraph(rp, cl, vl, g.N, node_idx, 1, train)
        _eq(s, s0)
        _eq(ei, ei0)
        _eq(w, w0)
        _, subset, adj = dg.batch(torch.from_numpy(node_idx), 1, train)
        rp0, cl0, vl0 = subgraph_ref.sparse_tensor_csr(ei0[0], ei0[1], w0, s0.numel(), s0.numel())
        _eq(adj.rowptr, rp0.to(torch.int32))
        _eq(adj.col, cl0.to(torch.int32))
        _eq(adj.value, vl0)
    # empty batch
    s, ei, w = dg.k_hop_subgraph(torch.zeros(0, dtype=torch.int64))
    assert s.numel() == 0 and tuple(ei.shape) == (2, 0) and w.numel() == 0
    _, subset, adj = dg.batch(torch.zeros(0, dtype=torch.int64))
    assert subset.numel() == 0 and adj.nnz() == 0 and adj.sparse_sizes() == (0, 0)
    # isolated node (no edges): a graph with an empty row
    rp2 = np.array([0, 1, 2, 2]), np.array([1, 0]), np.array([0.5, 0.25], np.float32)
    dg2 = DeviceGraph(torch.from_numpy(rp2[0]), torch.from_numpy(rp2[1]), torch.from_numpy(rp2[2]),
                      3, DEV)
    s, ei, w = dg2.k_hop_subgraph([2, 0])
    _eq(s, [2, 0, 1])
    _eq(ei, [[1, 2], [2, 1]])
    _eq(w, np.array([0.5, 0.25], np.float32))
    # node id outside the graph
    with pytest.raises(IndexError):
        dg.k_hop_subgraph(torch.tensor([1, g.N + 3]))
    with pytest.raises(IndexError):
        dg.batch(torch.tensor([-1, 2]))


def test_coo_to_csr_vs_sparse_tensor_order():
    rng = np.random.default_rng(0)
    n_rows, n_cols, nnz = 900, 1300, 20000
    row = rng.integers(0, n_rows, nnz)
    col = rng.integers(0, n_cols, nnz)
    row[:50], col[:50] = 7, 11                       # repeated (row, col) pairs
    val = rng.standard_normal(nnz).astype(np.float32)
    rp, cl, vl = kernels.coo_to_csr(torch.from_numpy(row).to(DEV), torch.from_numpy(col).to(DEV),
                                    torch.from_numpy(val).to(DEV), n_rows, n_cols)
    rp0, cl0, vl0 = subgraph_ref.sparse_tensor_csr(row, col, val, n_rows, n_cols)
    _eq(rp, rp0.to(torch.int32))
    _eq(cl, cl0.to(torch.int32))
    _eq(vl, vl0)
    # empty, and an index outside the matrix
    rp, cl, vl = kernels.coo_to_csr(torch.zeros(0, dtype=torch.int64, device=DEV),
                                    torch.zeros(0, dtype=torch.int64, device=DEV), None, 4, 4)
    _eq(rp, [0, 0, 0, 0, 0])
    with pytest.raises(IndexError):
        kernels.coo_to_csr(torch.tensor([0, 4], device=DEV), torch.tensor([0, 1], device=DEV),
                           None, 4, 4)


class _Data:
    def __init__(self, adj_t, num_nodes):
        self.adj_t, self.num_nodes = adj_t, num_nodes


class _AdjT:
    """torch_sparse-like adj_t: .csr() -> (rowptr, col, value)."""

    def __init__(self, rp, cl, vl):
        self._c = (torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vl))

    def csr(self):
        return self._c


@pytest.mark.parametrize("sampler", ["cluster", "node"])
def test_loader_and_prepare_batch_input(sampler):
    g, rp, cl, vl = _graph()
    data = _Data(_AdjT(rp, cl, vl), g.N)
    x = torch.randn(g.N, 16, device=DEV)
    if sampler == "cluster":
        clusters = [torch.arange(g.cluster_ptr[c], g.cluster_ptr[c + 1]) for c in range(8)]
        loader = OurDataLoader(data, clusters, batch_size=3, sampler_type="cluster",
                               shuffle=False)
    else:
        clusters = None
        loader = OurDataLoader(data, clusters, batch_size=1500, sampler_type="node",
                               shuffle=False)
    seen = 0
    for batches in loader:
        for batch in batches:
            sub, node_idx = batch
            assert isinstance(sub, SubgraphBatch)
            (x_B, (bidx, subset, adj)), (nB, nBp) = prepare_batch_input(x, batch, DEV)
            b = graph.k_hop_batch(rp, cl, vl, g.N, node_idx.numpy())
            _eq(subset, b.subset)
            _eq(adj.rowptr, b.rowptr)
            _eq(adj.col, b.col)
            _eq(adj.value, b.val)
            assert (nB, nBp) == (b.B, b.n - b.B)
            _eq(x_B, x[torch.from_numpy(b.batch_idx).to(DEV)])
            # the reference-form tuple through the COO -> CSR path gives the same CSR
            s, ei, w = sub[0], sub[1], sub[2]
            (_, (_, subset2, adj2)), _ = prepare_batch_input(x, ((s, ei, w), node_idx), DEV)
            _eq(subset2, subset)
            _eq(adj2.rowptr, adj.rowptr)
            _eq(adj2.col, adj.col)
            _eq(adj2.value, adj.value)
            seen += nB
    assert seen == g.N
