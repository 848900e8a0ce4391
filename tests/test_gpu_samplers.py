"""Random-walk samplers on the device (dataloader.py:70-90; include/vqgnn.h
§9b): the HIP walk is bit-identical to oracle/subgraph_ref.random_walk on the
kernel's own step uniforms (torch_cluster's uniform step; the RNG stream is
ours, parity unpinned for the draws), picks neighbours uniformly, and the
'edge' / 'rw' / 'cont' loaders produce the reference's node-list structure,
each batch the exact k-hop batch of its node list."""
import numpy as np
import pytest
import torch

from oracle import subgraph_ref
from vq_gnn_amd import graph, kernels
from vq_gnn_amd.loader import DeviceGraph, OurDataLoader

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _graph_with_sinks(N=3000, seed=5):
    g = graph.synthetic_graph(N, 6, 12000, seed=seed)
    rp, cl, vl = graph.norm_adj(g, "SAGE")      # no self loops: isolated nodes stay sinks
    # make nodes 10..19 sinks (drop their rows' edges)
    row = np.repeat(np.arange(N), np.diff(rp))
    keep = (row < 10) | (row >= 20)
    row, cl, vl = row[keep], cl[keep], vl[keep]
    rp = np.zeros(N + 1, np.int64)
    rp[1:] = np.cumsum(np.bincount(row, minlength=N))
    return rp, cl, vl, N


def test_random_walk_matches_oracle():
    rp, cl, vl, N = _graph_with_sinks()
    dg = DeviceGraph(rp, cl, vl, N, DEV)
    gen = torch.Generator().manual_seed(0)
    start = torch.cat([torch.randint(0, N, (700,), generator=gen), torch.arange(8, 24)])
    for seed, L in ((987654321, 4), (3, 1), (2 ** 62 + 17, 7)):
        out = kernels.random_walk(dg.rowptr, dg.col, N, start, L, seed).cpu().numpy()
        u = subgraph_ref.walk_uniforms(seed, start.numel(), L)
        ref = subgraph_ref.random_walk(rp, cl, start.numpy(), L, u)
        np.testing.assert_array_equal(out, ref)
    # sinks stay put; walk_length 0 returns the starts
    out = kernels.random_walk(dg.rowptr, dg.col, N, torch.arange(10, 20), 3, 1).cpu()
    assert torch.equal(out, torch.arange(10, 20)[:, None].expand(10, 4))
    assert torch.equal(kernels.random_walk(dg.rowptr, dg.col, N, start, 0, 1).cpu()[:, 0], start)
    with pytest.raises(IndexError):
        kernels.random_walk(dg.rowptr, dg.col, N, torch.tensor([N]), 2, 1)


def test_random_walk_uniform_choice():
    """From a node with k neighbours, one step lands on each about n/k times."""
    rp, cl, vl, N = _graph_with_sinks()
    dg = DeviceGraph(rp, cl, vl, N, DEV)
    deg = np.diff(rp)
    hub = int(np.argmax(deg))
    k = int(deg[hub])
    n = 4000 * k
    out = kernels.random_walk(dg.rowptr, dg.col, N, torch.full((n,), hub), 1, 42).cpu().numpy()
    counts = np.bincount(out[:, 1], minlength=N)[cl[rp[hub]:rp[hub + 1]]]
    assert counts.sum() == n
    assert np.abs(counts - 4000).max() < 5 * np.sqrt(4000)     # ~5 sigma


def _neighbours(rp, cl, v):
    return set(cl[rp[v]:rp[v + 1]].tolist()) or {v}


def _check_batch(batch, rp, cl, vl, N):
    sub, node_idx = batch
    subset = torch.as_tensor(sub[0]).cpu()
    ref_subset, _, _ = subgraph_ref.k_hop_subgraph(rp, cl, vl, N, node_idx.cpu())
    assert torch.equal(subset, ref_subset)


@pytest.mark.parametrize("sampler,walk_length,window", [("edge", None, 1), ("rw", 3, 1),
                                                         ("cont", 2, 1), ("cont", 3, 2)])
def test_random_walk_samplers(sampler, walk_length, window):
    rp, cl, vl, N = _graph_with_sinks(seed=9)
    dg = DeviceGraph(rp, cl, vl, N, DEV)
    torch.manual_seed(1)
    loader = OurDataLoader(dg, None, batch_size=600, sampler_type=sampler,
                           walk_length=walk_length, cont_sliding_window=window, shuffle=True)
    expect_seeds = {"edge": 300, "rw": 150, "cont": 600 // window}[sampler]
    assert loader.batch_size == expect_seeds
    batches = next(iter(loader))
    if sampler != "cont":
        assert len(batches) == 1
        node_idx = batches[0][1].cpu()
        assert torch.equal(node_idx, torch.unique(node_idx))          # sorted, unique
        _check_batch(batches[0], rp, cl, vl, N)
    else:
        lists = [b[1].cpu() for b in batches]
        assert len(lists) == walk_length + 1 - (window - 1)
        if window == 1:
            assert lists[0].numel() == expect_seeds
            for a, b in zip(lists, lists[1:]):
                assert b.numel() <= loader.batch_size
                assert torch.equal(b, torch.unique(b))
                reach = set()
                for v in a.tolist():
                    reach |= _neighbours(rp, cl, v)
                assert set(b.tolist()) <= reach
        for bt in batches:
            _check_batch(bt, rp, cl, vl, N)
