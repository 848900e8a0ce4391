"""GPU parity of vqgnn_mapper (include/vqgnn.h §11) with the v1 mapper
restatement (oracle/mapper_ref.py, vq_gnn_v1/utils/dataloader.py:144-192):
bit-exact structure and values (sequential sums in the same stable order)."""
import numpy as np
import pytest
import torch

from oracle import mapper_ref
from vq_gnn_amd import kernels, loader

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _case(seed, N=3000, B=400, M=64, deg=12):
    rng = np.random.default_rng(seed)
    batch_idx = np.sort(rng.choice(N, size=B, replace=False))
    pos = -np.ones(N, np.int64)
    pos[batch_idx] = np.arange(B)
    rows, cols = [], []
    for r in range(B):
        d = rng.integers(0, deg + 1)
        nb = np.sort(rng.choice(N, size=d, replace=False))
        rows.append(np.full(d, r))
        cols.append(nb)
    bn_row = np.concatenate(rows)
    bn_col = np.concatenate(cols)
    bn_val = rng.random(bn_row.size).astype(np.float32)
    inb = pos[bn_col] >= 0
    bb = (bn_row[inb], pos[bn_col[inb]], bn_val[inb])
    nb_val = (rng.random(bn_row.size) * 0.5).astype(np.float32)
    codes = rng.integers(0, M, size=N)
    deg_inv = (1.0 / (1 + rng.integers(1, 20, size=B))).astype(np.float32)
    return dict(bn=(bn_row, bn_col, bn_val), bb=bb, nb_val=nb_val, codes=codes,
                batch_idx=batch_idx, B=B, M=M, deg_inv=deg_inv)


def _codes_dev(codes, nb=3, branch=1):
    """Codes as one branch (column) of a node-major int16 [N, nb] c_indices."""
    full = np.zeros((codes.size, nb), np.int16)
    full[:, branch] = codes
    return torch.from_numpy(full).to(DEV)[:, branch]


@pytest.mark.parametrize("gnn_type,with_bb,with_nb", [
    ("GCN", True, False), ("GCN", False, False), ("SAGE", True, True), ("SAGE", False, True),
    ("GAT", True, True), ("GAT", True, False)])
@pytest.mark.parametrize("seed", [0, 1])
def test_mapper_matches_oracle(gnn_type, with_bb, with_nb, seed):
    k = _case(seed)
    bb = k["bb"] if with_bb else None
    nb = k["nb_val"] if with_nb else None
    rp, col, val = mapper_ref.mapper(*k["bn"], k["codes"], k["B"], k["M"], gnn_type, nb_val=nb,
                                     bb=bb, batch_idx=k["batch_idx"], deg_inv=k["deg_inv"])
    t = lambda a: torch.from_numpy(np.asarray(a)).to(DEV)
    g_rp, g_col, g_val = kernels.mapper(
        tuple(t(a) for a in k["bn"]), _codes_dev(k["codes"]), k["B"], k["M"], gnn_type,
        nb_val=t(nb) if nb is not None else None,
        bb=tuple(t(a) for a in bb) if bb is not None else None,
        batch_idx=t(k["batch_idx"]), deg_inv=t(k["deg_inv"]))
    assert np.array_equal(g_rp.cpu().numpy(), rp)
    assert np.array_equal(g_col.cpu().numpy(), col)
    assert np.array_equal(g_val.cpu().numpy(), val)


def test_mapper_loader_surface_and_heavy_repeats():
    """Few codewords -> long runs of repeated keys (sequential-sum order)."""
    k = _case(7, N=2000, B=300, M=3, deg=40)
    t = lambda a: torch.from_numpy(np.asarray(a)).to(DEV)
    batch = (t(k["deg_inv"]), tuple(t(a) for a in k["bn"]), tuple(t(a) for a in k["bb"]), None,
             t(k["batch_idx"]))
    adj = loader.mapper(batch, _codes_dev(k["codes"]), k["M"], "GCN")
    assert adj.sparse_sizes() == (k["B"] + k["M"],) * 2
    rp, col, val = mapper_ref.mapper(*k["bn"], k["codes"], k["B"], k["M"], "GCN", bb=k["bb"],
                                     batch_idx=k["batch_idx"], deg_inv=k["deg_inv"])
    assert np.array_equal(adj.rowptr.cpu().numpy(), rp)
    assert np.array_equal(adj.col.cpu().numpy(), col)
    assert np.array_equal(adj.value.cpu().numpy(), val)
    # symmetric pattern and values (to_symmetric)
    d = torch.zeros(adj.size(0), adj.size(0))
    r = np.repeat(np.arange(adj.size(0)), np.diff(rp))
    d[r, col] = torch.from_numpy(val)
    assert torch.equal(d, d.T)


def test_mapper_bad_code_raises():
    k = _case(2, N=500, B=50, M=8)
    codes = k["codes"].copy()
    codes[k["bn"][1][0]] = 99
    t = lambda a: torch.from_numpy(np.asarray(a)).to(DEV)
    with pytest.raises(ValueError, match="codeword"):
        kernels.mapper(tuple(t(a) for a in k["bn"]), _codes_dev(codes), k["B"], k["M"], "SAGE")


def test_mapper_empty():
    t = lambda a: torch.as_tensor(a).to(DEV)
    rp, col, val = kernels.mapper((t(np.zeros(0, np.int32)), t(np.zeros(0, np.int32)),
                                   t(np.zeros(0, np.float32))), _codes_dev(np.zeros(10, int)),
                                  4, 3, "GCN", deg_inv=t(np.full(4, 0.5, np.float32)))
    assert rp.cpu().tolist() == [0, 1, 2, 3, 4, 4, 4, 4]
    assert torch.equal(val.cpu(), torch.full((4,), 1.0))   # 0.5 + 0.5 (symmetrised loops)
