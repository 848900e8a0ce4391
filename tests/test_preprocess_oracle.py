"""CPU known answers for the preprocessing oracle (oracle/preprocess_ref.py:
norm_adj / to_symmetric / permute of vq_gnn_v2/utils/misc.py), hand-computed."""
import numpy as np
import torch

from oracle import preprocess_ref as P


def _csr(N, entries):
    entries = sorted(entries)
    rowptr = np.zeros(N + 1, np.int64)
    for r, _, _ in entries:
        rowptr[r + 1] += 1
    rowptr = np.cumsum(rowptr)
    col = np.array([c for _, c, _ in entries], np.int64)
    val = np.array([v for _, _, v in entries], np.float32)
    return rowptr, col, val


def test_norm_adj_gcn_known_answer():
    # path 0-1-2 (pattern), plus an existing diagonal at node 2 of value 5
    rp, cl, vl = _csr(3, [(0, 1, 1.), (1, 0, 1.), (1, 2, 1.), (2, 1, 1.), (2, 2, 5.)])
    rowptr, col, val = P.norm_adj(rp, cl, vl, 3, "GCN")
    assert rowptr.tolist() == [0, 2, 5, 7]
    assert col.tolist() == [0, 1, 0, 1, 2, 1, 2]
    f = np.float32
    dis = np.array([f(1) / np.sqrt(f(2)), f(1) / np.sqrt(f(3)), f(1) / np.sqrt(f(2))], np.float32)
    exp = [dis[0] * dis[0], dis[0] * dis[1], dis[1] * dis[0], dis[1] * dis[1], dis[1] * dis[2],
           dis[2] * dis[1], dis[2] * dis[2]]          # set_diag replaced the 5 by 1
    assert np.array_equal(val, np.array(exp, np.float32))


def test_norm_adj_sage_gat_known_answer():
    rp, cl, vl = _csr(3, [(0, 1, 2.), (0, 2, 1.), (1, 0, 4.)])
    _, col, val = P.norm_adj(rp, cl, vl, 3, "SAGE")       # no self loops, D^-1 A
    assert col.tolist() == [1, 2, 0]
    assert np.array_equal(val, np.array([2 / 3, 1 / 3, 1.0], np.float32))
    rowptr, col, val = P.norm_adj(rp, cl, None, 3, "GAT")  # self loops, D^-1 (A + I)
    assert rowptr.tolist() == [0, 3, 5, 6] and col.tolist() == [0, 1, 2, 0, 1, 2]
    assert np.array_equal(val, np.array([1 / 3] * 3 + [0.5, 0.5, 1.0], np.float32))


def test_rsqrt_of_torch_within_two_ulp():
    """The reference's deg.pow(-1/2) vs the IEEE 1/sqrt the device computes."""
    x = torch.arange(1, 200000, dtype=torch.float32)
    a = x.pow(-1 / 2).view(torch.int32)
    b = (1 / torch.sqrt(x)).view(torch.int32)
    assert int((a - b).abs().max()) <= 2


def test_to_symmetric_and_permute_known_answer():
    rp, cl, vl = _csr(3, [(0, 1, 1.5), (1, 2, 2.), (2, 1, 0.25)])
    rowptr, col, val = P.to_symmetric(rp, cl, vl, 3)
    assert rowptr.tolist() == [0, 1, 3, 4]
    assert col.tolist() == [1, 0, 2, 1]
    assert val.tolist() == [1.5, 1.5, 2.25, 2.25]
    _, _, vp = P.to_symmetric(rp, cl, None, 3)            # pattern: no sums
    assert vp.tolist() == [1, 1, 1, 1]
    # permute: new node i = old node perm[i]
    rowptr, col, val = P.permute(rp, cl, vl, 3, [2, 0, 1])
    # old (0,1)->(1,2); old (1,2)->(2,0); old (2,1)->(0,2)
    assert rowptr.tolist() == [0, 1, 2, 3] and col.tolist() == [2, 2, 0]
    assert val.tolist() == [0.25, 1.5, 2.0]
