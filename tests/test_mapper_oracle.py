"""Known-answer tests of the v1 mapper restatement (oracle/mapper_ref.py,
vq_gnn_v1/utils/dataloader.py:144-192).  The reference ships no fixtures for
it; these answers are worked by hand from the reference code."""
import numpy as np

from oracle import mapper_ref

F32 = np.float32
# N = 5 nodes, batch = global [0, 3] (B = 2), M = 2 codewords
C = np.array([0, 1, 1, 0, 1])
BATCH = np.array([0, 3])
BN = (np.array([0, 0, 0, 1, 1]), np.array([1, 2, 3, 0, 4]),
      np.array([0.5, 0.25, 1.0, 0.2, 0.4], F32))
BB = (np.array([0, 1]), np.array([1, 0]), np.array([1.0, 0.2], F32))
DEG_INV = np.array([0.5, 0.25], F32)


def _dense(rowptr, col, val, dim):
    d = np.zeros((dim, dim), F32)
    for r in range(dim):
        for k in range(rowptr[r], rowptr[r + 1]):
            d[r, col[k]] += val[k]
    return d


def test_mapper_gcn_known_answer():
    rp, col, val = mapper_ref.mapper(*BN, C, 2, 2, "GCN", bb=BB, batch_idx=BATCH,
                                     deg_inv=DEG_INV)
    # coalesce: (0,2) = 1.0 - 1.0 and (1,2) = 0.2 - 0.2 cancel and are dropped;
    # (0,3) = 0.5 + 0.25; self loops; to_symmetric sums (r,c) with (c,r)
    assert rp.tolist() == [0, 3, 6, 6, 8]
    assert col.tolist() == [0, 1, 3, 0, 1, 3, 0, 1]
    exp = [F32(0.5) + F32(0.5), F32(1.0) + F32(0.2), F32(0.5) + F32(0.25),
           F32(0.2) + F32(1.0), F32(0.25) + F32(0.25), F32(0.4),
           F32(0.5) + F32(0.25), F32(0.4)]
    assert np.array_equal(val, np.array(exp, F32))


def test_mapper_sage_no_loops_no_symmetric():
    rp, col, val = mapper_ref.mapper(*BN, C, 2, 2, "SAGE", bb=BB, batch_idx=BATCH)
    assert rp.tolist() == [0, 2, 4, 4, 4]
    assert col.tolist() == [1, 3, 0, 3]
    assert np.array_equal(val, np.array([1.0, F32(0.5) + F32(0.25), 0.2, 0.4], F32))


def test_mapper_with_a_nb_sign_cancel():
    nb = np.array([0.1, 0.2, 0.3, 0.4, 0.5], F32)
    rp, col, val = mapper_ref.mapper(*BN, C, 2, 2, "SAGE", nb_val=nb, bb=BB, batch_idx=BATCH)
    d = _dense(rp, col, val, 4)
    # codeword rows: (2,0) = 0.3 - 0.2 kept; (2,1) = 0.4 - 1.0 < 0 dropped;
    # (3,0) = 0.1 + 0.2; (3,1) = 0.5
    assert d[2, 0] == F32(0.3) + F32(-0.2)
    assert d[2, 1] == 0 and 1 not in col[rp[2]:rp[3]]
    assert d[3, 0] == F32(0.1) + F32(0.2)
    assert d[3, 1] == F32(0.5)
    assert rp[2] == 4 and rp[4] - rp[3] == 2


def test_mapper_gat_loops_without_symmetric_and_no_bb():
    rp, col, val = mapper_ref.mapper(*BN, C, 2, 2, "GAT", deg_inv=DEG_INV)
    # without A_BB nothing cancels: (0,2) = 1.0, (0,3) = 0.75, (1,2) = 0.2,
    # (1,3) = 0.4, then the self loops (not symmetrised)
    assert rp.tolist() == [0, 3, 6, 6, 6]
    assert col.tolist() == [0, 2, 3, 1, 2, 3]
    assert np.array_equal(val, np.array([0.5, 1.0, 0.75, 0.25, 0.2, 0.4], F32))


def test_mapper_repeated_keys_sum_in_order():
    # three entries on one key: ((0 + a) + b) + c in concatenation order
    a, b, c = F32(1e8), F32(1.0), F32(-1e8)
    rp, col, val = mapper_ref.mapper(np.array([0, 0, 0]), np.array([1, 2, 4]),
                                     np.array([a, b, c], F32), np.array([0, 1, 1, 0, 1]), 1, 2,
                                     "SAGE")
    s = F32(F32(F32(0) + a) + b) + c       # = 0 in fp32 -> dropped (not > 0)
    assert s == 0 and rp.tolist() == [0, 0, 0, 0]
