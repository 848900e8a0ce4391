"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot path (devnkong/VQ-GNN, vq_gnn_v2) used
as the parity checker by tests/, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of bench.py.  The product path (vq-gnn_amd/) never
imports anything from here; it runs only through the HIP library.

Pinning:
  * vq_ref.py (VectorQuantizerEMA.feature_update / update) is checked against
    golden vectors produced by importing the reference's own vq_gnn_v2/vq.py
    in the build container (tests/golden/make_golden.py) — pinned.
  * conv_ref.py (spmm_sum aggregation, GAT attention aggregation) follows
    convs.py + torch_sparse / torch_scatter semantics; the reference's conv
    modules are not importable (torch_geometric / torch_sparse / torch_scatter
    absent, no network) and ship no tests or fixtures, so these are pinned by
    hand-computed known-answer tests (tests/golden/kat_*.json) and an fp64
    cross-check — "parity pinned by KATs", not by reference outputs.
"""
