"""vq-gnn_amd — MI355X-native VQ-GNN per-layer hot path.

Drop-in for the reference's VectorQuantizerEMA (vq_gnn_v2/vq.py),
OurGCNConv / OurGATConv (vq_gnn_v2/convs.py) and LowRankGNNBlock /
LowRankGNNLayer / LowRankGNN (vq_gnn_v2/models.py), backed by hand-written
HIP kernels for gfx950 behind the C-ABI in include/vqgnn.h.

The directory name contains a hyphen, so it is imported as ``vq_gnn_amd``
through ``vqgnn_pkg.load()`` (repo root).
"""
__version__ = "0.1.0"
