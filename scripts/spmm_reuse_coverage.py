"""Source-row reuse available to an on-chip SpMM tiling of the arxiv bench
batch (CPU, numpy): the rows are cut into row-aligned tiles
of about Et edges, and each tile's C most referenced source rows (used at
least twice) are counted as 'hot' -- the share of the edges that could read
their source row from LDS, the uses per staged row and the staged bytes.
Usage: python scripts/spmm_reuse_coverage.py [row_bytes]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd.graph import CONFIGS, make_batch  # noqa: E402


def coverage(rowptr, col, Et, C):
    n, nnz = rowptr.size - 1, col.size
    cov = staged = tiles = 0
    r = 0
    while r < n:
        e0 = rowptr[r]
        r1 = min(max(int(np.searchsorted(rowptr, e0 + Et, side="left")), r + 1), n)
        _, cnt = np.unique(col[e0:rowptr[r1]], return_counts=True)
        top = np.sort(cnt[cnt >= 2])[::-1][:C]
        cov += int(top.sum())
        staged += top.size
        tiles += 1
        r = r1
    return tiles, cov / nnz, cov / max(staged, 1), staged


if __name__ == "__main__":
    row_bytes = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    _, _, b = make_batch(CONFIGS["arxiv_gcn"])
    print(f"arxiv_gcn batch: n={b.n} nnz={b.nnz}; staged slices of {row_bytes} B")
    for Et in (2048, 4096, 8192, 16384):
        for C in (128, 256, 512, 1024):
            t, cv, uses, st = coverage(b.rowptr, b.col, Et, C)
            print(f"  Et={Et:6d} C={C:5d} tiles={t:4d} hot edges {cv:.3f} "
                  f"uses/row {uses:5.1f} staged {st * row_bytes / 1e6:6.1f} MB")
