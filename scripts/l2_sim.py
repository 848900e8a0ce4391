"""LRU L2 model of the SpMM gather stream on the arxiv batch (CPU only).
Writes the batch CSR for scripts/probes/l2_lru_sim.c, builds it with gcc and
prints the modelled L2 hit rate and miss bytes for CSR order and for
length-sorted 2048-row windows.  Usage: python scripts/l2_sim.py"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd import graph  # noqa: E402

os.makedirs("/tmp/sim", exist_ok=True)
_, _, b = graph.make_batch(graph.CONFIGS["arxiv_gcn"])
b.rowptr.astype(np.int64).tofile("/tmp/sim/rp.bin")
b.col.astype(np.int32).tofile("/tmp/sim/col.bin")
exe = "/tmp/sim/l2_lru_sim"
subprocess.check_call(["gcc", "-O2", "-o", exe, os.path.join(ROOT, "scripts/probes/l2_lru_sim.c")])
for win, conc in ((0, 2048), (2048, 2048), (1 << 20, 2048), (2048, 512)):
    subprocess.check_call([exe, str(b.n), str(b.nnz), str(b.B), str(win), str(conc)])
