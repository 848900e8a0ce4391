"""Data-parallel VQ update on the GPU: 2 ranks (one GPU, gloo) with
CodebookSync vs one process on the union batch (multi-GPU
parity is checked against the single-GPU result on the concatenated batch)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_match_union_batch(tmp_path):
    env = dict(os.environ)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_gpu_worker.py"), str(tmp_path)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, timeout=300, capture_output=True, text=True)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    r0, r1 = (np.load(tmp_path / f"r{k}.npz") for k in range(2))
    # replicas are bit-identical (identical finalize on exact int64 statistics)
    for k in ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g", "codes"):
        np.testing.assert_array_equal(r0[k], r1[k])
    # and equal the single-process union batch: codes (tie-aware), state
    mism = int((r0["codes"] != r0["ref_codes"]).sum())
    assert mism <= 2, f"{mism} code mismatches vs the union batch"
    for k in ("rm_f", "rv_f", "rm_g", "rv_g"):
        np.testing.assert_allclose(r0[k], r0["ref_" + k], rtol=1e-6, atol=1e-7)
    for k in ("emb", "emb_out", "ema_w", "cs"):
        np.testing.assert_allclose(r0[k], r0["ref_" + k], rtol=1e-5, atol=1e-6)
    # repeated nodes across ranks: identical replicas, the last rank's codes
    np.testing.assert_array_equal(r0["dup_codes"], r1["dup_codes"])
    M, nb = 64, 6
    last = (np.arange(10)[:, None] + 7 * 2 + np.arange(nb)[None]) % M
    np.testing.assert_array_equal(r0["dup_codes"][:10], last)
    for rk in range(2):
        own = (np.arange(10, 20)[:, None] + 7 * (rk + 1) + np.arange(nb)[None]) % M
        np.testing.assert_array_equal(r0["dup_codes"][100 + 10 * rk:110 + 10 * rk], own)
