"""Data-parallel VQ update on the GPU: 2 ranks (one GPU, gloo) with
CodebookSync vs one process on the union batch (multi-GPU
parity is checked against the single-GPU result on the concatenated batch)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from helpers import tie_aware_mismatch

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
    # and equal the single-process union batch: codes bit-exact except rows
    # within 1e-5 of a tie under the fp64 distances (the multi-rank BN sums
    # are added in another order, so a coefficient may move by an ulp)
    node = r0["node"]
    other = np.setdiff1d(np.arange(r0["codes"].shape[0]), node)
    np.testing.assert_array_equal(r0["codes"][other], r0["ref_codes"][other])
    n_mis = n_bad = 0
    for b in range(r0["codes"].shape[1]):
        m, bad = tie_aware_mismatch(torch.from_numpy(r0["codes"][node, b].astype(np.int64)),
                                    torch.from_numpy(r0["ref_codes"][node, b].astype(np.int64)),
                                    torch.from_numpy(r0["ref_dist"][b]))
        n_mis, n_bad = n_mis + m, n_bad + bad
    assert n_bad == 0, f"{n_bad} of {n_mis} code mismatches are not near-ties"
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
    # two in-flight exchanges on shared wire buffers keep their own records
    for r in (r0, r1):
        ids = np.arange(24)
        loc = (ids // 2)[:, None] + np.arange(nb)[None]
        np.testing.assert_array_equal(r["two_a"], loc % M)
        np.testing.assert_array_equal(r["two_b"], (loc % M + 5) % M)
    # staleness contract over three deferred updates
    rs = (r0, r1)
    sets = [[r0[f"set_{r}_{k}"] for k in range(3)] for r in range(2)]
    own = [[rs[r][f"stale_{k}"][sets[r][k]] for k in range(3)] for r in range(2)]
    codes0 = r0["stale_codes0"]
    for r in range(2):
        o = 1 - r
        for k in range(3):
            snap = rs[r][f"stale_{k}"]
            # the other rank's step-k rows: not landed yet (their old codes)
            np.testing.assert_array_equal(snap[sets[o][k]], codes0[sets[o][k]])
            # the other rank's step-(k-1) rows: landed, exactly its codes
            if k > 0:
                np.testing.assert_array_equal(snap[sets[o][k - 1]], own[o][k - 1])
            # own rows of every earlier step are still the own codes
            for kk in range(k):
                np.testing.assert_array_equal(snap[sets[r][kk]], own[r][kk])
    np.testing.assert_array_equal(r0["stale_final"], r1["stale_final"])
    # the overlapped step's landing: the same codes after every step, and the
    # side stream saw the serial aggregation's codes on every node outside the
    # rank's own step-k batch (the nodes an aggregation reads from codes)
    for r in range(2):
        for k in range(3):
            np.testing.assert_array_equal(rs[r][f"ostale_{k}"], rs[r][f"stale_{k}"],
                                          err_msg=f"rank {r} step {k}")
            outside = np.setdiff1d(np.arange(codes0.shape[0]), sets[r][k])
            np.testing.assert_array_equal(rs[r][f"oseen_{k}"][outside],
                                          rs[r][f"stale_{k}"][outside],
                                          err_msg=f"rank {r} step {k} (walk's view)")
    for r in range(2):
        for k in range(3):
            np.testing.assert_array_equal(r0["stale_final"][sets[r][k]], own[r][k])
    # over capacity: no hang, both ranks raise, the statistics stayed inside
    # the fixed-point bound (finite state) and the replicas agree
    for tag in ("over500", "over700"):
        assert int(r0[f"{tag}_raised"]) == 1 and int(r1[f"{tag}_raised"]) == 1, tag
        # codes too: rows past the capacity are scattered nowhere, so the
        # replicas keep identical c_indices (vq.py _exchange_codes)
        for k in ("emb", "emb_out", "ema_w", "cs", "codes"):
            np.testing.assert_array_equal(r0[f"{tag}_{k}"], r1[f"{tag}_{k}"], err_msg=tag + k)
        for k in ("emb_out", "ema_w", "cs"):
            assert np.isfinite(r0[f"{tag}_{k}"]).all(), tag + k
        assert np.abs(r0[f"{tag}_ema_w"]).max() < 1e3, tag   # no saturated fixed point


def test_rccl_world1_deferred_update(tmp_path):
    """The RCCL path itself (one GPU per box: a world of one): asynchronous
    EMA all-reduce + code all_gather with work queued behind them give the
    same state, bit for bit, as the single-process bank -- with a capacity
    (no host collective) and without one."""
    env = dict(os.environ)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_nccl_worker.py"), str(tmp_path)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, timeout=300, capture_output=True, text=True)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    r = np.load(tmp_path / "nccl.npz")
    for tag in ("cap", "nocap"):
        for k in ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g", "codes"):
            np.testing.assert_array_equal(r[f"{tag}_{k}"], r["ref_" + k], err_msg=f"{tag} {k}")
    # capacity 4x the batch: the BatchNorm state is exact, the EMA state within
    # the fixed-point grid's rounding, codes equal but for rare near-ties
    for k in ("rm_f", "rv_f", "rm_g", "rv_g"):
        np.testing.assert_array_equal(r[f"cap4x_{k}"], r["ref_" + k], err_msg=k)
    for k in ("emb", "emb_out", "ema_w", "cs"):
        np.testing.assert_allclose(r[f"cap4x_{k}"], r["ref_" + k], rtol=1e-5, atol=1e-6,
                                   err_msg=k)
    assert (r["cap4x_codes"] != r["ref_codes"]).mean() <= 1e-3


def _wire_round(kernels, dev, rng, N, nb, M, max_B, world, node_pool, ref, codes_own):
    rec = kernels.codes_wire_record(nb, M)
    recv = torch.zeros(world * max_B * rec, dtype=torch.uint8, device=dev)
    for rk in range(world):
        B = max_B - 100 * (rk % 2)
        ids = rng.choice(node_pool, size=B, replace=False)     # ranks overlap in the pool
        loc = rng.integers(0, M, size=(B, nb))
        send = torch.empty(max_B * rec, dtype=torch.uint8, device=dev)
        kernels.pack_codes(torch.from_numpy(ids).to(dev), torch.from_numpy(loc).to(torch.int16).to(dev),
                           M, max_B, send, codes=codes_own)
        recv[rk * max_B * rec:(rk + 1) * max_B * rec] = send
        ref[ids] = loc                                      # later ranks overwrite
    return recv


@pytest.mark.parametrize("nb,M", [(32, 256), (8, 200), (6, 64), (16, 1024), (40, 256), (24, 256)])
def test_wire_pack_scatter_last_record_wins(nb, M):
    """The packed code exchange without RCCL: three 'ranks' pack their rows
    (own codes scattered at once), the records are concatenated in rank order
    (what all_gather_into_tensor delivers) and scattered: every node takes the
    codes of its LAST record, and the 8-codes-per-thread kernels (uint8 wire,
    8 | nb) agree with the one-thread-per-record ones.  Three exchanges on one
    stamp table (epochs 1, 2, 3): later exchanges always win."""
    from vq_gnn_amd import kernels
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(nb * 7 + M)
    N, max_B, world = 5000, 700, 3
    ref = np.zeros((N, nb), np.int64)
    codes_own = torch.zeros(N, nb, dtype=torch.int16, device=dev)
    winner = torch.zeros(N, dtype=torch.int64, device=dev)
    codes = torch.zeros(N, nb, dtype=torch.int16, device=dev)
    for epoch in (1, 2, 3):
        recv = _wire_round(kernels, dev, rng, N, nb, M, max_B, world, np.arange(2000), ref,
                           codes_own)
        kernels.scatter_wire(recv, world * max_B, nb, M, winner, codes, epoch)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(codes.cpu().numpy(), ref, err_msg=f"epoch {epoch}")
        # own-codes scatter of the pack: the last packing rank's codes for shared nodes
        np.testing.assert_array_equal(codes_own.cpu().numpy(), ref)


@pytest.mark.parametrize("nb", [40, 24, 32])
def test_wire_scatter_many_records(nb):
    """Far more records than the GPU holds resident at once (8 ranks x 131,072
    rows, ~10^6 records, nodes repeated across ranks), with a record's
    8-code chunks straddling waves (nb / 8 does not divide 64 for nb = 40 and
    24): every node still takes exactly its last record's codes."""
    from vq_gnn_amd import kernels
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(nb)
    N, max_B, world, M = 400_000, 131_072, 8, 256
    ref = np.zeros((N, nb), np.int64)
    codes_own = torch.zeros(N, nb, dtype=torch.int16, device=dev)
    winner = torch.zeros(N, dtype=torch.int64, device=dev)
    codes = torch.zeros(N, nb, dtype=torch.int16, device=dev)
    recv = _wire_round(kernels, dev, rng, N, nb, M, max_B, world, np.arange(300_000), ref,
                       codes_own)
    kernels.scatter_wire(recv, world * max_B, nb, M, winner, codes, 1)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(codes.cpu().numpy(), ref)
