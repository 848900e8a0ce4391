"""Multi-process host logic of the data-parallel path (vq-gnn_amd/dist.py) on
CPU: world_size 2 over gloo, rendezvous on 127.0.0.1."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import vqgnn_pkg
    vqgnn_pkg.load()
    from vq_gnn_amd.dist import CodebookSync
    sync = CodebookSync(count_group=dist.new_group(backend="gloo"))
    B = [5, 3][rank]
    res = {}
    res["count"] = sync.global_count(B)
    res["max"] = sync.global_max(B)
    # per-rank batch sizes that change between calls: without a capacity,
    # every call agrees on this call's max(B)
    res["max_seq"] = np.array([sync.rows_per_rank(b) for b in ([5, 2, 9], [3, 7, 1])[rank]])
    # the update path's BatchNorm all-reduce carries the row count: [4F + 2]
    # fp64 sums with B at 4F and the over-capacity flag last
    # (bn_stats(with_count=True))
    for b in ([5, 2, 9], [3, 7, 1])[rank]:
        flat = torch.zeros(4 * 2 + 2, dtype=torch.float64)
        flat[:8] = torch.arange(8, dtype=torch.float64) * (rank + 1)
        flat[8] = b
        sync.allreduce_stats_(flat, b)
        res.setdefault("counts_seq", []).append(float(flat[8]))
    res["counts_seq"] = np.array(res["counts_seq"])
    # with a capacity the update path issues no host-side collective
    capped = CodebookSync(count_group=sync.count_group, capacity=9)
    real = dist.all_reduce

    def no_host_collective(t, *a, **k):
        if t.dtype == torch.int64 and t.numel() == 1:
            raise AssertionError("host collective on the capped update path")
        return real(t, *a, **k)

    dist.all_reduce = no_host_collective
    try:
        flat = torch.zeros(10, dtype=torch.float64)
        flat[8] = B
        res["capped_bound"] = capped.allreduce_stats_(flat, B)
        res["capped_count"] = float(flat[8])
        res["over_none"] = int(capped.take_overflow())
        try:
            capped.rows_per_rank(10)
            res["over"] = 0
        except ValueError:
            res["over"] = 1
        # one rank over capacity: no raise inside the collective (the other
        # rank would hang in it); both ranks see the flag afterwards
        flat = torch.zeros(10, dtype=torch.float64)
        b_over = [12, 4][rank]
        flat[8] = b_over
        res["over_bound"] = capped.allreduce_stats_(flat, b_over)
        res["over_flag"] = int(capped.take_overflow())
        res["over_flag_after"] = int(capped.take_overflow())
    finally:
        dist.all_reduce = real
    # BN sums (fp64) and EMA statistic (int64) all-reduce
    sums = torch.arange(8, dtype=torch.float64).view(4, 2) * (rank + 1)
    sync.allreduce_(sums)
    res["sums"] = sums.numpy()
    st = torch.full((1, 2, 3, 5), rank + 1, dtype=torch.int64)
    st[0, 1, 2, 4] = (1 << 40) * (rank + 1)           # large fixed-point values stay exact
    sync.allreduce_(st)
    res["stats"] = st.numpy()
    # codes: rank r owns nodes {r, r+2, ...}
    idx = torch.arange(rank, 2 * B, 2, dtype=torch.int64)[:B]
    loc = (idx[:, None] * 10 + torch.arange(3)[None]).to(torch.int16)
    _, all_idx, all_loc = sync.gather_codes(idx, loc, M=64)
    res["all_idx"] = all_idx.numpy()
    res["all_loc"] = all_loc.numpy()
    # int16 wire format (M > 256) and the async form
    pend, ai2, al2 = sync.gather_codes(idx, loc * 7, M=4096, async_op=True)
    for w in pend:
        w.wait()
    res["all_loc16"] = al2.numpy()
    res["all_idx16"] = ai2.numpy()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def test_codebook_sync_gloo_world2(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(2)]
    for k in range(2):
        assert int(r[k]["count"]) == 8 and int(r[k]["max"]) == 5
        np.testing.assert_array_equal(r[k]["max_seq"], [5, 7, 9])
        np.testing.assert_array_equal(r[k]["counts_seq"], [8.0, 9.0, 10.0])
        assert int(r[k]["capped_bound"]) == 9 and float(r[k]["capped_count"]) == 8.0
        assert int(r[k]["over"]) == 1 and int(r[k]["over_none"]) == 0
        assert int(r[k]["over_bound"]) == 9
        assert int(r[k]["over_flag"]) == 1 and int(r[k]["over_flag_after"]) == 0
        np.testing.assert_array_equal(r[k]["sums"], np.arange(8).reshape(4, 2) * 3.0)
        st = r[k]["stats"]
        assert st[0, 0, 0, 0] == 3 and st[0, 1, 2, 4] == 3 * (1 << 40)
        # padded union of (batch_idx, codes), rank-major
        idx, loc = r[k]["all_idx"], r[k]["all_loc"]
        assert idx.shape == (10,) and loc.shape == (10, 3)
        np.testing.assert_array_equal(idx[:5], [0, 2, 4, 6, 8])
        np.testing.assert_array_equal(idx[5:], [1, 3, 5, -1, -1])
        valid = idx >= 0
        np.testing.assert_array_equal(loc[valid], idx[valid, None] * 10 + np.arange(3))
        assert loc.dtype == np.uint8 and r[k]["all_loc16"].dtype == np.int16
        l16 = r[k]["all_loc16"]
        np.testing.assert_array_equal(l16[valid], (idx[valid, None] * 10 + np.arange(3)) * 7)
        np.testing.assert_array_equal(r[k]["all_idx16"], idx)
    # every rank sees the same gathered codes (replicas stay identical)
    np.testing.assert_array_equal(r[0]["all_loc"], r[1]["all_loc"])


def test_rccl_binding_unique_id_and_dtypes():
    """vq-gnn_amd/rccl.py binds torch's own librccl: a unique id is the full
    128 bytes (no NUL truncation), and only the exchange's dtypes map."""
    from vq_gnn_amd import rccl
    try:
        u = rccl.unique_id()
    except OSError as e:          # no RCCL in this torch build
        pytest.skip(f"librccl not loadable: {e}")
    assert isinstance(u, bytes) and len(u) == rccl.NCCL_UNIQUE_ID_BYTES
    assert rccl.unique_id() != u
    for dt in (torch.uint8, torch.int32, torch.int64, torch.float32, torch.float64):
        assert rccl.Communicator._dtype(torch.empty(1, dtype=dt)) >= 0
    with pytest.raises(TypeError):
        rccl.Communicator._dtype(torch.empty(1, dtype=torch.int16))
    with pytest.raises(ValueError):
        rccl.Communicator(1, 0, b"short")


def _gloo_direct_flag(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import vqgnn_pkg
    vqgnn_pkg.load()
    from vq_gnn_amd.dist import CodebookSync
    with open(os.path.join(out_dir, f"direct{rank}.txt"), "w") as f:
        f.write(str(int(CodebookSync()._direct)))
    dist.destroy_process_group()


def test_codebook_sync_direct_rccl_only_on_nccl(tmp_path):
    """The direct RCCL path is chosen only on the nccl backend: gloo groups
    (the CPU tests, the one-GPU rehearsals) keep torch.distributed."""
    mp.spawn(_gloo_direct_flag, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert [open(tmp_path / f"direct{r}.txt").read() for r in range(2)] == ["0", "0"]


def test_release_comms_aborts_unless_closed():
    """CodebookSync's finalizer destroys its communicators only
    after close() ran; any other release (an exception exit, sys.exit from a
    handler, a failing thread, collection) aborts them."""
    from vq_gnn_amd.dist import _release_comms

    class Fake:
        def __init__(self):
            self.calls = []

        def abort(self):
            self.calls.append("abort")

        def destroy(self):
            self.calls.append("destroy")

    a, b = Fake(), Fake()
    _release_comms(a, b, [False])
    assert a.calls == b.calls == ["abort"]
    a, b = Fake(), Fake()
    _release_comms(a, None, [True])
    assert a.calls == ["destroy"] and b.calls == []
