"""Worker for tests/test_gpu_dist.py::test_rccl_world1_deferred_update
(torch.distributed.run, ONE rank, backend nccl = RCCL): the bench's multi-GPU
step order -- update(defer=True) with the asynchronous RCCL all-reduce of the
EMA statistics and the asynchronous all_gather of the codes, work queued
behind them, finish_update(), sync_codes() -- against a single-process bank
with the same (fp64) BatchNorm arithmetic.  Results -> <out>/nccl.npz."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_dir):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    import vqgnn_pkg
    vqgnn_pkg.load()
    from vq_gnn_amd import kernels
    from vq_gnn_amd.dist import CodebookSync
    from vq_gnn_amd.vq import VQBank
    nb, M, D, N, B = 8, 128, 4, 5000, 2500
    F = nb * D
    gen = torch.Generator().manual_seed(21)
    X = torch.randn(B, F, generator=gen).to(dev)
    G = (torch.randn(B, F, generator=gen) * 1e-3).to(dev)
    node = torch.randperm(N, generator=gen)[:B].to(dev)
    codes0 = torch.randint(0, M, (N, nb), dtype=torch.int16, generator=gen).to(dev)

    def fresh_bank():
        torch.manual_seed(0)
        bank = VQBank(nb, M, D, warm_up_flag=True)
        for b in range(nb):
            bank.init_branch(b)
        return bank.to(dev)

    res = {}
    # "cap4x": capacity above B -> a coarser fixed-point grid of the EMA
    # statistic (dist.CodebookSync docstring): not bit-exact, within the EMA
    # tolerance
    for tag, capacity in (("cap", B), ("nocap", None), ("cap4x", 4 * B)):
        bank = fresh_bank()
        bank.comm = CodebookSync(count_group=dist.new_group(backend="gloo"), capacity=capacity)
        codes = codes0.clone()
        bank.feature_update(X, 0, nb, True, codes=codes, batch_idx=node)
        for _ in range(3):
            bank.update(X, G, 0, nb, True, codes=codes, batch_idx=node, defer=True)
            y = torch.empty(B, F, device=dev)          # work queued behind the collectives
            kernels.gather_codewords(node, 0, codes, bank.emb_out, D)
            y.copy_(X * 2)
            bank.finish_update()
            bank.sync_codes()
        torch.cuda.synchronize()
        for k in ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g"):
            res[f"{tag}_{k}"] = getattr(bank, k).cpu().numpy()
        res[f"{tag}_codes"] = codes.cpu().numpy()
    ref = fresh_bank()
    ref.bn_arith = "fp64"
    rc = codes0.clone()
    ref.feature_update(X, 0, nb, True, codes=rc, batch_idx=node)
    for _ in range(3):
        ref.update(X, G, 0, nb, True, codes=rc, batch_idx=node)
    torch.cuda.synchronize()
    for k in ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g"):
        res["ref_" + k] = getattr(ref, k).cpu().numpy()
    res["ref_codes"] = rc.cpu().numpy()
    np.savez(os.path.join(out_dir, "nccl.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
