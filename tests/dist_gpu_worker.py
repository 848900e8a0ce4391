"""Worker for tests/test_gpu_dist.py (launched by torch.distributed.run, 2 ranks
on one GPU over gloo): each rank runs VQBank.feature_update + update on its
half of a batch with CodebookSync; rank 0 then replays the union batch in a
single-process bank.  Results -> <out>/r<rank>.npz."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_dir):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import vqgnn_pkg
    vqgnn_pkg.load()
    from vq_gnn_amd.dist import CodebookSync
    from vq_gnn_amd.vq import VQBank
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    nb, M, D, N, Bu = 6, 64, 4, 4000, 3000
    F = nb * D
    gen = torch.Generator().manual_seed(11)
    X = torch.randn(Bu, F, generator=gen)
    G = torch.randn(Bu, F, generator=gen) * 1e-3
    node = torch.randperm(N, generator=gen)[:Bu]
    codes0 = torch.randint(0, M, (N, nb), dtype=torch.int16, generator=gen)

    def fresh_bank():
        torch.manual_seed(0)
        bank = VQBank(nb, M, D, warm_up_flag=True)
        for b in range(nb):
            bank.init_branch(b)
        return bank.to(dev)

    # uneven batches: rank 0 takes the first 1,800 rows of the union, rank 1
    # the remaining 1,200 (no capacity: the ranks agree on max(B) per call)
    cut = 1800
    mine = torch.arange(0, cut) if rank == 0 else torch.arange(cut, Bu)
    bank = fresh_bank()
    bank.comm = CodebookSync(count_group=dist.new_group(backend="gloo"))
    codes = codes0.to(dev)
    Xr, Gr, nr = X[mine].to(dev), G[mine].to(dev), node[mine].to(dev)
    bank.feature_update(Xr, 0, nb, True, codes=codes, batch_idx=nr)
    bank.update(Xr, Gr, 0, nb, True, codes=codes, batch_idx=nr)
    bank.sync_codes()
    torch.cuda.synchronize()
    res = {k: getattr(bank, k).cpu().numpy() for k in
           ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g")}
    res["codes"] = codes.cpu().numpy()
    if rank == 0:                                  # single-process union batch
        ref = fresh_bank()
        ref.bn_arith = "fp64"       # the multi-rank statistics' arithmetic
        rc = codes0.to(dev)
        Xu, Gu, nu = X.to(dev), G.to(dev), node.to(dev)
        ref.feature_update(Xu, 0, nb, True, codes=rc, batch_idx=nu)
        emb_pre = ref.emb.clone()
        ref.update(Xu, Gu, 0, nb, True, codes=rc, batch_idx=nu)
        torch.cuda.synchronize()
        # fp64 distances of the update (vq.py:223-236 on the union batch's
        # statistics) to classify any index mismatch as a near-tie or not
        x64, g64 = X.double(), G.double()
        zx = (x64 - x64.mean(0)) / torch.sqrt(x64.var(0, unbiased=False) + 1e-5)
        zg = (g64 - g64.mean(0)) / torch.sqrt(g64.var(0, unbiased=False) + 1e-24)
        e64 = emb_pre.double().cpu()
        dists = []
        for b in range(nb):
            z = torch.cat([zx[:, b * D:(b + 1) * D], zg[:, b * D:(b + 1) * D]], 1)
            e = e64[b]
            dists.append(((z * z).sum(1, keepdim=True) + (e * e).sum(1)[None] - 2 * z @ e.T)
                         .float().numpy())
        res["ref_dist"] = np.stack(dists)
        res["node"] = node.numpy()
        for k in ("emb", "emb_out", "ema_w", "cs", "rm_f", "rv_f", "rm_g", "rv_g"):
            res["ref_" + k] = getattr(ref, k).cpu().numpy()
        res["ref_codes"] = rc.cpu().numpy()
    # repeated nodes across ranks: nodes 0..9 in both ranks' rows with
    # rank-specific codes; every replica keeps the LAST record's (rank 1)
    sync = bank.comm
    c2 = torch.zeros(N, nb, dtype=torch.int16, device=dev)
    ids = torch.cat([torch.arange(10), torch.arange(100 + 10 * rank, 110 + 10 * rank)]).to(dev)
    loc = (torch.arange(20, device=dev)[:, None] + 7 * (rank + 1) +
           torch.arange(nb, device=dev)[None]).to(torch.int16) % M
    sync.start_codes_exchange(ids, loc.contiguous(), c2, max_B=24, M=M).wait()
    torch.cuda.synchronize()
    res["dup_codes"] = c2.cpu().numpy()
    # two exchanges of the same shape in flight on one CodebookSync (two
    # layers' banks): the second start lands the first before reusing the
    # shared wire buffers, so each codes array gets its own records
    ca = torch.zeros(N, nb, dtype=torch.int16, device=dev)
    cb = torch.zeros(N, nb, dtype=torch.int16, device=dev)
    ids = (torch.arange(12) * 2 + rank).to(dev)
    la = ((torch.arange(12, device=dev)[:, None] + torch.arange(nb, device=dev)[None]) % M).to(torch.int16)
    lb = ((la.to(torch.int32) + 5) % M).to(torch.int16)
    pa = sync.start_codes_exchange(ids, la.contiguous(), ca, max_B=12, M=M)
    pb = sync.start_codes_exchange(ids, lb.contiguous(), cb, max_B=12, M=M)
    pb.wait()
    pa.wait()
    torch.cuda.synchronize()
    res["two_a"] = ca[:24].cpu().numpy()
    res["two_b"] = cb[:24].cpu().numpy()
    # staleness contract of the deferred exchange, with a
    # capacity (no host collective) as bench.py runs it: three consecutive
    # update(defer=True) steps on disjoint node sets S[rank][step]; after step
    # k a rank's codes hold its own step-k codes and the other rank's
    # step-(k-1) codes, the other rank's step-k rows still hold their old
    # codes; after sync_codes() the replicas are identical
    sb = fresh_bank()
    sb.comm = CodebookSync(count_group=sync.count_group, capacity=700)
    sc = codes0.to(dev)
    perm = torch.randperm(N, generator=torch.Generator().manual_seed(3))
    sets = [[perm[(2 * k + r) * 600:(2 * k + r) * 600 + 600 - 50 * r] for k in range(3)]
            for r in range(world)]
    for k in range(3):
        gk = torch.Generator().manual_seed(100 + 10 * k + rank)
        nodes = sets[rank][k]
        Xk = torch.randn(nodes.numel(), F, generator=gk).to(dev)
        Gk = (torch.randn(nodes.numel(), F, generator=gk) * 1e-3).to(dev)
        sb.update(Xk, Gk, 0, nb, True, codes=sc, batch_idx=nodes.to(dev), defer=True)
        sb.finish_update()
        torch.cuda.synchronize()
        res[f"stale_{k}"] = sc.cpu().numpy()
    sb.sync_codes()
    torch.cuda.synchronize()
    res["stale_final"] = sc.cpu().numpy()
    # the overlapped step (bench.py --overlap on): the previous exchange lands
    # on a side stream (VQBank.land_codes_on) where the aggregation's walk then
    # reads the codes, beside the update on the compute stream; the codes
    # after every step must equal the serial steps' above, and what the side
    # stream reads must be the codes the serial step's aggregation reads
    ob2 = fresh_bank()
    ob2.comm = CodebookSync(count_group=sync.count_group, capacity=700)
    oc2 = codes0.to(dev)
    side = torch.cuda.Stream()
    for k in range(3):
        gk = torch.Generator().manual_seed(100 + 10 * k + rank)
        nodes = sets[rank][k]
        Xk = torch.randn(nodes.numel(), F, generator=gk).to(dev)
        Gk = (torch.randn(nodes.numel(), F, generator=gk) * 1e-3).to(dev)
        ob2.land_codes_on(side)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            seen = oc2.clone()                     # the walk's view
        ob2.update(Xk, Gk, 0, nb, True, codes=oc2, batch_idx=nodes.to(dev), defer=True)
        torch.cuda.current_stream().wait_stream(side)
        ob2.finish_update()
        torch.cuda.synchronize()
        res[f"ostale_{k}"] = oc2.cpu().numpy()
        res[f"oseen_{k}"] = seen.cpu().numpy()
    res["stale_codes0"] = codes0.numpy()
    for r in range(world):
        for k in range(3):
            res[f"set_{r}_{k}"] = sets[r][k].numpy()
    # a batch over the CodebookSync capacity (capacity 300, world 2): rank 0
    # at 500 rows (the summed rows exceed world * capacity) and then at 700
    # (over world * capacity itself).  Neither rank raises between the
    # collectives (no hang), the EMA statistics stay inside the fixed-point
    # row bound (finite, identical replicas), and both ranks raise together
    # at the check after the update.
    # (the flags are read by the explicit check below, as with
    # VQGNN_DEFER_BAD_INIT=1, not inside finish_update)
    import vq_gnn_amd.vq as vqmod
    strict, vqmod.STRICT_BAD_INIT = vqmod.STRICT_BAD_INIT, False
    for tag, b_over in (("over500", 500), ("over700", 700)):
        ob = fresh_bank()
        ob.comm = CodebookSync(count_group=sync.count_group, capacity=300)
        oc = codes0.to(dev)
        nodes = perm[:b_over] if rank == 0 else perm[2000:2200]
        go = torch.Generator().manual_seed(7 + rank)
        Xo = torch.randn(nodes.numel(), F, generator=go).to(dev)
        Go = (torch.randn(nodes.numel(), F, generator=go) * 1e-3).to(dev)
        ob.update(Xo, Go, 0, nb, True, codes=oc, batch_idx=nodes.to(dev), defer=True)
        ob.finish_update()
        ob.sync_codes()
        torch.cuda.synchronize()
        try:
            ob.check_bad_init()
            res[f"{tag}_raised"] = 0
        except ValueError as exc:
            res[f"{tag}_raised"] = int("capacity" in str(exc))
        for k in ("emb", "emb_out", "ema_w", "cs"):
            res[f"{tag}_{k}"] = getattr(ob, k).cpu().numpy()
        res[f"{tag}_codes"] = oc.cpu().numpy()
    vqmod.STRICT_BAD_INIT = strict
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
