"""Benchmark: edges/sec of the VQ-GNN per-layer hot path (BASELINE.json metric).

One step = one layer step on a synthetic arxiv-shaped mini-batch:
  (i)   VQ assign + EMA for all nb branches on the B batch rows — update()
        semantics (W = 2D: features and gradients), one launch sequence
        (BN stats -> BN finalize -> MFMA assign + fused EMA statistics ->
        EMA finalize), c_indices scattered in place;
  (ii)  the aggregation over all nnz edges and all n rows: for GCN / SAGE with
        M <= 319 the codebook-source SpMM (the B' out-of-batch rows read as
        codewords from an LDS image, kernels.spmm_codebook), otherwise the
        codeword gather (x_first_order) + two-source SpMM (GAT: the fused
        attention aggregation).
With update() semantics the EMA finalize is queued after (ii): the
aggregation reads the codebook from before this step's update, as the
reference's forward does (its update runs in the backward hook,
models.py:181-185); one process runs it inside the aggregation's fix-up
launch (--overlap on: the aggregation's walk on a side stream beside (i)'s
BN statistics and assign, the fix-up after both).  With N > 1 the
all-reduce of the EMA statistics overlaps (ii).
value = edges of all ranks / time.  Inputs are resident in HBM before timing.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU, RCCL); each rank takes its own batch
of the same graph (weak scaling) and ranks keep one codebook via an RCCL
all-reduce of the sufficient statistics and an all-gather of the codes.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="arxiv_gcn")
    p.add_argument("--semantics", default="update", choices=["update", "feature_update"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    # rehearsal of the N>1 path on one GPU: --backend gloo with
    # VQGNN_BENCH_ONE_DEVICE=1 puts every rank on cuda:0
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    # rehearsal of the multi-GPU host path on one process (world size 1 under
    # torch.distributed.run): the collectives run on a single rank
    p.add_argument("--force-comm", action="store_true")
    # capture one step in a HIP graph and replay it in the timed region (the
    # same kernels and collectives; no per-kernel host launches)
    p.add_argument("--graph", action="store_true")
    # kernel events inside the timed region (the roofline kernel's launches);
    # off only to measure what they cost
    p.add_argument("--no-kernel-events", action="store_true")
    # the GCN/SAGE aggregation's out-of-batch rows from an LDS image of the
    # codebook (kernels.spmm_codebook) where the shape allows
    # it; --gather-rows: materialise x_first_order and run the two-source SpMM
    p.add_argument("--gather-rows", action="store_true")
    # one process, codebook source: the update's EMA finalize runs inside the
    # aggregation's fix-up launch (vqgnn_spmm_task_cb_fin);
    # --separate-finalize: its own launch after the aggregation
    p.add_argument("--separate-finalize", action="store_true")
    # on: the codebook-source walk on a side stream beside BN statistics +
    # assign (data-independent; the fix-up with the EMA finalize joins both;
    # N > 1: the code exchange lands on the side stream, VQBank.land_codes_on).
    # 2 % faster at N = 1, but the assign then waits for CUs behind the walk
    # and its event-timed duration (the roofline kernel's) grows from 87 to
    # ~144 us, so the default is the serial step
    p.add_argument("--overlap", default="off", choices=["on", "off"])
    # (study) the whole aggregation -- walk and fix-up -- on the side stream,
    # the EMA finalize in its own launch after the join
    p.add_argument("--overlap-whole", action="store_true")
    # (study) the walk queued after the update's BatchNorm launches
    p.add_argument("--walk-after-bn", action="store_true")
    return p.parse_args()


def launcher_cmd(argv, gpus, port):
    """The torch.distributed.run command bench.py starts as a child process
    when called as ``python bench.py --gpus N`` (N > 1) outside a launcher:
    one rank per GPU on this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1",
            "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relay_ranks(args):
    """--gpus N > 1 without WORLD_SIZE: run N ranks under torch.distributed.run
    as a CHILD process (no exec, and nothing here has touched the GPU), relay
    its output (rank 0 prints the JSON line) and exit with its return code."""
    import subprocess
    cmd = launcher_cmd(sys.argv[1:], args.gpus, free_port())
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.run(cmd, env=env)
    sys.exit(proc.returncode)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        relay_ranks(args)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}")
    import torch.distributed as dist
    import vqgnn_pkg
    vqgnn_pkg.load()
    from vq_gnn_amd import kernels
    from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch, synthetic_graph
    from vq_gnn_amd.vq import VQBank
    import vq_gnn_amd.vq as vqmod

    vqmod.STRICT_BAD_INIT = False   # 'Bad Init!' flag checked after the timed region
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("VQGNN_BENCH_ONE_DEVICE") == "1":
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    comm = None
    if world > 1 or args.force_comm:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        from vq_gnn_amd.dist import CodebookSync
        cgroup = dist.new_group(backend="gloo")
        # --graph: the process-group path (a side stream's collective left in
        # flight across a captured step cannot be captured)
        comm = CodebookSync(count_group=cgroup, direct=False if args.graph else None)

    cfg = CONFIGS[args.config]
    if cfg.get("device_build"):      # reddit-sized: graph and batch built on the device
        from vq_gnn_amd.graph import make_batch_device
        dgraph, (bidx, subset, adj) = make_batch_device(cfg, rank=rank, device=dev)
        N_graph = dgraph.N
        B, n, nnz = int(bidx.numel()), int(subset.numel()), adj.nnz()
        del dgraph
        batch = None
    else:
        g = synthetic_graph(cfg["N"], cfg["parts"], cfg["edges"], seed=cfg.get("seed", 0))
        _, _, batch = make_batch(cfg, rank=rank, graph=g)
        N_graph = g.N
        B, n, nnz = batch.B, batch.n, batch.nnz
    F, M, D = cfg["F"], cfg["M"], 4
    nb = F // D
    W = 2 * D if args.semantics == "update" else D

    gen = torch.Generator().manual_seed(1)
    X = torch.randn(B, F, generator=gen)
    G = torch.randn(B, F, generator=torch.Generator().manual_seed(2)) * 1e-3
    codes0 = torch.randint(0, M, (N_graph, nb), dtype=torch.int16,
                           generator=torch.Generator().manual_seed(5))
    torch.manual_seed(0)
    bank = VQBank(nb, M, D, warm_up_flag=True)
    for b in range(nb):
        bank.init_branch(b)
    bank = bank.to(dev)
    Xd, Gd = X.to(dev), G.to(dev)
    codes = codes0.to(dev)
    if batch is not None:
        bidx, subset, adj = batch_to_device(batch, dev)
    if comm is not None:
        bank.comm = comm
        # every rank's batch rows bounded once (the loader's batch bound): the
        # timed steps then issue no host-side collective
        comm.capacity = comm.global_max(B)
    gat = None
    if cfg["conv"] == "GAT":
        from vq_gnn_amd.convs_gat import OurGATConv
        torch.manual_seed(4)
        gat = OurGATConv(F + 1, F + 1, bias=False, add_self_loops=False).to(dev)
    # per-batch adjacency preparation (like the reference's SparseTensor build
    # in the data loader): the SpMM task plan, built once per batch before the
    # timed region; its cost is reported as plan_ms
    spmm_plan = adj.plan(F, B=B)
    use_cb = (gat is None and not args.gather_rows and
              hasattr(kernels.lib(), "vqgnn_spmm_task_cb") and   # (older A/B builds lack it)
              kernels.codebook_source_ok(Xd, F, M, D, codes=codes, n_rows=n, n_branches=nb)
              and kernels.codebook_source_preferred(M))
    if use_cb:   # per batch as well: the records with out-of-batch columns -> nodes
        spmm_plan = adj.plan_codebook(B, subset, N_graph)
    plan_ms = time_plan(adj, n, nnz, cb=(B, subset, N_graph) if use_cb else None)
    # codebook state = one feature_update warm pass
    bank.feature_update(Xd, 0, nb, True, codes=codes, batch_idx=bidx)
    torch.cuda.synchronize()

    ev = []

    def vq_update(before_assign=None):
        if W == 2 * D:
            bank.update(Xd, Gd, 0, nb, True, codes=codes, batch_idx=bidx, defer=True,
                        before_assign=before_assign)
        else:
            bank.feature_update(Xd, 0, nb, True, codes=codes, batch_idx=bidx,
                                before_assign=before_assign)

    overlap = args.overlap == "on" and use_cb and not args.graph
    side = torch.cuda.Stream() if (overlap or args.overlap_whole) else None

    def step(record):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if record else None
        if record:
            e[0].record()
        if side is not None and not record:
            # the aggregation's walk first, on the side stream (it reads X,
            # the out-of-batch nodes' codes and the codebook from before this
            # step's update; the assign writes only batch nodes' codes), then
            # BN statistics + assign on this stream; the fix-up -- with the
            # update's EMA finalize -- after both
            if use_cb and not args.overlap_whole:
                # multi-GPU: the other ranks' previous codes land on the side
                # stream ahead of the walk; the update's own codes wait for it
                bank.land_codes_on(side)
                # the walk queued first (--walk-after-bn: from the update's
                # before_assign hook, after its BatchNorm launches; measured
                # 1.7 % slower)
                wk = kernels.spmm_codebook_walk(adj.rowptr, n, nnz, Xd, F, B, codes,
                                                bank.emb_out, D, spmm_plan, stream=side,
                                                deferred=args.walk_after_bn)
                vq_update(before_assign=wk.launch)
                fin = None if args.separate_finalize else bank.take_fused_finalize()
                fin_fused[0] = fin is not None
                kernels.spmm_codebook_fixup(wk, finalize=fin)     # joins the walk
            else:
                bank.land_codes_on(side)
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    aggregate(False, None, fuse=False)
                vq_update()
                torch.cuda.current_stream().wait_stream(side)
            bank.finish_update()
            if args.graph:
                bank.sync_codes()
            return
        vq_update()
        if record:
            e[1].record()
        aggregate(record, e)
        bank.finish_update()  # EMA finalize (multi-GPU: after the overlapped all-reduce)
        if args.graph:
            bank.sync_codes()     # a captured step joins its code exchange
        # multi-GPU: the other ranks' codes land in the next update, after its
        # assign (VQBank.update): the exchange overlaps gather + SpMM + BN + assign
        if record:
            e[4].record()
            ev.append(e)

    fin_fused = [False]

    def aggregate(record, e, fuse=True):
        if use_cb:          # no x_first_order: the SpMM reads the codebook
            if record:
                e[2].record()
            # the pending EMA finalize inside the SpMM's fix-up launch (one
            # process; multi-GPU it waits for its all-reduce: finish_update)
            fin = None if args.separate_finalize or not fuse else bank.take_fused_finalize()
            fin_fused[0] = fin is not None
            kernels.spmm_codebook(adj.rowptr, n, nnz, Xd, F, B, codes, bank.emb_out, D,
                                  spmm_plan, finalize=fin)
            if record:
                e[3].record()
            return
        x_first, _ = kernels.gather_codewords(subset, B, codes, bank.emb_out, D)
        if record:
            e[2].record()
        if gat is not None:     # attention aggregation (alpha, coefficients, SpMM, normalise)
            with torch.no_grad():
                gat.fused_forward(Xd, adj, x_first, B)
        else:
            kernels.spmm(adj.rowptr, adj.col, adj.value, n, nnz, Xd, F, X2=x_first, B=B,
                         plan=spmm_plan)
        if record:
            e[3].record()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    run = lambda: step(False)  # noqa: E731
    if args.graph:
        gs = torch.cuda.Stream()
        gs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(gs):
            for _ in range(2):
                step(False)
        torch.cuda.current_stream().wait_stream(gs)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step(False)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        run = graph.replay
        barrier()
        torch.cuda.synchronize()
    # timed region: the roofline kernel's launches carry a start/stop HIP
    # event pair taken by hipExtLaunchKernel itself (include/vqgnn.h §5a: the
    # kernel's own duration, no events between kernels on the stream); the
    # per-phase breakdown is a separate pass below.  (--graph: the replays
    # carry no events; the assign is timed in an eager pass after them)
    from vq_gnn_amd._lib import lib as _vqlib
    L = _vqlib()
    kernel_events = not args.no_kernel_events and not args.graph
    if kernel_events:
        L.vqgnn_assign_timing(1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    t_issue = time.perf_counter() - t0      # host time to enqueue the K steps
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    import ctypes

    def read_assign_ms():
        buf = (ctypes.c_float * (4 * args.steps + 8))()
        n = L.vqgnn_assign_timing_read(buf, len(buf))
        L.vqgnn_assign_timing(0)
        return [buf[i] for i in range(n) if buf[i] > 0]

    assign_ms_list = read_assign_ms() if kernel_events else []
    # per-phase breakdown (untimed for value): update | gather | aggregation
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if not assign_ms_list:      # --no-kernel-events / --graph: a separate eager pass
        L.vqgnn_assign_timing(1)
        for _ in range(args.steps):
            step(False)
        torch.cuda.synchronize()
        assign_ms_list = read_assign_ms()
    bank.check_bad_init()

    dt = t1 - t0
    tvec = torch.tensor([dt, float(nnz)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = tvec[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        edges = tvec[1:].clone()
        dist.all_reduce(edges, op=dist.ReduceOp.SUM)
        dt, total_edges = float(tmax.item()), float(edges.item())
    else:
        total_edges = float(nnz)
    ms_step = dt / args.steps * 1e3
    value = total_edges * args.steps / dt

    # VQ update = BN + assign (e0 -> e1) + the deferred finalize (e3 -> e4;
    # with the finalize fused into the aggregation's fix-up launch it is
    # inside the aggregation phase, e2 -> e3)
    vq_ms = float(np.mean([e[0].elapsed_time(e[1]) + e[3].elapsed_time(e[4]) for e in ev]))
    gather_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    spmm_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in ev]))
    assign_ms = float(np.mean(assign_ms_list))

    # Algorithmic work per launch:
    #  the assign: 2*B*M*W flops per branch (the distance contraction in f32,
    #  the exact path's work; for W <= 8 vq_filter_kernel scores on f16 MFMA
    #  and recomputes only the candidates);
    #  SpMM (spmm_task_kernel + spmm_task_fixup_kernel): rowptr + (col, val) + every
    #  input row once (x and x_first_order) + the output rows.
    #  Codebook source (spmm_task_cb_kernel): the records, the B batch rows, the
    #  out-of-batch nodes' codes (nb int16 each), the codebook's feature
    #  halves once, the output rows; the codeword gather kernel is gone.
    spmm_bytes = 4 * (n + 1) + 8 * nnz + 4 * n * F + 4 * n * F
    if use_cb:
        spmm_bytes = 8 * nnz + 4 * B * F + 2 * (n - B) * nb + 4 * nb * M * D + 4 * n * F
    vq_flops = 2.0 * B * M * W * nb
    pmc, pmc_ctr, pmc_note = load_pmc(args)
    agg_name = ("gat aggregation (alpha + fused coefficient/SpMM/normalise walker)"
                if gat is not None else
                "spmm_task_cb_kernel+spmm_task_fixup_kernel (codebook source)" if use_cb else
                "spmm_task_kernel+spmm_task_fixup_kernel")
    agg_pmc = "spmm_task_cb_kernel" if use_cb else "spmm_task_kernel"
    rl_spmm = dict(kernel=agg_name, bound="hbm",
                   achieved=spmm_bytes / (spmm_ms * 1e-3) / 1e9, peak=8000.0, unit="GB/s",
                   bytes_per_launch=spmm_bytes, ms_per_launch=spmm_ms,
                   traffic=pmc.get(agg_pmc))
    rl_spmm["frac"] = rl_spmm["achieved"] / rl_spmm["peak"]
    if rl_spmm["traffic"]:
        rl_spmm["traffic_over_algorithmic"] = rl_spmm["traffic"] / spmm_bytes
    if gat is None:
        # the kernel's own floor: the same plan shape with every column folded
        # onto 1,024 hot rows (all gathers hit L2), DESIGN.md §4.2
        rl_spmm["floor_ms"], rl_spmm["floor_note"] = spmm_floor(kernels, adj, Xd, B, n, nnz, F)
    if args.config in FABRIC_CEILING:
        # counter-backed ceiling of the per-edge row gathers:
        # L2-miss bytes measured per launch at the fabric rate they saturate
        gb, hit, rate = FABRIC_CEILING[args.config]
        rl_spmm["ceiling_ms"] = gb / rate
        rl_spmm["ceiling_note"] = (f"{gb:.1f} GB of L2-miss (MALL/HBM) traffic per launch at "
                                   f"L2 hit {hit:.2f}, at the {rate:.2f} TB/s the gathers saturate "
                                   "(profiles/r03_reddit_spmm_pmc.txt)")
    asg_name = ("vq_filter_kernel" if W <= 8 and os.environ.get("VQGNN_ASSIGN_EXACT", "0") in ("", "0")
                else "vq_assign_kernel")
    rl_vq = assign_roofline(asg_name, assign_ms, B, M, W, nb, vq_flops, pmc_ctr.get(asg_name))
    rl_vq["traffic"] = pmc.get(asg_name)
    dominant = rl_spmm if spmm_ms >= assign_ms else rl_vq
    roofline = dict(bound=dominant["bound"], achieved=dominant["achieved"], peak=dominant["peak"],
                    unit=dominant["unit"], frac=dominant["frac"], traffic=dominant["traffic"],
                    kernel=dominant["kernel"], traffic_source=pmc_note)
    for k in ("limiter", "mfma_issue_frac", "valu_issue_frac", "wait_frac", "effective_f32_frac"):
        if k in dominant:
            roofline[k] = dominant[k]

    # measured device copy rate beside the 8 TB/s spec (a 1 GiB HBM -> HBM
    # copy, read + write bytes), after the timed region
    copy_peak = None
    if rank == 0:
        src = torch.empty(1 << 28, dtype=torch.float32, device=dev)
        dst = torch.empty_like(src)
        dst.copy_(src)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record()
        for _ in range(5):
            dst.copy_(src)
        c1.record()
        torch.cuda.synchronize()
        copy_peak = 2 * src.numel() * 4 * 5 / (c0.elapsed_time(c1) * 1e-3) / 1e9
        del src, dst
    rl_spmm["measured_copy_gbs"] = copy_peak

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_leg(args, X, G, batch, bidx, subset, adj, codes0, M, D, B, nnz, nb, gat)

    if rank == 0:
        out = dict(
            metric="edges/sec (VQ-assign + aggregate) on arxiv-shaped GCN, 1/2/4/8 MI355X",
            value=value, unit="edges/s", n_gpus=world, steps=args.steps, warmup=args.warmup,
            ms_per_step=ms_step, higher_is_better=True, scaling="weak", vs_baseline=None,
            dtype="f32", data="synthetic (seeded arxiv-shaped graph, random features)",
            config=dict(workload=f"{args.config}: one layer step (VQ {args.semantics} + EMA for "
                                 f"{nb} branches, "
                                 + ("SpMM with the out-of-batch rows read from the codebook)"
                                    if use_cb else
                                    "codeword gather, " +
                                    ("GAT attention aggregation)" if gat is not None else "SpMM)")),
                        aggregation=("codebook_source" if use_cb else "gathered_rows"),
                        ema_finalize=("in the aggregation's fix-up launch" if fin_fused[0]
                                      else "own launch"),
                        schedule=("aggregation walk on a side stream beside BN statistics + "
                                  "assign, fix-up after both" if side is not None and use_cb
                                  and not args.overlap_whole else
                                  "whole aggregation on a side stream" if side is not None
                                  else "serial"),
                        B=B, B_prime=n - B, nnz=nnz, F=F, M=M, D=D, W=W,
                        parallelism=f"dp{world}", world=world,
                        backend=(args.backend if comm is not None else None),
                        rccl_ranks=(world if comm is not None and args.backend == "nccl" else 0),
                        devices=(1 if os.environ.get("VQGNN_BENCH_ONE_DEVICE") == "1" else world)),
            roofline=roofline,
            kernels=dict(vq_update_ms=vq_ms, codeword_gather_ms=gather_ms, spmm_ms=spmm_ms,
                         spmm=rl_spmm, vq_assign=rl_vq),
            cpu_baseline=cpu,
            host_issue_ms_per_step=t_issue / args.steps * 1e3,
            plan_ms=plan_ms,
        )
        print(json.dumps(out))
    if comm is not None:
        comm.close()            # direct RCCL communicators: a clean destroy on every rank
    if dist.is_initialized():
        dist.destroy_process_group()


def lib_digest():
    """sha256 of the libvqgnn.so this process loaded: ties PMC traffic to the
    build it was measured on."""
    import hashlib
    from vq_gnn_amd._lib import LIB_PATH
    h = hashlib.sha256()
    with open(LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


# reddit SpMM: fabric (L2-miss) read + write GB per launch, L2 hit rate, and the
# fabric rate in TB/s the per-edge gathers reach (the same 7.2-7.4 TB/s at F =
# 128 and 604 and for the tiled plan's remainder pass), from the PMC passes
# of scripts/gpu_pmc_reddit.sh (profiles/r03_reddit_spmm_pmc.txt)
FABRIC_CEILING = {"reddit_gcn": (27.2, 0.56, 7.39), "reddit_gcn_l1": (164.8, 0.54, 7.39)}


def load_pmc(args):
    """Per-launch HBM bytes and SQ counters from profiles/pmc_latest.json
    (scripts/pmc_to_json.py) -- only when they were captured on this config
    AND on the library this process runs (its lib_sha256); otherwise none,
    with the reason."""
    if not os.path.exists(args.pmc_json):
        return {}, {}, "no PMC file"
    try:
        pm = json.load(open(args.pmc_json))
    except (OSError, ValueError) as exc:
        return {}, {}, f"unreadable PMC file ({exc})"
    if pm.get("config") != args.config or pm.get("semantics", "update") != args.semantics:
        return {}, {}, f"PMC file is for {pm.get('config')}/{pm.get('semantics')}"
    lib_hash = lib_digest()
    if pm.get("lib_sha256") != lib_hash:
        return {}, {}, (f"PMC file from another build (lib {str(pm.get('lib_sha256'))[:12]}, "
                        f"running {lib_hash[:12]}): traffic withheld")
    return pm.get("hbm_bytes_per_launch", {}), pm.get("counters_per_launch", {}), (
        f"{os.path.relpath(args.pmc_json, ROOT)} (lib {lib_hash[:12]}, git {pm.get('git_head')})")


# gfx950 (MI355X_MICROARCH.md): dense f16 matrix peak, f32 matrix peak, SIMDs,
# nominal clock, cycles per wave64 VALU instruction on a SIMD32
F16_PEAK_TF, F32_PEAK_TF, SIMDS, CLOCK_HZ, VALU_CYCLES = 2500.0, 157.3, 1024, 2.4e9, 2


def assign_roofline(name, assign_ms, B, M, W, nb, f32_flops, ctr):
    """The assign's roofline by SURVEY §8(d): algorithmic flops (2*B*M*W*nb,
    the distance contraction) / the kernel's own launch time / the dense peak
    of the matrix pipe the kernel computes them on.  vq_filter_kernel scores
    every codeword with v_mfma_f32_16x16x32_f16, so its peak is the dense f16
    peak; the exact f32 path (vq_assign_kernel, W > 8) is
    priced against the f32 matrix peak.  Beside it, from the hash-stamped PMC
    counters of this build: mfma_issue_frac = f16 MFMA flops ISSUED
    (SQ_INSTS_MFMA x 16,384: the hi/lo split issues ~4.3x the algorithmic
    flops) over the same peak, the VALU issue fraction and the share of wave
    cycles spent waiting.  effective_f32_frac = the algorithmic flops over the
    f32 peak (what the exact path would need; not a roofline)."""
    t = assign_ms * 1e-3
    eff = f32_flops / t / 1e12 / F32_PEAK_TF
    if name != "vq_filter_kernel":
        return dict(kernel=name, bound="mfma", achieved=f32_flops / t / 1e12, peak=F32_PEAK_TF,
                    unit="TFLOP/s", frac=eff, flops_per_launch=f32_flops, ms_per_launch=assign_ms,
                    flops_note="2*B*M*W*nb f32 flops (exact sweep, v_mfma_f32_16x16x4_f32)",
                    effective_f32_frac=eff)
    out = dict(kernel=name, bound="mfma", achieved=f32_flops / t / 1e12, peak=F16_PEAK_TF,
               unit="TFLOP/s", flops_per_launch=f32_flops, ms_per_launch=assign_ms,
               flops_note="2*B*M*W*nb algorithmic distance flops (SURVEY 8d) over the dense f16 "
                          "peak of the pipe the filter scores on",
               effective_f32_frac=eff,
               effective_f32_note="the same flops / time / 157.3 TF/s (f32 peak): what the exact "
                                  "path would need, not a roofline")
    out["frac"] = out["achieved"] / out["peak"]
    if ctr and ctr.get("SQ_INSTS_MFMA"):
        mfma = ctr["SQ_INSTS_MFMA"]
        src = "SQ_INSTS_MFMA x 16384 (PMC, this build)"
    else:
        mfma = nb * -(-B // 64) * 4 * (M // 16)
        src = "analytic lower bound: nb * ceil(B/64) * 4 groups * M/16 tiles (no PMC for this build)"
    issued = mfma * 16384.0
    out["mfma_issue_frac"] = issued / t / 1e12 / F16_PEAK_TF
    out["mfma_issued_flops"] = issued
    out["mfma_issue_note"] = f"f16 MFMA flops issued: {src}, over the dense f16 peak"
    if ctr and ctr.get("SQ_INSTS_VALU") and ctr.get("SQ_WAVE_CYCLES"):
        out["valu_issue_frac"] = ctr["SQ_INSTS_VALU"] * VALU_CYCLES / SIMDS / CLOCK_HZ / t
        out["wait_frac"] = ctr.get("SQ_WAIT_ANY", 0.0) / ctr["SQ_WAVE_CYCLES"]
        busiest = max(("f16 MFMA", out["mfma_issue_frac"]), ("VALU issue", out["valu_issue_frac"]),
                      key=lambda kv: kv[1])
        out["limiter"] = (f"latency: {out['wait_frac']:.0%} of wave cycles waiting; busiest issue "
                          f"port {busiest[0]} at {busiest[1]:.0%} (PMC)")
    return out


def time_plan(adj, n, nnz, reps=5, cb=None):
    """Device time of one task-plan build (records, task starts, fix-up jobs and
    the job-count readback; cb = (B, subset, nodes): plus the codebook-source
    records), the per-batch preparation outside the timed step."""
    from vq_gnn_amd import kernels
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p = kernels.spmm_task_plan(adj.rowptr, adj.col, adj.value, n, nnz)
        if cb is not None:
            p.with_codebook_source(*cb)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts[1:])) * 1e3


def spmm_floor(kernels, adj, Xd, B, n, nnz, F, hot=1024, reps=10):
    """SpMM over the same rows and row lengths with every column folded onto
    `hot` rows of X (all gathers L2 hits): the per-edge gather issue floor of
    the kernel, no memory system behind it."""
    if B < hot:
        return None, "batch smaller than the hot set"
    col = torch.remainder(adj.col, hot).to(torch.int32)
    plan = kernels.spmm_task_plan(adj.rowptr, col, adj.value, n, nnz)
    out = torch.empty(n, F, dtype=torch.float32, device=Xd.device)
    run = lambda: kernels.spmm(adj.rowptr, col, adj.value, n, nnz, Xd[:hot], F,  # noqa: E731
                               out=out, plan=plan)
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, f"columns folded onto {hot} hot rows, same plan shape"


def cpu_leg(args, X, G, batch, bidx, subset, adj, codes0, M, D, B, nnz, nb, gat):
    """cpu_baseline: the reference layer step (oracle/cpu_baseline.py) on the
    host cores this process may use -- the affinity set, capped by
    OMP_NUM_THREADS when the box sets it (its CPU share) -- and on one
    thread, each on a bounded sample of the same workload scaled to edges/s
    (about 10-30 s of CPU work in total)."""
    from types import SimpleNamespace

    from oracle.cpu_baseline import host_topology, layer_step_timer
    if batch is None:          # device-built batch: the same CSR on the host
        rp, cl, vl = adj.csr()
        batch = SimpleNamespace(batch_idx=bidx.cpu().numpy(), subset=subset.cpu().numpy(),
                                rowptr=rp.cpu().numpy(), col=cl.cpu().numpy(),
                                val=vl.cpu().numpy(), n=int(subset.numel()))
    host = host_topology()
    threads = host["affinity"]
    cap_source = f"sched_getaffinity ({threads} CPUs)"
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0 and int(omp) < threads:
        threads = int(omp)
        cap_source = f"OMP_NUM_THREADS={omp} (the box's CPU share; affinity {host['affinity']})"
    att = None
    if gat is not None:
        att = (gat.att_l.detach().cpu().view(-1).numpy(), gat.att_r.detach().cpu().view(-1).numpy())
    # the headline config: the full step on `threads` threads (~4 s per step
    # on 16); the other configs: a quarter of the branches and at most 8 M
    # edges per step
    full = args.config == "arxiv_gcn"
    t_all, n_all, desc_all = layer_step_timer(
        X, G, batch, codes0, M, D, threads, max_seconds=args.cpu_seconds,
        branch_sample=None if full else max(2, nb // 4),
        edge_sample=None if full else 8_000_000, gat=att)
    # one thread: every 8th branch (at least 2) and 1/16 of the edges (at most
    # 128 M edge-columns)
    t_one, n_one, desc_one = layer_step_timer(
        X, G, batch, codes0, M, D, 1, max_seconds=4.0, min_steps=5,
        branch_sample=max(2, nb // 8),
        edge_sample=max(min(nnz // 16, 128_000_000 // X.shape[1]), 1), gat=att)
    torch.set_num_threads(threads)
    sem = "update semantics" + (", GAT aggregation" if gat is not None else "")
    return dict(value=nnz / t_all, unit="edges/s", cores=threads, kind="port",
                sample=f"{args.config} layer step ({sem}, {nb} branches, B={B}, nnz={nnz}): "
                       f"{desc_all}; median of {n_all} steps after 1 warm-up; "
                       f"oracle/cpu_baseline.py, torch {torch.__version__} CPU",
                thread_cap=cap_source,
                value_1thread=nnz / t_one,
                sample_1thread=f"{desc_one}; median of {n_one} steps",
                host=host)


if __name__ == "__main__":
    main()
