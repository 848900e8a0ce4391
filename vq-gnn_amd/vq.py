"""Drop-in ``VectorQuantizerEMA`` (reference: vq_gnn_v2/vq.py:60-279) on HIP.

State layout.  The reference keeps one ``VectorQuantizerEMA`` per branch
(feature slice of D columns) with its own small buffers.  Here the state of
all ``nb`` branches of a layer lives in one ``VQBank`` ([nb, M, 2D] codebooks,
[nb, M] cluster sizes, [nb, D] BatchNorm running stats) so that one kernel
launch serves every branch; each per-branch ``VectorQuantizerEMA`` exposes
views of its slice under the reference's buffer names (``_embedding``,
``_embedding_output``, ``_ema_cluster_size``, ``_ema_w``,
``batch_norm_feat.running_mean`` ...), and ``state_dict()`` /
``load_state_dict()`` use the reference's keys.

Numerics.  BatchNorm follows the ATen CPU path the reference takes for the
same input layout (``bn_arith = "aten"``, the default on one process): the
cascade-sum statistics of a strided branch slice, or the per-thread row
chunks of a contiguous [B, D] input with ``ref_threads`` threads (see
include/vqgnn.h §2 and oracle/bn_ref.py).  With multi-GPU statistics
(``comm`` set) or ``bn_arith = "fp64"`` the batch statistics are fp64 sums,
identical for any number of ranks.  The normalisation, distance and argmin
follow ATen's CPU arithmetic exactly (csrc/vq_kernels.hip), so codeword
indices are bit-exact.  The EMA statistics (counts and encodingsᵀ·x_norm)
are int64 fixed-point sums, exact and order-free, rounded to fp32 once
(DESIGN §2.2); the reference's MKL sgemm sums them in fp32 in an order of
its own, so EMA state matches within the documented bound.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from . import kernels
from .kernels import (BN_CONTIG, BN_EVAL, BN_EVAL_INIT, BN_FP64, BN_TRAIN, BN_TRAIN_INIT,
                      bn_arith_of)

# 'Bad Init!' (vq.py:188) is a device flag.  The reference checks it with a
# host sync on every call; VQGNN_DEFER_BAD_INIT=1 defers the check to
# VQBank.check_bad_init() (used by bench.py so the timed step has no sync).
STRICT_BAD_INIT = os.environ.get("VQGNN_DEFER_BAD_INIT", "0") != "1"


class FusedFinalize:
    """A pending EMA finalize handed to an aggregation
    (VQBank.take_fused_finalize): ``operands`` = (args, kw) of
    kernels.vq_ema_finalize for the fused fix-up launch; done() -- called by
    kernels.spmm_codebook once that launch is queued, idempotent -- retires it
    from the bank.  Until then the bank keeps it pending."""

    def __init__(self, bank, entry):
        self._bank, self._entry = bank, entry
        self.operands = (entry[1], entry[2])

    def done(self):
        bank = self._bank
        if bank._pending_finalize is self._entry:
            bank._pending_finalize = None
            bank._clean(*self._entry[3])
            bank._finish()


class VQBank(nn.Module):
    """Packed EMA-VQ state of ``nb`` branches.  Buffers are non-persistent: the
    per-branch ``VectorQuantizerEMA`` modules own the state_dict entries."""

    def __init__(self, nb, num_embeddings, embedding_dim, decay=0.99, epsilon=1e-24,
                 grad_normalize_scale=(1, 1), warm_up_flag=False, momentum=0.1):
        super().__init__()
        M, D = int(num_embeddings), int(embedding_dim)
        self.nb, self.M, self.D = int(nb), M, D
        self.W = 2 * D
        self.decay, self.epsilon = float(decay), float(epsilon)
        self.grad_normalize_scale = grad_normalize_scale
        self.warm_up_flag = bool(warm_up_flag)
        self.momentum = float(momentum)
        z = lambda *s: torch.zeros(*s, dtype=torch.float32)  # noqa: E731
        self.register_buffer("emb", z(nb, M, self.W), persistent=False)
        self.register_buffer("emb_out", z(nb, M, self.W), persistent=False)
        self.register_buffer("ema_w", z(nb, M, self.W), persistent=False)
        self.register_buffer("cs", z(nb, M), persistent=False)
        self.register_buffer("rm_f", z(nb, D), persistent=False)
        self.register_buffer("rv_f", torch.ones(nb, D), persistent=False)
        self.register_buffer("rm_g", z(nb, D), persistent=False)
        self.register_buffer("rv_g", torch.ones(nb, D), persistent=False)
        self.register_buffer("nbt_f", torch.zeros(nb, dtype=torch.long), persistent=False)
        self.register_buffer("nbt_g", torch.zeros(nb, dtype=torch.long), persistent=False)
        self.register_buffer("bad_flag", torch.zeros(1, dtype=torch.int32), persistent=False)
        # EMA sufficient-statistic slabs (int64 fixed point, include/vqgnn.h
        # §3), kept zero between calls: the finalize clears what it consumes,
        # so the assign needs no memset.  dirty[b]: branch b's slab may hold
        # data (an update interrupted between assign and finalize).
        zl = lambda W: torch.zeros(1, nb, M, W + 1, dtype=torch.int64)  # noqa: E731
        self.register_buffer("stats_f", zl(D), persistent=False)
        self.register_buffer("stats_u", zl(2 * D), persistent=False)
        self._dirty = {D: [False] * nb, 2 * D: [False] * nb}
        self.bn_inited = [False] * nb
        # multi-GPU: a dist.CodebookSync (all-reduce of sufficient statistics,
        # all-gather of codes); None on one GPU
        self.comm = None
        # optional list: (start, end) HIP events around every assign launch
        # (bench.py times vq_assign_kernel alone with it); None = off
        self.assign_events = None
        # multi-GPU: codes of the other ranks' batches arrive asynchronously
        # (dist.PendingCodes); sync_codes() lands them
        self._pending_codes = None
        # update(defer=True): the finalize (and, multi-GPU, the wait for the
        # asynchronous all-reduce of the EMA statistics) left for
        # finish_update(), so work that reads the pre-update codebook (the
        # reference forward's gather + aggregation) runs in between
        self._pending_finalize = None
        # last batched call's logging stash (vq.py:208-214, :276-277)
        self.last_batch = None       # [4, nb*D] mean_f, std_f, mean_g, std_g
        self.last_inputs = None      # (X, G) of the last update()
        # BatchNorm arithmetic: "aten" reproduces the reference's ATen CPU
        # path for the input layout; "fp64" = rank-count-invariant fp64 sums
        # (always used with multi-GPU statistics).  ref_threads: the
        # reference's torch.get_num_threads() for contiguous inputs (None:
        # VQGNN_REF_THREADS, else this process's torch.get_num_threads()).
        self.bn_arith = "aten"
        self.ref_threads = None

    def init_branch(self, b):
        """Per-branch random init in the reference's RNG order (vq.py:73-98)."""
        M, D = self.M, self.D
        self.emb[b].copy_(torch.randn(M, self.W))
        if self.warm_up_flag:
            self.ema_w[b].normal_()
        s0 = self.grad_normalize_scale[0]
        self.emb[b, :, D:2 * D] *= s0
        self.ema_w[b, :, D:2 * D] *= s0

    # ------------------------------------------------------------------ #
    def check_bad_init(self):
        if self.comm is not None and self.comm.take_overflow():
            raise ValueError(f"a rank's batch exceeded CodebookSync capacity "
                             f"{self.comm.capacity}")
        if int(self.bad_flag.item()) != 0:
            self.bad_flag.zero_()
            raise ValueError('Bad Init!')

    def _finish(self):
        if STRICT_BAD_INIT:
            self.check_bad_init()

    _arange_cache = {}

    def _arange(self, B, device):
        key = (B, str(device))
        t = VQBank._arange_cache.get(key)
        if t is None:
            t = torch.arange(B, dtype=torch.int64, device=device)
            VQBank._arange_cache[key] = t
        return t

    def sync_codes(self):
        """Land the other ranks' codes of the last update (multi-GPU); a no-op
        on one GPU.  Called before the next VQ call and by the layer after its
        aggregation, so the exchange overlaps the gather + SpMM.  After
        land_codes_on(stream) the current stream waits for that landing."""
        ev, self._codes_landed = self._codes_landed, None
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        p, self._pending_codes = self._pending_codes, None
        if p is not None:
            p.wait()

    _codes_landed = None

    def land_codes_on(self, stream):
        """Multi-GPU, the overlapped step (an aggregation walk on `stream`
        beside the next update): land the last update's code exchange on
        `stream`, ahead of the walk that reads the codes there.  The next
        sync_codes() -- the update's, before it scatters its own codes --
        makes its stream wait for this landing, so the order of the code
        writes (the other ranks' previous codes, then this rank's new ones)
        is the serial step's.  A no-op when nothing is pending."""
        if self._pending_codes is None:
            return
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            p, self._pending_codes = self._pending_codes, None
            p.wait()
            ev = torch.cuda.Event()
            ev.record(stream)
        self._codes_landed = ev

    def _exchange_codes(self, batch_idx, local, codes, max_B):
        """Own codes now (scattered by the pack kernel), everyone's
        asynchronously (landed by sync_codes).  Rows past max_B (a batch over
        the CodebookSync capacity, raised at the next check on every rank)
        are not scattered at all: every replica keeps those nodes' previous
        codes, so the replicas stay identical even for a caller that catches
        the error, and the collective keeps its shape."""
        if local.shape[0] > max_B:
            batch_idx, local = batch_idx[:max_B], local[:max_B]
        self._pending_codes = self.comm.start_codes_exchange(batch_idx, local, codes,
                                                             max_B, self.M)

    _local_cache = None

    def _local_codes(self, B, nbr, device):
        """This rank's codes of an exchanging update (multi-GPU): a buffer
        reused across updates of one shape (the pack kernel reads it on the
        stream before the next update overwrites it)."""
        key = (B, nbr, str(device))
        c = self._local_cache
        if c is None or c[0] != key:
            c = self._local_cache = (key, torch.empty(B, nbr, dtype=torch.int16, device=device))
        return c[1]

    def _slab(self, W, b0, nbr):
        """Zeroed statistic slab [1, nbr, M, W+1] for branches [b0, b0+nbr)."""
        buf = self.stats_f if W == self.D else self.stats_u
        view = buf[:, b0:b0 + nbr]
        dirty = self._dirty[W]
        if any(dirty[b0:b0 + nbr]):
            view.zero_()
        for b in range(b0, b0 + nbr):
            dirty[b] = True
        return view

    def _clean(self, W, b0, nbr):
        for b in range(b0, b0 + nbr):
            self._dirty[W][b] = False

    def _assign(self, *args, **kw):
        if self.assign_events is None:
            return kernels.vq_assign(*args, **kw)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        out = kernels.vq_assign(*args, **kw)
        ev[1].record()
        self.assign_events.append(ev)
        return out

    def _assign_capped(self, X, G, coef, scale, emb, W, idx_out, codes, batch_idx, training,
                       count, slab, cap):
        """The assign.  A multi-GPU batch over the CodebookSync capacity (an
        error every rank raises together at the next check) takes its EMA
        statistics from its first ``cap`` rows only: the summed rows then
        never exceed the fixed-point row bound world * capacity (no
        saturation, no corrupted codebook), and no rank raises on its own
        between two collectives (the others would wait forever).  Its other
        rows are still assigned (indices and codes)."""
        D = self.D
        B = X.shape[0]
        if cap is None or B <= cap or not training:
            return self._assign(X, G, coef, scale, emb, D, W, idx_out=idx_out, codes=codes,
                                batch_idx=batch_idx, want_stats=training, stat_count=count,
                                stats_out=slab)
        parts = []
        for lo, hi, stats in ((0, cap, True), (cap, B, False)):
            io = None if idx_out is None else torch.empty(idx_out.shape[0], hi - lo,
                                                          dtype=idx_out.dtype, device=X.device)
            st = self._assign(X[lo:hi], None if G is None else G[lo:hi], coef, scale, emb, D, W,
                              idx_out=io, codes=codes,
                              batch_idx=None if batch_idx is None else batch_idx[lo:hi],
                              want_stats=stats, stat_count=count,
                              stats_out=slab if stats else None)
            if io is not None:
                idx_out[:, lo:hi].copy_(io)
            parts.append(st)
        return parts[0]

    def _sel(self, b0, nbr):
        return slice(b0, b0 + nbr)

    def _threads(self):
        if self.ref_threads is not None:
            return int(self.ref_threads)
        env = os.environ.get("VQGNN_REF_THREADS")
        return int(env) if env else torch.get_num_threads()

    def _arith(self, t, comm):
        """(arith for batch statistics, arith for the eval form) of input t."""
        layout = bn_arith_of(t, self.D)
        if comm is not None or self.bn_arith == "fp64":
            return BN_FP64, layout
        return layout, layout

    def _bn_fold(self, B, nbr, W, ax, ag):
        """Single process: whether the BatchNorm finalize folds into the
        assign's prologue (kernels.bn_stats_partial + vq_assign(BnFold): one
        launch fewer, the same bits as bn_stats_finalize + vq_assign;
        include/vqgnn.h §3a).  Opt-in (VQGNN_BN_FOLD=1): every row part's
        workgroup folds its branch's columns, so the assign reads 16x the
        partials and grows by about the finalize it replaces; the step
        measured -2.7 % and +0.3 % on two boxes."""
        if os.environ.get("VQGNN_BN_FOLD", "0") == "0":
            return False
        if BN_CONTIG in (ax, ag) or (ax == BN_FP64 and ag == BN_FP64):
            return False
        return kernels.bn_fold_supported(B, nbr, self.D, self.M, W)

    def feature_update(self, X, b0, nbr, training, idx_out=None, codes=None, batch_idx=None,
                       before_assign=None):
        """vq.py:160-202 for branches [b0, b0+nbr): X is [B, nbr*D] (a row-major view).
        before_assign: called after the BatchNorm launches, before the
        assign's (update())."""
        self.finish_update()
        exchanging = training and self.comm is not None and codes is not None
        if not exchanging:
            self.sync_codes()
        D, F = self.D, nbr * self.D
        sl = self._sel(b0, nbr)
        B = X.shape[0]
        if training and B <= 1:
            raise ValueError("Expected more than 1 value per channel when training")
        comm = self.comm if training else None
        ax, ax_eval = self._arith(X, comm)
        if training and comm is None:      # one process: statistics + finalize
            count = B
            if self._bn_fold(B, nbr, D, ax, ax):
                coef = kernels.bn_stats_partial(X, None, F, BN_TRAIN, 0.1, 1e-5, 0.0, 0.0, 0.0,
                                                self.rm_f[sl], self.rv_f[sl],
                                                nbt_f=self.nbt_f[sl], D=D, arith_x=ax)
            else:
                coef, _, _ = kernels.bn_stats_finalize(X, None, F, BN_TRAIN, 0.1, 1e-5, 0.0,
                                                       0.0, 0.0, self.rm_f[sl], self.rv_f[sl],
                                                       nbt_f=self.nbt_f[sl], D=D, arith_x=ax,
                                                       ref_threads=self._threads())
        elif training:         # multi-GPU: the global count rides in the sums
            sums = kernels.bn_stats(X, None, F, with_count=True)
            max_B = comm.allreduce_stats_(sums, B)
            count = comm.world * max_B      # row bound of the fixed-point shift
            coef, _ = kernels.bn_finalize(sums, 0, F, False, BN_TRAIN, 0.1, 1e-5, 0.0, 0.0,
                                          0.0, self.rm_f[sl], self.rv_f[sl], nbt_f=self.nbt_f[sl],
                                          D=D)
        else:
            count = B
            coef, _ = kernels.bn_finalize(None, B, F, False, BN_EVAL, 0.1, 1e-5, 0.0, 0.0, 0.0,
                                          self.rm_f[sl], self.rv_f[sl], arith_x=ax_eval)
        slab = self._slab(D, b0, nbr) if training else None
        local = None
        cap = max_B if comm is not None else None
        if before_assign is not None:
            before_assign()
        if comm is not None and codes is not None:
            local = self._local_codes(B, nbr, X.device)
            stats = self._assign_capped(X, None, coef, 1.0, self.emb[sl], D, idx_out, local,
                                        self._arange(B, X.device), training, count, slab, cap)
        else:
            stats = self._assign_capped(X, None, coef, 1.0, self.emb[sl], D, idx_out, codes,
                                        batch_idx, training, count, slab, cap)
        if comm is not None:
            stats = kernels.vq_ema_reduce(stats)
            comm.allreduce_(stats)
            if local is not None:
                self.sync_codes()           # the previous exchange lands before ours
                self._exchange_codes(batch_idx, local, codes, max_B)
        if training:
            kernels.vq_ema_finalize(stats, D, D, self.decay, self.warm_up_flag, 1.0, self.epsilon,
                                    self.cs[sl], self.ema_w[sl], self.emb[sl], self.emb_out[sl],
                                    self.rm_f[sl], self.rv_f[sl], self.rm_g[sl], self.rv_g[sl],
                                    self.bad_flag, count, zero_after=True)
            self._clean(D, b0, nbr)
            self._finish()

    def finish_update(self):
        """Complete an update(defer=True): wait for the EMA-statistics
        all-reduce (multi-GPU; a stream wait, not a host wait) and run the
        finalize.  A no-op when nothing is pending."""
        p, self._pending_finalize = self._pending_finalize, None
        if p is None:
            return
        work, fin_args, fin_kw, clean = p
        if work is not None:
            work.wait()
        kernels.vq_ema_finalize(*fin_args, **fin_kw)
        self._clean(*clean)
        self._finish()

    def take_fused_finalize(self):
        """Hand the pending finalize of an update(defer=True) to the caller's
        next aggregation, which runs it inside its fix-up launch
        (kernels.spmm_codebook(finalize=handle), include/vqgnn.h §6b)
        -> a FusedFinalize handle, or None when nothing is pending or when the
        finalize must wait for the multi-GPU all-reduce of its statistics
        (finish_update() then).  The finalize stays pending until the
        aggregation has queued it (handle.done(), which spmm_codebook calls):
        an aggregation that raises first leaves it to finish_update()."""
        p = self._pending_finalize
        if p is None or p[0] is not None:
            return None
        return FusedFinalize(self, p)

    def update(self, X, G, b0, nbr, training, idx_out=None, codes=None, batch_idx=None,
               defer=False, before_assign=None):
        """vq.py:204-279 for branches [b0, b0+nbr): X, G are [B, nbr*D] views.

        defer=True (training): return after the assign with the finalize
        pending (finish_update()); multi-GPU, the all-reduce of the EMA
        statistics is then asynchronous and overlaps what the caller queues
        before finish_update().  Until then emb / emb_out hold the codebook
        from before this update, as the reference's forward sees it (the
        hook's update runs after the aggregation, models.py:181-185).

        Multi-GPU, the previous update's code exchange is landed after this
        update's assign, just before its own codes are scattered (the assign
        reads no codes): the all_gather then overlaps the caller's gather +
        SpMM and this update's statistics and assign.

        before_assign: called after the BatchNorm launches, before the
        assign's -- where bench.py queues the aggregation's walk on a side
        stream (kernels.spmm_codebook_walk(deferred=True).launch), so the
        BatchNorm pass runs while the walk's launch crosses streams."""
        self.finish_update()
        exchanging = training and self.comm is not None and codes is not None
        if not exchanging:
            self.sync_codes()
        D, F = self.D, nbr * self.D
        sl = self._sel(b0, nbr)
        B = X.shape[0]
        inited = self.bn_inited[b0:b0 + nbr]
        if any(inited) != all(inited):
            raise RuntimeError("batched update() over branches with mixed bn_inited state")
        init = not inited[0]
        if training and B <= 1:
            raise ValueError("Expected more than 1 value per channel when training")
        comm = self.comm if training else None
        count = B
        mode = (BN_TRAIN_INIT if init else BN_TRAIN) if training else \
            (BN_EVAL_INIT if init else BN_EVAL)
        bn_args = (mode, 0.1, 1e-5, self.momentum, self.epsilon, self.epsilon, self.rm_f[sl],
                   self.rv_f[sl], self.rm_g[sl], self.rv_g[sl])
        bn_kw = dict(want_batch=True, nbt_f=self.nbt_f[sl] if training else None,
                     nbt_g=self.nbt_g[sl] if training else None, D=D)
        ax, ax_eval = self._arith(X, comm)
        ag, ag_eval = self._arith(G, comm)
        if comm is None and self._bn_fold(B, nbr, 2 * D, ax, ag):
            # one process, the finalize folded into the assign (the stash too)
            coef = kernels.bn_stats_partial(X, G, F, *bn_args, **bn_kw, arith_x=ax, arith_g=ag)
            batch = coef.batch
        elif comm is None:   # one process: statistics + finalize (the stash in every mode)
            coef, batch, _ = kernels.bn_stats_finalize(X, G, F, *bn_args, **bn_kw, arith_x=ax,
                                                       arith_g=ag,
                                                       ref_threads=self._threads())
        else:                  # multi-GPU: the global count rides in the sums
            sums = kernels.bn_stats(X, G, F, with_count=True)
            max_B = comm.allreduce_stats_(sums, B)
            count = comm.world * max_B      # row bound of the fixed-point shift
            coef, batch = kernels.bn_finalize(sums, 0, F, True, *bn_args, **bn_kw,
                                              arith_x=ax_eval, arith_g=ag_eval)
        for b in range(b0, b0 + nbr):
            self.bn_inited[b] = True
        self.last_batch = batch
        self.last_inputs = (X, G)
        scale = float(self.grad_normalize_scale[0])
        slab = self._slab(2 * D, b0, nbr) if training else None
        local = None
        cap = max_B if comm is not None else None
        if before_assign is not None:
            before_assign()
        if comm is not None and codes is not None:
            local = self._local_codes(B, nbr, X.device)
            stats = self._assign_capped(X, G, coef, scale, self.emb[sl], 2 * D, idx_out, local,
                                        self._arange(B, X.device), training, count, slab, cap)
        else:
            stats = self._assign_capped(X, G, coef, scale, self.emb[sl], 2 * D, idx_out, codes,
                                        batch_idx, training, count, slab, cap)
        work = None
        if comm is not None:
            stats = kernels.vq_ema_reduce(stats)
            if local is not None:
                self.sync_codes()           # the previous exchange lands before ours
            if defer:
                # the EMA all-reduce first: the finalize at the end of the
                # step waits for it, the codes only land in the next update
                # (both share one communicator's queue, so order matters)
                work = comm.allreduce_(stats, async_op=True)
                if local is not None:
                    self._exchange_codes(batch_idx, local, codes, max_B)
            else:
                comm.allreduce_(stats)
                if local is not None:
                    self._exchange_codes(batch_idx, local, codes, max_B)
        if training:
            fin_args = (stats, D, 2 * D, self.decay, self.warm_up_flag, scale, self.epsilon,
                        self.cs[sl], self.ema_w[sl], self.emb[sl], self.emb_out[sl],
                        self.rm_f[sl], self.rv_f[sl], self.rm_g[sl], self.rv_g[sl],
                        self.bad_flag, count)
            self._pending_finalize = (work, fin_args, dict(zero_after=True), (2 * D, b0, nbr))
            if not defer:
                self.finish_update()


class _BNView(nn.Module):
    """BatchNorm1d(affine=False) state view of one branch (vq.py:86-88).  Only
    the running statistics are state; normalisation runs inside the kernels."""

    def __init__(self, owner, which, num_features, eps, momentum):
        super().__init__()
        self.__dict__["_owner"] = owner
        self.__dict__["_which"] = which
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.affine, self.track_running_stats = False, True

    def _bank(self):
        return self._owner._get_bank()

    @property
    def running_mean(self):
        return getattr(self._bank(), "rm_" + self._which)[self._owner._branch]

    @property
    def running_var(self):
        return getattr(self._bank(), "rv_" + self._which)[self._owner._branch]

    @property
    def num_batches_tracked(self):
        return getattr(self._bank(), "nbt_" + self._which)[self._owner._branch]

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        destination[prefix + "running_mean"] = self.running_mean.detach().clone()
        destination[prefix + "running_var"] = self.running_var.detach().clone()
        destination[prefix + "num_batches_tracked"] = self.num_batches_tracked.detach().clone()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        for k in ("running_mean", "running_var", "num_batches_tracked"):
            if prefix + k in state_dict:
                with torch.no_grad():
                    getattr(self, k).copy_(state_dict[prefix + k])
            elif strict:
                missing_keys.append(prefix + k)

    def forward(self, x):  # pragma: no cover - never on the hot path
        raise NotImplementedError("normalisation is fused into the VQ kernels")


class VectorQuantizerEMA(nn.Module):
    """Reference: vq_gnn_v2/vq.py:60-279.  Same constructor, methods and buffer
    names.  ``_bank``/``_branch`` are internal: a LowRankGNNLayer passes its
    packed bank so that all branches share one launch."""

    def __init__(self, num_embeddings, embedding_dim, commitment_cost=0.5, decay=0.99,
                 epsilon=1e-24, grad_normalize_scale=(1, 1), warm_up_flag=False, momentum=0.1,
                 add_flag=False, _bank=None, _branch=0):
        super().__init__()
        if add_flag:
            raise NotImplementedError(
                "add_flag=True (2D+1 codebook) is unused on the v2 path: models.py:30 hard-codes "
                "add_flag = False")
        self.add_flag = add_flag
        self._embedding_dim = embedding_dim
        self._num_embeddings = num_embeddings
        self._commitment_cost = commitment_cost
        self._warm_up_flag = warm_up_flag
        self._decay = decay
        self._epsilon = epsilon
        self.grad_normalize_scale = grad_normalize_scale
        if type(self.grad_normalize_scale) is not list:   # vq.py:91-92
            raise ValueError('grad scale type wrong!')
        if _bank is None:
            self._own_bank = VQBank(1, num_embeddings, embedding_dim, decay, epsilon,
                                    grad_normalize_scale, warm_up_flag, momentum)
            self.__dict__["_shared_bank"] = None
            self._branch = 0
            self._own_bank.init_branch(0)
        else:
            self.__dict__["_shared_bank"] = _bank
            self._branch = int(_branch)
        self.batch_norm_feat = _BNView(self, "f", embedding_dim, 1e-5, 0.1)
        self.batch_norm_grad = _BNView(self, "g", embedding_dim, epsilon, momentum)
        self.mean = self.std = None
        self.running_mean = self.running_std = None

    # ---- state views -------------------------------------------------- #
    def _get_bank(self) -> VQBank:
        sb = self.__dict__.get("_shared_bank")
        return sb if sb is not None else self._own_bank

    @property
    def _embedding(self):
        return self._get_bank().emb[self._branch]

    @property
    def _embedding_output(self):
        return self._get_bank().emb_out[self._branch]

    @property
    def _ema_cluster_size(self):
        return self._get_bank().cs[self._branch]

    @property
    def _ema_w(self):
        return self._get_bank().ema_w[self._branch]

    @property
    def bn_inited(self):
        return self._get_bank().bn_inited[self._branch]

    @bn_inited.setter
    def bn_inited(self, v):
        self._get_bank().bn_inited[self._branch] = bool(v)

    _STATE = ("_embedding", "_embedding_output", "_ema_cluster_size", "_ema_w")

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        for k in self._STATE:
            destination[prefix + k] = getattr(self, k).detach().clone()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        for k in self._STATE:
            if prefix + k in state_dict:
                with torch.no_grad():
                    getattr(self, k).copy_(state_dict[prefix + k])
            elif strict:
                missing_keys.append(prefix + k)

    # ---- reference methods -------------------------------------------- #
    def feature_kmeans_init(self, kmeans_centroids, kmeans_counts):   # vq.py:102-105
        D = self._embedding_dim
        with torch.no_grad():
            self._embedding[:, :D] = kmeans_centroids
            self._ema_cluster_size.copy_(kmeans_counts)
            self._ema_w[:, :D] = kmeans_centroids * kmeans_counts.unsqueeze(1)

    def kmeans_init(self, kmeans_centroids, kmeans_counts):            # vq.py:108-118
        D = self._embedding_dim
        s0 = self.grad_normalize_scale[0]
        with torch.no_grad():
            self._embedding.copy_(kmeans_centroids)
            self._ema_cluster_size.copy_(kmeans_counts)
            self._ema_w.copy_(kmeans_centroids * kmeans_counts.unsqueeze(1))
            self._embedding[:, D:2 * D] *= s0
            self._ema_w[:, D:2 * D] *= s0

    def get(self):                                                     # vq.py:120-121
        return self._embedding_output

    def get_codebook(self):                                            # vq.py:123-124
        return self._embedding_output[:, :self._embedding_dim]

    def get_grad(self):                                                # vq.py:126-127
        return self._embedding_output[:, self._embedding_dim:]

    def get_feat_cen_norm(self):                                       # vq.py:129-131
        return torch.norm(torch.mean(self._embedding[:, :self._embedding_dim], dim=0)).item()

    def get_grad_cen_norm(self):                                       # vq.py:133-135
        return torch.norm(torch.mean(self._embedding[:, self._embedding_dim:], dim=0)).item()

    def feature_update(self, X_B):                                     # vq.py:160-202
        bank = self._get_bank()
        idx = torch.empty(X_B.shape[0], 1, dtype=torch.long, device=X_B.device)
        bank.feature_update(X_B, self._branch, 1, self.training, idx_out=idx.view(1, -1))
        return idx

    def update(self, X_B, grad):                                       # vq.py:204-279
        bank = self._get_bank()
        B = X_B.shape[0]
        idx = torch.empty(B, 1, dtype=torch.long, device=X_B.device)
        bank.update(X_B, grad, self._branch, 1, self.training, idx_out=idx.view(1, -1))
        self._stash_update_logs(bank, 0, X_B, grad)
        # The dense [B, M] one-hot of the reference is returned as a sparse COO
        # tensor (same values; .to_dense() reproduces it) instead of 4*B*M bytes.
        ones = torch.ones(B, dtype=torch.float32, device=X_B.device)
        rows = torch.arange(B, device=X_B.device)
        encodings = torch.sparse_coo_tensor(torch.stack([rows, idx[:, 0]]), ones,
                                            (B, self._num_embeddings))
        return idx, encodings

    def _stash_update_logs(self, bank, local_b, X_B, grad):
        D = self._embedding_dim
        batch = bank.last_batch          # [4, nbr*D]
        sl = slice(local_b * D, (local_b + 1) * D)
        self.mean = torch.cat([batch[0, sl], batch[2, sl]]).unsqueeze(0)
        self.std = torch.cat([batch[1, sl], batch[3, sl]]).unsqueeze(0)
        self.__dict__["_zero_rate_src"] = (X_B[:, 0], grad[:, 0], self.std, X_B.shape[0])
        if self.training:
            b = self._branch
            rv = torch.cat([bank.rv_f[b] + 1e-5, bank.rv_g[b] + self._epsilon])
            self.running_std = torch.sqrt(rv).unsqueeze(0)
            self.running_mean = torch.cat([bank.rm_f[b], bank.rm_g[b]]).unsqueeze(0)

    # logging-only attributes of vq.py:213-214, computed on access
    @property
    def feat_zero_rate(self):
        src = self.__dict__.get("_zero_rate_src")
        if src is None:
            return None
        x0, _, std, B = src
        return torch.sum(torch.abs(x0) < std[0][0] * 1e-5) / B

    @property
    def grad_zero_rate(self):
        src = self.__dict__.get("_zero_rate_src")
        if src is None:
            return None
        _, g0, std, B = src
        return torch.sum(g0 < std[0][self._embedding_dim] * 1e-5) / B
