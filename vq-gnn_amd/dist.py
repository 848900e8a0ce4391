"""Data-parallel codebook consistency across GPUs (no counterpart in the
reference, which is single-process: vq_gnn_v2/main_node.py:186-187).

Each rank processes its own mini-batch (weak scaling).  Per VQ step the only
exchange is:
  1. all-reduce of the BatchNorm sufficient statistics  (fp64 [4, F])
  2. all-reduce of the EMA sufficient statistics          (int64 fixed point
     [nb, M, W+1], include/vqgnn.h §3: the sum is exact)
  3. all-gather of (batch_idx, codes) so every replica's c_indices agree
so every rank then runs the identical finalize and holds identical codebooks.
The union-batch semantics: N ranks with batches B_1..B_N produce the
statistics of one GPU on the concatenated batch — the EMA statistic exactly,
the BN sums up to fp64 summation order.
Backend "nccl" is RCCL on ROCm (xGMI); "gloo" runs the same code in the CPU
tests.  Codes travel as bytes: RCCL has no 16-bit integer type.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import kernels


class CodebookSync:
    """capacity: an upper bound of every rank's batch rows B (e.g. the loader's
    batch size, OurDataLoader.max_batch_rows()).  With it an update issues no
    host-side collective: the global row count travels inside the BatchNorm
    all-reduce (bn_stats(with_count=True)), the fixed-point shift of the EMA
    statistic uses world * capacity as its row bound, and the code exchange
    pads to capacity rows.  Without it every update first agrees on max(B)
    with one blocking all-reduce (correct for any batch sizes, but a host
    round trip per call).

    Exactness: the EMA statistic is an exact int64 sum at every world size,
    but its fixed-point resolution follows the row bound (world * capacity,
    or world * max(B)), so the codebooks are bit-identical to one process on
    the union batch only when that bound equals the one process's row count
    (capacity == every rank's B); otherwise they differ by the rounding of
    the normalised values to the coarser grid (include/vqgnn.h §3), within
    the EMA tolerance the tests use."""

    def __init__(self, group=None, count_group=None, capacity=None, direct=None):
        self.group = group
        # host-integer collectives (max B when no capacity is given) run over a
        # CPU (gloo) group when given, so the device stream never syncs for them
        self.count_group = count_group
        self.world = dist.get_world_size(group)
        self.capacity = None if capacity is None else int(capacity)
        self._overflow = None  # reduced over-capacity flags not yet read (allreduce_stats_)
        self._wire = {}       # persistent code-exchange buffers per shape
        self._inflight = {}   # buffer key -> the PendingWire still reading them
        self._epoch = {}      # buffer key -> exchanges issued on its winner table
        # RCCL called directly on chosen streams (rccl.py): the default on the
        # nccl backend (VQGNN_DIRECT_RCCL=0: through torch.distributed)
        if direct is None:
            direct = (dist.get_backend(group) == "nccl"
                      and os.environ.get("VQGNN_DIRECT_RCCL", "1") != "0")
        self._direct = bool(direct)
        if self._direct:
            self._init_direct()

    def _init_direct(self):
        """Two communicators over the world: A on the compute stream (the
        BatchNorm all-reduce, in order), B on one side stream (the EMA
        all-reduce and the code all-gather, overlapping the caller's work).
        Rank 0's unique ids travel over the gloo count group."""
        import weakref

        from . import rccl
        bgroup = self.count_group or self.group
        if dist.get_world_size(bgroup) != self.world:
            raise ValueError("CodebookSync: count_group must span the ranks of group")
        # broadcast_object_list takes a GLOBAL source rank: the global rank of
        # the broadcast group's rank 0, which creates the ids
        src = dist.get_global_rank(bgroup, 0) if bgroup is not None else 0
        ids = [rccl.unique_id(), rccl.unique_id()] if dist.get_rank(bgroup) == 0 else None
        box = [ids]
        dist.broadcast_object_list(box, src=src, group=bgroup)
        rank = dist.get_rank(self.group)
        self._ca = rccl.Communicator(self.world, rank, box[0][0])
        self._cb = rccl.Communicator(self.world, rank, box[0][1])
        self._side = torch.cuda.Stream()
        # reused events (creating one per collective costs host time): an
        # event is re-recorded only after its StreamWork was waited on (at
        # most 2 exchanges + 2 all-reduces are in flight at once)
        self._events = [torch.cuda.Event() for _ in range(16)]
        self._ev_i = 0
        # no strong reference from an exit hook: a dropped CodebookSync frees
        # its communicators and side stream at once
        # close() flips the flag: only a clean shutdown destroys (which flushes
        # and can wait on a peer); any other release aborts
        self._clean = [False]
        self._finalizer = weakref.finalize(self, _release_comms, self._ca, self._cb, self._clean)

    def close(self):
        """Destroy the direct communicators after this rank's work drained
        (call on every rank at a clean shutdown).  Without it they are
        released when the object is collected or at exit by ncclCommAbort
        (whatever the exit path: an uncaught exception, sys.exit from a
        handler, a failing thread), so a rank whose peer died mid-collective
        exits instead of hanging in a destroy."""
        if getattr(self, "_finalizer", None) is not None and self._finalizer.alive:
            torch.cuda.synchronize()
            self._clean[0] = True
            self._finalizer()
        self._ca = self._cb = None

    def _on_side(self, launch):
        """Run ``launch(side_stream)`` after the current stream's work so far;
        -> the StreamWork the current stream waits on later."""
        from . import rccl
        ev0, ev1 = self._events[self._ev_i], self._events[self._ev_i + 1]
        self._ev_i = (self._ev_i + 2) % len(self._events)
        ev0.record(torch.cuda.current_stream())
        self._side.wait_event(ev0)
        launch(self._side)
        ev1.record(self._side)
        return rccl.StreamWork(ev1)

    def allreduce_(self, t: torch.Tensor, async_op: bool = False):
        """In-place sum over the ranks; async_op=True returns the work (its
        wait() orders the current stream after the collective).  Direct RCCL:
        synchronous calls run in order on the compute stream, asynchronous
        ones on the side stream (tensors must stay alive until wait())."""
        if self._direct:
            if not async_op:
                self._ca.all_reduce_(t, torch.cuda.current_stream())
                return None
            return self._on_side(lambda s: self._cb.all_reduce_(t, s))
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)

    def rows_per_rank(self, B: int) -> int:
        """The per-rank row bound every rank agrees on: capacity, or max(B)
        over the ranks (one blocking collective) when no capacity is set."""
        if self.capacity is not None:
            if B > self.capacity:
                raise ValueError(f"batch of {B} rows exceeds CodebookSync capacity "
                                 f"{self.capacity}")
            return self.capacity
        return self.global_max(B)

    def allreduce_stats_(self, sums: torch.Tensor, B: int) -> int:
        """All-reduce the fp64 BatchNorm sums in place ([4F + 2]: the row count
        at 4F, read on the device by bn_finalize(count=0), and at 4F + 1 the
        number of ranks whose batch exceeds ``capacity``) -> the per-rank row
        bound.  A rank over capacity does not raise here (the other ranks
        would wait in this collective forever): the flag travels with the
        sums, so every rank raises together at the next 'Bad Init!' check
        (take_overflow), after the update's collectives all completed."""
        if self.capacity is not None and B > self.capacity:
            sums[-1:].fill_(1.0)
        self.allreduce_(sums)
        if self.capacity is not None:
            # the reduced flag stays in the sums; read at the next check (no
            # device op here: a torch launch right after the collective costs
            # ~140 us of host time)
            if self._overflow is None:
                self._overflow = []
            self._overflow.append(sums[-1:])
            if len(self._overflow) >= 64:     # bounded: fold once per 64 updates
                self._overflow = [torch.cat(self._overflow).sum(0, keepdim=True)]
            return self.capacity
        return self.global_max(B)

    def take_overflow(self) -> bool:
        """True (on every rank alike) when some rank's batch exceeded capacity
        in an update since the last call; one device read."""
        if not self._overflow:
            return False
        flags, self._overflow = self._overflow, []
        return float(torch.cat(flags).sum().item()) > 0

    def global_count(self, B: int) -> int:
        """Sum of B over the ranks (a blocking host collective; not on the
        update path, which carries the count in the BatchNorm all-reduce)."""
        t = torch.tensor([B], dtype=torch.int64)
        if self.count_group is not None:
            dist.all_reduce(t, group=self.count_group)
            return int(t.item())
        dev = t.to(_device_of(self.group))
        dist.all_reduce(dev, group=self.group)
        return int(dev.item())

    @staticmethod
    def _wire_dtype(M):
        return torch.uint8 if M <= 256 else torch.int16

    def gather_codes(self, batch_idx: torch.Tensor, local: torch.Tensor,
                     max_B: int | None = None, M: int = 32767, async_op: bool = False):
        """All ranks' (batch_idx, local codes), padded to max_B rows per rank
        (padding: batch_idx = -1).  Wire format: node ids int32, codes uint8
        when M <= 256 (else int16), both as bytes (RCCL has no 16-bit ints).
        -> (pending, idx [world*max_B] int32, codes [world*max_B, nb] wire
        dtype); ``pending`` is a list of async works (empty if not async_op)."""
        B, nb = local.shape
        if max_B is None:
            max_B = self.global_max(B)
        dev = local.device
        wd = self._wire_dtype(M)
        pad_idx = torch.full((max_B,), -1, dtype=torch.int32, device=dev)
        pad_idx[:B] = batch_idx
        pad_loc = torch.zeros(max_B, nb, dtype=wd, device=dev)
        pad_loc[:B] = local
        all_idx = torch.empty(self.world, max_B, dtype=torch.int32, device=dev)
        all_loc = torch.empty(self.world, max_B, nb, dtype=wd, device=dev)
        w1 = dist.all_gather(list(all_idx.unbind(0)), pad_idx, group=self.group,
                             async_op=async_op)
        w2 = dist.all_gather(list(all_loc.view(torch.uint8).unbind(0)),
                             pad_loc.view(torch.uint8), group=self.group, async_op=async_op)
        pending = [w for w in (w1, w2) if w is not None] if async_op else []
        return pending, all_idx.view(-1), all_loc.view(-1, nb)

    def allgather_codes_(self, batch_idx: torch.Tensor, local: torch.Tensor,
                         codes: torch.Tensor, max_B: int | None = None, M: int = 32767) -> None:
        """Scatter every rank's (batch_idx, local codes) into ``codes`` (HIP)."""
        _, all_idx, all_loc = self.gather_codes(batch_idx, local, max_B, M)
        kernels.scatter_codes(all_idx.to(torch.int64), all_loc.to(torch.int16), codes)

    def start_codes_exchange(self, batch_idx, local, codes, max_B=None, M=32767):
        """Asynchronous code exchange on the device (include/vqgnn.h §5b): the
        rank's rows packed into a persistent send buffer (and scattered into
        its own ``codes`` at once), one all_gather_into_tensor, and a
        PendingCodes whose wait() scatters every rank's records with "the
        last record wins" for repeated nodes (the same on every replica).
        Call wait() before ``codes`` is next read for other ranks' nodes."""
        B, nb = local.shape
        if max_B is None:
            max_B = self.global_max(B)
        key = (max_B, nb, M, codes.shape[0], str(local.device))
        # an exchange still in flight on these buffers (another bank of the
        # same shape) is landed first: its all_gather reads `send` and its
        # scatter reads `recv`
        prev = self._inflight.pop(key, None)
        if prev is not None:
            prev.wait()
        send, recv, winner = self._wire_buffers(key)
        epoch = self._epoch.get(key, 0) + 1
        if epoch >= (1 << 31):              # stamps are epoch << 32 | record: restart
            winner.zero_()
            epoch = 1
        self._epoch[key] = epoch
        kernels.pack_codes(batch_idx, local, M, max_B, send, codes=codes)
        if self._direct:
            work = self._on_side(lambda s: self._cb.all_gather(send, recv, s))
        else:
            work = dist.all_gather_into_tensor(recv, send, group=self.group, async_op=True)
        pend = PendingWire(work, recv, self.world * max_B, nb, M, winner, codes, epoch)
        self._inflight[key] = pend
        return pend

    def _wire_buffers(self, key):
        max_B, nb, M, N, device = key
        buf = self._wire.get(key)
        if buf is None:
            rec = kernels.codes_wire_record(nb, M)
            send = torch.empty(max_B * rec, dtype=torch.uint8, device=device)
            recv = torch.empty(self.world * max_B * rec, dtype=torch.uint8, device=device)
            # stamp table of the scatter's "last record wins" (int64, never reset)
            winner = torch.zeros(N, dtype=torch.int64, device=device)
            buf = self._wire[key] = (send, recv, winner)
        return buf


    def global_max(self, B: int) -> int:
        t = torch.tensor([B], dtype=torch.int64)
        if self.count_group is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.count_group)
            return int(t.item())
        dev = t.to(_device_of(self.group))
        dist.all_reduce(dev, op=dist.ReduceOp.MAX, group=self.group)
        return int(dev.item())


class PendingCodes:
    def __init__(self, works, all_idx, all_loc, codes):
        self.works, self.all_idx, self.all_loc, self.codes = works, all_idx, all_loc, codes

    def wait(self):
        for w in self.works:
            w.wait()
        kernels.scatter_codes(self.all_idx.to(torch.int64), self.all_loc.to(torch.int16),
                              self.codes)
        self.works = []

class PendingWire:
    """An in-flight all_gather of packed code records (start_codes_exchange)."""

    def __init__(self, work, recv, n_records, nb, M, winner, codes, epoch):
        self.work, self.recv, self.n, self.nb, self.M = work, recv, n_records, nb, M
        self.winner, self.codes, self.epoch = winner, codes, epoch

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
            kernels.scatter_wire(self.recv, self.n, self.nb, self.M, self.winner, self.codes,
                                 self.epoch)


def _release_comms(ca, cb, clean):
    """Finalizer of CodebookSync's direct communicators: destroy them only
    after close() drained this rank's work (clean[0]); on any other release
    -- collection or interpreter exit without close(), on any error path --
    a collective may still wait for a peer that will never come, so abort
    them (ncclCommAbort does not wait)."""
    for c in (ca, cb):
        if c is not None:
            c.destroy() if clean[0] else c.abort()


def _device_of(group):
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")
