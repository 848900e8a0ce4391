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

import torch
import torch.distributed as dist

from . import kernels


class CodebookSync:
    def __init__(self, group=None, count_group=None):
        self.group = group
        # row counts are host integers: summed over a CPU (gloo) group when
        # given, so the device stream never syncs for them
        self.count_group = count_group
        self.world = dist.get_world_size(group)
        self._count_cache = {}

    def allreduce_(self, t: torch.Tensor) -> None:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def global_count(self, B: int) -> int:
        if B in self._count_cache:
            return self._count_cache[B]
        t = torch.tensor([B], dtype=torch.int64)
        if self.count_group is not None:
            dist.all_reduce(t, group=self.count_group)
            total = int(t.item())
        else:
            dev = t.to(_device_of(self.group))
            dist.all_reduce(dev, group=self.group)
            total = int(dev.item())
        return total

    def cache_count(self, B: int, total: int) -> None:
        """Fixed batches (bench): remember the global count for this local B."""
        self._count_cache[B] = total

    def gather_codes(self, batch_idx: torch.Tensor, local: torch.Tensor,
                     max_B: int | None = None):
        """All ranks' (batch_idx, local codes), padded to max_B rows per rank
        (padding: batch_idx = -1).  -> (idx [world*max_B] int64,
        codes [world*max_B, nb] int16), on local's device."""
        B, nb = local.shape
        if max_B is None:
            max_B = self.global_max(B)
        dev = local.device
        pad_idx = torch.full((max_B,), -1, dtype=torch.int64, device=dev)
        pad_idx[:B] = batch_idx
        pad_loc = torch.zeros(max_B, nb, dtype=torch.int16, device=dev)
        pad_loc[:B] = local
        all_idx = torch.empty(self.world, max_B, dtype=torch.int64, device=dev)
        all_loc = torch.empty(self.world, max_B, nb, dtype=torch.int16, device=dev)
        dist.all_gather(list(all_idx.unbind(0)), pad_idx, group=self.group)
        dist.all_gather(list(all_loc.view(torch.uint8).unbind(0)),
                        pad_loc.view(torch.uint8), group=self.group)
        return all_idx.view(-1), all_loc.view(-1, nb)

    def allgather_codes_(self, batch_idx: torch.Tensor, local: torch.Tensor,
                         codes: torch.Tensor, max_B: int | None = None) -> None:
        """Scatter every rank's (batch_idx, local codes) into ``codes`` (HIP)."""
        all_idx, all_loc = self.gather_codes(batch_idx, local, max_B)
        kernels.scatter_codes(all_idx, all_loc, codes)

    def global_max(self, B: int) -> int:
        t = torch.tensor([B], dtype=torch.int64)
        if self.count_group is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.count_group)
            return int(t.item())
        dev = t.to(_device_of(self.group))
        dist.all_reduce(dev, op=dist.ReduceOp.MAX, group=self.group)
        return int(dev.item())


def _device_of(group):
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")
