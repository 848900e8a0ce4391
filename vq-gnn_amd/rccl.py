"""Direct RCCL communicators for the codebook exchange (dist.CodebookSync).

torch.distributed's ProcessGroupNCCL runs every collective on its own
internal stream, so each call costs two cross-queue event hops on the
device (compute stream -> NCCL stream -> compute stream) plus the process
group's host bookkeeping.  In the one-rank rehearsal of the bench step those
hops and the host work took 65-115 us per step against a 0.225 ms step
(DESIGN.md §6).  Here a collective is one ``ncclAllReduce`` /
``ncclAllGather`` call enqueued on a HIP stream the caller chooses:

- the BatchNorm all-reduce, which the assign needs at once, runs in order on
  the compute stream (no hop at all);
- the EMA-statistics all-reduce and the code all-gather, which overlap the
  caller's gather + SpMM, run on a second communicator bound to one side
  stream (one communicator per stream, so every rank issues each
  communicator's collectives in the same order on one stream -- RCCL's
  ordering rule);

The library is the RCCL that torch itself loaded (torch/lib/librccl.so), so
one RCCL and one HIP runtime live in the process.  The unique id travels over
the gloo count group.
"""
from __future__ import annotations

import ctypes
import os

import torch

NCCL_UNIQUE_ID_BYTES = 128
_SUM = 0
_DTYPES = {torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float32: 7, torch.float64: 8}


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_ubyte * NCCL_UNIQUE_ID_BYTES)]   # ubyte: no NUL truncation


_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not os.path.exists(path):
            path = "librccl.so"
        L = ctypes.CDLL(path)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), i, _UniqueId, i]
        L.ncclAllReduce.argtypes = [vp, vp, sz, i, i, vp, vp]
        L.ncclAllGather.argtypes = [vp, vp, sz, i, vp, vp]
        L.ncclCommDestroy.argtypes = [vp]
        L.ncclCommAbort.argtypes = [vp]
        L.ncclGetErrorString.argtypes = [i]
        L.ncclGetErrorString.restype = ctypes.c_char_p
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclAllGather",
                  "ncclCommDestroy", "ncclCommAbort"):
            getattr(L, f).restype = i
        _LIB = L
    return _LIB


def _check(rc, what):
    if rc != 0:
        msg = _lib().ncclGetErrorString(rc)
        raise RuntimeError(f"{what}: RCCL error {rc} ({msg.decode() if msg else '?'})")


def unique_id() -> bytes:
    uid = _UniqueId()
    _check(_lib().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    return bytes(uid.internal)


class Communicator:
    """One RCCL communicator over the ranks of the job (all GPUs of the
    world), created on the current HIP device."""

    def __init__(self, world: int, rank: int, uid: bytes):
        if len(uid) != NCCL_UNIQUE_ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        u = _UniqueId()
        ctypes.memmove(u.internal, uid, NCCL_UNIQUE_ID_BYTES)
        comm = ctypes.c_void_p()
        _check(_lib().ncclCommInitRank(ctypes.byref(comm), int(world), u, int(rank)),
               "ncclCommInitRank")
        self.comm, self.world, self.rank = comm, world, rank

    @staticmethod
    def _dtype(t: torch.Tensor) -> int:
        dt = _DTYPES.get(t.dtype)
        if dt is None:
            raise TypeError(f"RCCL collective: unsupported dtype {t.dtype}")
        return dt

    def all_reduce_(self, t: torch.Tensor, stream: torch.cuda.Stream) -> None:
        """In-place sum of a contiguous device tensor, enqueued on ``stream``."""
        if not t.is_contiguous():
            raise ValueError("RCCL all-reduce needs a contiguous tensor")
        _check(_lib().ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), self._dtype(t), _SUM,
                                    self.comm, stream.cuda_stream), "ncclAllReduce")

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor,
                   stream: torch.cuda.Stream) -> None:
        """recv[r * n: (r + 1) * n] = rank r's send (n = send.numel()), on ``stream``."""
        if not (send.is_contiguous() and recv.is_contiguous()):
            raise ValueError("RCCL all-gather needs contiguous tensors")
        if recv.numel() != send.numel() * self.world or recv.dtype != send.dtype:
            raise ValueError("RCCL all-gather: recv must be world x send")
        _check(_lib().ncclAllGather(send.data_ptr(), recv.data_ptr(), send.numel(),
                                    self._dtype(send), self.comm, stream.cuda_stream),
               "ncclAllGather")

    def destroy(self):
        """ncclCommDestroy: waits for this communicator's outstanding
        collectives (a clean shutdown)."""
        if self.comm:
            _lib().ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()

    def abort(self):
        """ncclCommAbort: frees the communicator without waiting for its
        outstanding collectives (an error exit whose peers may be gone)."""
        if self.comm:
            _lib().ncclCommAbort(self.comm)
            self.comm = ctypes.c_void_p()


class StreamWork:
    """An asynchronous collective on a side stream: wait() orders the current
    stream after it (a device-side wait on an event, no host sync)."""

    def __init__(self, event: torch.cuda.Event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)
