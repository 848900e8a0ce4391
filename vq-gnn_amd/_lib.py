"""ctypes binding of the vqgnn C-ABI (include/vqgnn.h) — the only door from the
Python host layer into the HIP kernels.

There is deliberately no CPU fallback: every product op goes through
``libvqgnn.so``; if the library is missing or cannot be loaded, ``lib()``
raises.  Tensors are passed as raw device pointers; every call is queued on
``torch.cuda.current_stream()``.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_HERE, "lib", "libvqgnn.so")
LIB_PATH = os.environ.get("VQGNN_LIB", _DEFAULT_LIB)

_c_void_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_size = ctypes.c_size_t



class EmaFinalizeArgs(ctypes.Structure):
    """include/vqgnn.h §4b vqgnn_ema_finalize_args (C layout and order)."""
    _fields_ = [
        ("ema_parts", _c_void_p), ("nparts", _i32), ("zero_after", _i32),
        ("stat_count", _i64),
        ("nb", _i32), ("M", _i32), ("D", _i32), ("W", _i32), ("ldw", _i32),
        ("decay", _f32), ("laplace", _i32), ("grad_scale", _f32), ("epsilon", _f32),
        ("cluster_size", _c_void_p), ("cs_bstride", _i64),
        ("ema_w", _c_void_p), ("embedding", _c_void_p), ("embedding_output", _c_void_p),
        ("emb_bstride", _i64),
        ("rm_f", _c_void_p), ("rv_f", _c_void_p), ("rm_g", _c_void_p), ("rv_g", _c_void_p),
        ("bad_init", _c_void_p),
    ]


# name -> (restype, argtypes); mirrors include/vqgnn.h one to one.
SIGNATURES = {
    "vqgnn_last_error": (ctypes.c_char_p, []),
    "vqgnn_version": (ctypes.c_int, []),
    "vqgnn_bn_stats_workspace": (_size, [_i32, _i32]),
    "vqgnn_bn_stats": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _i64, _i32, _i32, _i32,
                                      _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_bn_stats_count": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _i64, _i32, _i32, _i32,
                                      _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_bn_finalize": (ctypes.c_int, [_c_void_p, _i64, _i32, _i32, _i32, _i32, _i32, _f64,
                                         _f64, _f64, _f64, _f64, _c_void_p, _c_void_p,
                                         _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                         _c_void_p, _i32, _c_void_p]),
    "vqgnn_vq_stat_shifts": (None, [_i64, _f32, _c_void_p, _c_void_p]),
    "vqgnn_vq_ema_parts": (_i32, [_i32, _i32, _i32, _i32]),
    "vqgnn_vq_assign_workspace": (_size, [_i32, _i32, _i32, _i32]),
    "vqgnn_vq_ema_reduce": (ctypes.c_int, [_c_void_p, _i32, _i64, _c_void_p, _c_void_p]),
    "vqgnn_vq_assign": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _i64, _i32, _i32, _i32,
                                       _i32, _i32, _c_void_p, _f32, _c_void_p, _i32, _i64,
                                       _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p,
                                       _i32, _i64, _c_void_p, _c_void_p]),
    "vqgnn_vq_assign_bn_supported": (_i32, [_i32, _i32, _i32, _i32, _i32]),
    "vqgnn_bn_stats_partial": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _i64, _i32, _i32, _i32,
                                              _c_void_p, _c_void_p]),
    "vqgnn_vq_assign_bn": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _i64, _i32, _i32, _i32,
                                          _i32, _i32, _f32, _c_void_p, _i32, _i64, _c_void_p,
                                          _c_void_p, _i64, _c_void_p, _c_void_p, _i32, _i64,
                                          _c_void_p, _c_void_p, _i32, _i32, _i32, _f64, _f64,
                                          _f64, _f64, _f64, _c_void_p, _c_void_p, _c_void_p,
                                          _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                          _c_void_p, _i32, _c_void_p]),
    "vqgnn_vq_ema_finalize": (ctypes.c_int, [_c_void_p, _i32, _i32, _i64, _i32, _i32, _i32, _i32,
                                             _i32, _f32,
                                             _i32, _f32, _f32, _c_void_p, _i64, _c_void_p,
                                             _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p,
                                             _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_gather_codewords": (ctypes.c_int, [_c_void_p, _i32, _i32, _c_void_p, _i64, _i64,
                                              _i32, _i32, _c_void_p, _i32, _i32, _i32, _i64,
                                              _i32, _c_void_p, _i64, _c_void_p, _c_void_p]),
    "vqgnn_scatter_codes": (ctypes.c_int, [_c_void_p, _i32, _c_void_p, _i32, _c_void_p, _i64,
                                           _c_void_p]),
    "vqgnn_spmm_task_size": (_i64, [_i64, _i32, _i32]),
    "vqgnn_spmm_task_plan": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i32, _i64, _i32,
                                            _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_spmm_task_records": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i32, _i64,
                                               _c_void_p, _c_void_p]),
    "vqgnn_spmm_task_workspace": (_size, [_i64, _i32, _i32]),
    "vqgnn_spmm_task": (ctypes.c_int, [_c_void_p, _i32, _i32, _i64, _i32, _c_void_p, _i64,
                                       _c_void_p, _i64, _i32, _c_void_p, _i64, _c_void_p,
                                       _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p]),
    "vqgnn_spmm_task_records_cb": (ctypes.c_int, [_c_void_p, _i64, _i32, _c_void_p, _i32, _i64,
                                                  _c_void_p]),
    "vqgnn_spmm_task_cb_lds": (_size, [_i32]),
    "vqgnn_spmm_task_cb_supported": (_i32, [_i32, _i32, _i64, _i32, _i64, _i64, _i64, _i32,
                                            _i32, _i32]),
    "vqgnn_spmm_task_cb": (ctypes.c_int, [_c_void_p, _i32, _i64, _i32, _c_void_p, _i64, _i32,
                                          _c_void_p, _i64, _i64, _c_void_p, _i64, _i64, _i32,
                                          _i32, _i32, _c_void_p, _i64, _c_void_p, _c_void_p,
                                          _i32, _i32, _i32, _c_void_p, _c_void_p]),
    "vqgnn_spmm_task_cb_fin": (ctypes.c_int, [_c_void_p, _i32, _i64, _i32, _c_void_p, _i64, _i32,
                                              _c_void_p, _i64, _i64, _c_void_p, _i64, _i64, _i32,
                                              _i32, _i32, _c_void_p, _i64, _c_void_p, _c_void_p,
                                              _i32, _i32, _i32, _c_void_p,
                                              ctypes.POINTER(EmaFinalizeArgs), _c_void_p]),
    "vqgnn_spmm_task_cb_walk": (ctypes.c_int, [_c_void_p, _i32, _i64, _i32, _c_void_p, _i64,
                                               _i32, _c_void_p, _i64, _i64, _c_void_p, _i64, _i64,
                                               _i32, _i32, _i32, _c_void_p, _i64, _c_void_p,
                                               _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p]),
    "vqgnn_spmm_task_cb_fixup": (ctypes.c_int, [_c_void_p, _i32, _i64, _i32, _c_void_p, _i64,
                                                _i32, _c_void_p, _i64, _i64, _c_void_p, _i64, _i64,
                                                _i32, _i32, _i32, _c_void_p, _i64, _c_void_p,
                                                _c_void_p, _i32, _i32, _i32, _c_void_p,
                                                ctypes.POINTER(EmaFinalizeArgs), _c_void_p]),
    "vqgnn_gat_att_grad_workspace": (_size, [_i32, _i32, _i32]),
    "vqgnn_gat_att_grad": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _i64, _i32, _i32, _i32,
                                          _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                          _c_void_p, _c_void_p]),
    "vqgnn_gat_spmm_task": (ctypes.c_int, [_c_void_p, _i32, _i32, _i64, _i32, _c_void_p, _i64,
                                           _c_void_p, _i64, _i32, _c_void_p, _i64, _c_void_p,
                                           _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p,
                                           _c_void_p, _f32, _i32, _c_void_p,
                                           _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_csr_transpose_workspace": (_size, [_i32, _i32, _i64]),
    "vqgnn_csr_transpose": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i64,
                                           _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                           _c_void_p, _c_void_p]),
    "vqgnn_csr_expand_rows": (ctypes.c_int, [_c_void_p, _i32, _i64, _c_void_p, _c_void_p]),
    "vqgnn_gat_alpha_workspace": (_size, [_i32]),
    "vqgnn_gat_alpha": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _i64, _i32, _i32, _i32, _i32,
                                       _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                       _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_gat_coef": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i32, _i64, _c_void_p,
                                      _c_void_p, _f32, _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_gat_normalize": (ctypes.c_int, [_c_void_p, _i64, _i32, _i32, _c_void_p, _f32,
                                           _c_void_p]),
    "vqgnn_gat_edge_grad": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _i64,
                                           _c_void_p, _i64, _i32, _i32, _c_void_p, _i64,
                                           _c_void_p, _c_void_p, _c_void_p, _c_void_p, _f32,
                                           _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_bn_stats_finalize": (ctypes.c_int, [_c_void_p, _i64, _c_void_p, _i64, _i32, _i32, _i32,
                                               _c_void_p, _i32, _i32, _i32, _i32, _f64, _f64,
                                               _f64, _f64, _f64, _c_void_p, _c_void_p,
                                               _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                               _c_void_p, _c_void_p, _i32, _c_void_p,
                                               _c_void_p]),
    # §9 mini-batch construction
    "vqgnn_khop_workspace": (_size, [_i64]),
    "vqgnn_khop_subset": (ctypes.c_int, [_c_void_p, _c_void_p, _i64, _c_void_p, _i32, _i32, _i32,
                                         _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                         _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_khop_edges_workspace": (_size, [_i64, _i64]),
    "vqgnn_khop_edges": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p,
                                        _c_void_p, _i64, _i64, _i32, _i32, _i32, _c_void_p, _i64,
                                        _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    # §10 full-graph preprocessing
    "vqgnn_norm_adj_workspace": (_size, [_i64]),
    "vqgnn_norm_adj": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _i32, _c_void_p,
                                      _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_to_symmetric_workspace": (_size, [_i64, _i64]),
    "vqgnn_to_symmetric": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _i64, _c_void_p,
                                          _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_csr_permute_workspace": (_size, [_i64, _i64]),
    "vqgnn_csr_permute": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _i64, _c_void_p,
                                         _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                         _c_void_p]),
    "vqgnn_partition_workspace": (_size, [_i64]),
    "vqgnn_partition": (ctypes.c_int, [_c_void_p, _c_void_p, _i64, _i32, _c_void_p, _c_void_p,
                                       _c_void_p, _c_void_p, _c_void_p]),
    # §5a measurement
    "vqgnn_assign_timing": (ctypes.c_int, [_i32]),
    "vqgnn_assign_timing_read": (_i32, [_c_void_p, _i32]),
    # §5b multi-GPU code exchange
    "vqgnn_codes_wire_record": (_i32, [_i32, _i32]),
    "vqgnn_pack_codes": (ctypes.c_int, [_c_void_p, _i32, _c_void_p, _i32, _i32, _i32, _c_void_p,
                                        _c_void_p, _i64, _c_void_p]),
    "vqgnn_scatter_wire": (ctypes.c_int, [_c_void_p, _i64, _i32, _i32, _c_void_p, _i64, _i64,
                                          _c_void_p, _i64, _c_void_p]),
    # §11 v1 compressed adjacency
    "vqgnn_mapper_capacity": (_i64, [_i64, _i64, _i32, _i32, _i32, _i32]),
    "vqgnn_mapper_workspace": (_size, [_i64, _i64, _i32, _i32, _i32]),
    "vqgnn_mapper": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p,
                                    _c_void_p, _c_void_p, _i64, _c_void_p, _i32, _c_void_p, _i64,
                                    _i32, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p,
                                    _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_coo_to_csr_workspace": (_size, [_i64, _i64, _i64]),
    "vqgnn_random_walk": (ctypes.c_int, [_c_void_p, _c_void_p, _i64, _c_void_p, _i64, _i32,
                                         ctypes.c_uint64, _c_void_p, _c_void_p, _c_void_p]),
    "vqgnn_coo_to_csr": (ctypes.c_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _i64, _i64,
                                        _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                        _c_void_p]),
}

_lock = threading.Lock()
_LIB = None


class VQGNNError(RuntimeError):
    """A C-ABI call returned a non-zero vqgnn_status."""


def lib():
    """Load libvqgnn.so once (thread-safe).  Raises if it is absent: the
    product path has no fallback."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _lock:
        if _LIB is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"vqgnn HIP library not found at {LIB_PATH}; run "
                    "`python -c 'import __graft_entry__ as g; g.build()'` "
                    "(hipcc --offload-arch=gfx950)")
            h = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in SIGNATURES.items():
                # a measurement build selected by VQGNN_LIB may predate an
                # entry point (its calls then raise); the product library
                # must export every one
                if os.path.abspath(LIB_PATH) != _DEFAULT_LIB and not hasattr(h, name):
                    continue
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            _LIB = h
    return _LIB


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().vqgnn_last_error()
        raise VQGNNError(f"{what} failed (status {rc}): {msg.decode() if msg else ''}")


def workspace(nbytes: int, device) -> torch.Tensor:
    """Scratch from the PyTorch caching allocator (the library never allocates)."""
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def require_gpu(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(
            f"{what}: tensor on {t.device}; the VQ-GNN hot path runs only on the GPU "
            "(HIP kernels, no CPU fallback)")
