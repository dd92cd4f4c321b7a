"""ctypes binding of ``lib/libhgnn.so`` (the C ABI declared in ``include/hgnn.h``).

Only plain pointers, sizes and a ``hipStream_t`` (as ``void*``) cross this boundary.  There is no
CPU fallback anywhere in the package: if the library is missing, or a tensor is not on a ROCm
device, the call raises.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
from typing import Optional, Sequence

import torch

LIB_PATH = pathlib.Path(__file__).resolve().parent / "lib" / "libhgnn.so"
# A/B measurement of two builds of the same sources (scripts/build_variant.py): HGNN_LIB names
# another in-tree build under lib/ (libhgnn_<name>.so); never a path outside the package, and
# never a library whose build stamp does not match this tree's sources (build.check_library).
if os.environ.get("HGNN_LIB"):
    LIB_PATH = LIB_PATH.parent / pathlib.Path(os.environ["HGNN_LIB"]).name

HGNN_MEAN = 1
HGNN_ACCUMULATE = 2
MAX_SEG = 6

_c_i32, _c_i64, _c_sz, _p = ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/hgnn.h
_SIGS = {
    "hgnn_version": (_c_i32, []),
    "hgnn_last_error_string": (ctypes.c_char_p, []),
    "hgnn_coo_to_csr_ws_bytes": (_c_sz, [_c_i64, _c_i64]),
    "hgnn_coo_to_csr": (_c_i32, [_p, _p, _c_i64, _c_i64, _c_i64, _p, _p, _p, _p, _p, _c_sz, _p]),
    "hgnn_plan_ws_bytes": (_c_sz, [_c_i64]),
    "hgnn_plan_count": (_c_i32, [_p, _c_i64, _c_i32, _p, _p, _c_sz, _p]),
    "hgnn_plan_fill": (_c_i32, [_p, _c_i64, _c_i32, _p, _p, _p, _c_sz, _p]),
    "hgnn_inv_degree": (_c_i32, [_p, _c_i64, _p, _p]),
    "hgnn_gather_reduce": (_c_i32, [_p, _c_i64, _c_i32, _p, _p, _c_i64, _p, _p, _c_i32, _p, _p,
                                    _c_i64, _c_i64, _c_i32, _p, _p, _p]),
    "hgnn_gather_reduce_multi": (_c_i32, [_c_i32, _p, _p, _c_i32, _p, _p, _p, _p, _c_i32, _p,
                                          _p, _p]),
    "hgnn_gather_reduce_scaled": (_c_i32, [_p, _c_i64, _c_i32, _p, _p, _c_i64, _p, _p, _p,
                                           _c_i32, _p, _p, _c_i64, _c_i64, _c_i32, _p, _p, _p]),
    "hgnn_gather_mean_fwd": (_c_i32, [_p, _c_i64, _c_i32, _p, _p, _c_i64, _p, _p, _c_i64,
                                      _c_i64, _c_i32, _p, _p, _p]),
    "hgnn_scatter_mean_bwd": (_c_i32, [_p, _c_i64, _p, _p, _p, _c_i64, _c_i32, _p, _p, _c_i64,
                                       _c_i64, _c_i32, _p, _p, _c_i32, _p]),
    "hgnn_linear_fwd": (_c_i32, [_c_i32, _p, _p, _c_i64, _p, _c_i32, _p, _c_i32, _p, _p]),
    "hgnn_linear_fwd_add": (_c_i32, [_c_i32, _p, _p, _c_i64, _p, _c_i32, _p, _p, _c_i32, _p,
                                     _p]),
    "hgnn_linear_fwd_mask": (_c_i32, [_c_i32, _p, _p, _c_i64, _p, _c_i32, _p, _p, _c_i32, _p,
                                      _p, _p]),
    "hgnn_linear_bwd_mask": (_c_i32, [_c_i32, _p, _p, _c_i64, _p, _c_i32, _p, _p, _p, _p, _p,
                                      _p, _p, _p, _c_sz, _p]),
    "hgnn_linear_bwd_ex": (_c_i32, [_c_i32, _p, _p, _c_i64, _p, _c_i32, _p, _p, _p, _p,
                                    ctypes.c_uint32, _p, _p, _p, _p, _c_sz, _p]),
    "hgnn_adam_multi": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _p, _p, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, _p]),
    "hgnn_linear_fwd_multi": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _c_i32, _p, _p, _p, _p, _p]),
    "hgnn_linear_bwd_multi_ws_bytes": (_c_sz, [_c_i32, _p, _p, _c_i32]),
    "hgnn_linear_bwd_multi": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _c_i32, _p, _p, _p, _p, _p,
                                       _p, _p, _p, _c_sz, _p]),
    "hgnn_fuse_weights": (_c_i32, [_c_i32, _p, _p, _p, _c_i32, _p, _p, _c_i32, _p, _p, _p]),
    "hgnn_split_weight_grads": (_c_i32, [_c_i32, _p, _p, _p, _c_i32, _p, _c_i32, _p, _p, _p,
                                         _p]),
    "hgnn_fuse_weights_multi": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _p, _p, _c_i32, _p, _p,
                                         _p]),
    "hgnn_split_weight_grads_multi": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _p, _c_i32, _p, _p,
                                               _p, _p]),
    "hgnn_linear_bwd_ws_bytes": (_c_sz, [_c_i64, _c_i32, _c_i32]),
    "hgnn_linear_bwd": (_c_i32, [_c_i32, _p, _p, _c_i64, _p, _c_i32, _p, _p, _p, _p, _p, _p,
                                 _c_sz, _p]),
    "hgnn_linear_bwd_dz": (_c_i32, [_c_i32, _p, _p, _c_i64, _p, _c_i32, _p, _p, _p, _p, _p, _p,
                                    _p, _c_sz, _p]),
    "hgnn_sort_pairs_ws_bytes": (_c_sz, [_c_i64, _c_i64]),
    "hgnn_sort_pairs_i32": (_c_i32, [_p, _p, _p, _c_i64, _c_i64, _p, _p, _p, _p, _p, _c_sz, _p]),
    "hgnn_draw_sort_negatives": (_c_i32, [_p, _p, _c_i64, _c_i64, _p, _p, _p, _p, _c_sz, _p]),
    "hgnn_sort_pairs_i64": (_c_i32, [_p, _p, _p, _c_i64, _c_i64, _p, _p, _p, _p, _p, _c_sz, _p]),
    "hgnn_score_gather": (_c_i32, [_p, _c_i64, _p, _c_i32, _p, _p, _c_i64, _c_i32, _p,
                                   ctypes.c_float, _p, _p, _c_i64, _c_i64, _c_i32, _p, _p,
                                   _c_i32, _p]),
    "hgnn_score_gather2": (_c_i32, [_p, _c_i64, _p, _c_i32, _p, _p, _p, _p, _c_i64, _p,
                                    ctypes.c_float, _p, _p, _c_i64, _c_i64, _c_i32, _p, _p, _p]),
    "hgnn_sample_ws_bytes": (_c_sz, [_c_i64]),
    "hgnn_sample_hop_ws_bytes": (_c_sz, [_c_i64]),
    "hgnn_sample_hop_count": (_c_i32, [_c_i32, _p, _p, _p, _p, _c_i32, _p, _p, _p, _c_sz, _p]),
    "hgnn_sample_hop_fill": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _c_i32, ctypes.c_uint64, _p,
                                      _p, _p]),
    "hgnn_sample_fill": (_c_i32, [_p, _p, _c_i64, _p, _c_i64, _c_i32, ctypes.c_uint64, _p, _p,
                                  _p]),
    "hgnn_csr_transpose": (_c_i32, [_p, _p, _c_i64, _c_i64, _c_i64, _p, _p, _p, _p, _p, _c_sz,
                                    _p]),
    "hgnn_csr_transpose_multi_ws_bytes": (_c_sz, [_c_i64, _c_i64]),
    "hgnn_csr_transpose_multi": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_sz,
                                          _p]),
    "hgnn_sample_neighbors": (_c_i32, [_p, _p, _c_i64, _p, _c_i64, _c_i32, ctypes.c_uint64, _p,
                                       _p, _p, _c_sz, _p]),
    "hgnn_relabel_ws_bytes": (_c_sz, [_c_i64, _c_i64]),
    "hgnn_relabel": (_c_i32, [_p, _c_i64, _p, _c_i64, _p, _p, _p, _p, _c_sz, _p]),
    "hgnn_relabel_checked": (_c_i32, [_p, _c_i64, _c_i64, _p, _c_i64, _p, _p, _p, _p, _c_sz,
                                      _p]),
    "hgnn_relabel_multi_ws_bytes": (_c_sz, [_c_i64, _c_i64]),
    "hgnn_set_k3_split": (_c_i32, [_c_i32]),
    "hgnn_pad_csr_multi": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "hgnn_gather_rows_multi": (_c_i32, [_c_i32, _p, _p, _p, _c_i64, _p, _p]),
    "hgnn_link_seeds": (_c_i32, [_p, _p, _p, _p, _c_i64, _p, _p, _p, _p, _p, _p, _p]),
    "hgnn_sample_hop_static": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _p, _p, _c_i32,
                                        ctypes.c_uint64, _p, _p, _p, _p, _p, _p, _p, _c_sz, _p]),
    "hgnn_relabel_static_ws_bytes": (_c_sz, [_c_i64, _c_i64]),
    "hgnn_relabel_static": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _c_i32, _p, _p, _p, _p, _p, _p,
                                     _p, _c_sz, _p]),
    "hgnn_link_group_ws_bytes": (_c_sz, [_c_i64]),
    "hgnn_link_group": (_c_i32, [_p, _p, _p, _c_i64, _c_i64, _c_i64, _p, _p, _p, _p, _p, _p, _p,
                                 _p, _p, _p, _c_sz, _p]),
    "hgnn_relabel_multi": (_c_i32, [_c_i32, _p, _p, _p, _p, _p, _p, _p, _p, _c_i32, _p, _c_sz,
                                    _p]),
    "hgnn_topk_metrics": (_c_i32, [_p, _c_i64, _c_i64, _c_i64, _p, _p, _p, _c_i32, _p, _p, _p,
                                   _p]),
    "hgnn_topk_metrics_rows": (_c_i32, [_p, _c_i64, _c_i64, _c_i64, _p, _p, _p, _p, _c_i32, _p,
                                        _p, _p, _p]),
    "hgnn_score_topk_lds_bytes": (_c_sz, [_c_i32, _c_i32]),
    "hgnn_score_topk": (_c_i32, [_p, _p, _c_i64, _p, _c_i64, _c_i32, _c_i32, _p, _p, _p]),
    "hgnn_topk_finish": (_c_i32, [_p, _p, _c_i64, _c_i32, _c_i64, _c_i32, _p, _p, _p, _p, _p, _p,
                                  _p]),
    "hgnn_edge_score_parts": (_c_i64, [_c_i64]),
    "hgnn_edge_score_fwd": (_c_i32, [_p, _p, _c_i32, _c_i64, _c_i64, _p, _p, _p, _p, _c_i64, _p,
                                     _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "hgnn_edge_score_fwd_i32": (_c_i32, [_p, _p, _c_i32, _c_i64, _c_i64, _p, _p, _p, _c_i64, _p,
                                         _p, _p, _p, _p, _p]),
    "hgnn_edge_score_fwd_draw": (_c_i32, [_p, _p, _c_i32, _c_i64, _c_i64, _p, _p, _p, _c_i64,
                                          _p, _p, _p, _p, _p, _p]),
    "hgnn_uniform_i32": (_c_i32, [_p, _c_i64, _c_i32, _p, _p]),
    "hgnn_scale_unless_one": (_c_i32, [_p, _c_i64, _p, _p]),
    "hgnn_linear_fwd_f32": (_c_i32, [_p, _c_i64, _c_i32, _p, _c_i32, _p, _p, _p]),
    "hgnn_linear_dgrad_f32": (_c_i32, [_p, _c_i64, _c_i32, _p, _c_i32, _p, _p]),
    "hgnn_linear_wgrad_f32": (_c_i32, [_p, _p, _c_i64, _c_i32, _c_i32, _p, _p, _p, _c_sz, _p]),
    "hgnn_hetero_epilogue": (_c_i32, [_c_i32, _p, _p, _c_i64, _c_i32, _p, _p]),
    "hgnn_hetero_epilogue_bwd": (_c_i32, [_c_i32, _p, _c_i64, _c_i32, _p, _p, _p, _p]),
    "hgnn_idmap_capacity": (_c_i64, [_c_i64]),
    "hgnn_idmap_build": (_c_i32, [_p, _p, _p, _c_i64, _p, _c_i64, _p]),
    "hgnn_idmap_lookup": (_c_i32, [_p, _c_i64, _p, _p, _p, _p, _p, _p, _p, _p, _c_i64, _p, _p]),
    "hgnn_compact_rows_ws_bytes": (_c_sz, [_c_i64]),
    "hgnn_compact_rows": (_c_i32, [_p, _c_i32, _c_i64, _p, _p, _c_i32, _p, _p, _c_sz, _p]),
}

_lib: Optional[ctypes.CDLL] = None


class NativeError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load the library once.  torch is imported first so its HIP runtime (same SONAME
    libamdhip64.so.7) is the one the library binds to — one runtime, one set of streams."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise NativeError(f"hgnn native library not found at {LIB_PATH}; build it with "
                              "`python -m truth_recommendation_gnn_amd.build` (no CPU fallback)")
        from . import build as _build
        try:
            _build.check_library(LIB_PATH)
        except RuntimeError as e:
            raise NativeError(str(e)) from None
        l = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in _SIGS.items():
            fn = getattr(l, name, None)
            if fn is None:
                continue
            fn.restype, fn.argtypes = res, args
        _lib = l
    return _lib


def exported_symbols() -> Sequence[str]:
    l = lib()
    return [n for n in _SIGS if hasattr(l, n)]


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().hgnn_last_error_string().decode(errors="replace")
        raise NativeError(f"{what} failed (code {rc}): {msg}")


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else _p(t.data_ptr())


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device: torch.device):
    """The device's current HIP stream as a raw pointer.  torch's own raw accessor (the one its
    generated code uses) costs well under a microsecond; ``torch.cuda.current_stream`` builds a
    Stream object per call (~5 us), which at a few hundred calls per sampled mini-batch step was
    a visible share of the host time."""
    if _raw_stream is not None:
        i = device.index
        return _p(_raw_stream(torch.cuda.current_device() if i is None else i))
    return _p(torch.cuda.current_stream(device).cuda_stream)


def require_device(*tensors: Optional[torch.Tensor]) -> torch.device:
    dev = None
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise ValueError("hgnn runs only on a ROCm GPU (MI355X / gfx950); got a tensor on "
                             f"{t.device} — move the graph and model with .to('cuda')")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"tensors on different devices: {dev} vs {t.device}")
    if dev is None:
        raise ValueError("no tensor to infer the device from")
    return dev


def workspace(nbytes: int, device: torch.device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def ptr_array(ts: Sequence[Optional[torch.Tensor]]):
    arr = (_p * max(MAX_SEG, len(ts)))()
    for i, t in enumerate(ts):
        arr[i] = None if t is None else t.data_ptr()
    return arr


def int_array(vals: Sequence[int]):
    arr = (_c_i32 * max(MAX_SEG, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr


def i64_array(vals: Sequence[int]):
    arr = (_c_i64 * max(MAX_SEG, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr


def float_array(vals: Sequence[float]):
    arr = (ctypes.c_float * max(MAX_SEG, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = float(v)
    return arr
