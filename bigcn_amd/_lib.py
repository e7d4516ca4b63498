"""ctypes binding of ``libbgcn.so`` (the C ABI declared in ``include/bgcn.h``).

The library is built in-tree (``make -C bigcn_amd/csrc`` or ``__graft_entry__.build()``)
and linked against ``libamdhip64.so.7`` by SONAME, so inside a PyTorch process it
shares the HIP runtime torch already loaded (same streams, same device memory).

There is deliberately no fallback: if the library is missing or no ROCm device is
present, every op raises.  The oracle under ``oracle/`` is test infrastructure and
is never imported from here.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import (POINTER, Structure, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_size_t,
                    c_uint64, c_void_p)

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BGCN_LIB", os.path.join(_HERE, "libbgcn.so"))

BGCN_DEGREE_ON_COL = 0
BGCN_DEGREE_ON_ROW = 1
BGCN_EPI_NONE = 0
BGCN_EPI_RELU = 1
BGCN_FEAT_AUTO = 0
BGCN_FEAT_DENSE = 1
BGCN_FEAT_SPARSE = 2
BGCN_SPARSE_CAP = 32
BGCN_SPARSE_SPILL_PER_ROW = 32   # spill pool capacity per row (rows over the ELL cap)
BGCN_DTYPE_F32 = 0
BGCN_DTYPE_BF16 = 1
ABI_VERSION = 12   # BGCN_ABI_VERSION of include/bgcn.h
BGCN_STATUS_CROSS_TREE = 16

# every symbol include/bgcn.h declares (checked by tests/test_capi.py)
EXPORTED_SYMBOLS = (
    "bgcn_abi_version", "bgcn_last_error",
    "bgcn_graph_workspace_size", "bgcn_build_graph", "bgcn_graph_dinv",
    "bgcn_edge_weight_grad_workspace_size", "bgcn_edge_weight_grad",
    "bgcn_graph_pair_workspace_size", "bgcn_build_graph_pair", "bgcn_graph_pair_plans",
    "bgcn_spmm_workspace_size", "bgcn_spmm",
    "bgcn_gemm_xwt", "bgcn_gemm_xw", "bgcn_gemm_tn_workspace_size", "bgcn_gemm_tn",
    "bgcn_colsum_workspace_size", "bgcn_colsum",
    "bgcn_scatter_mean_workspace_size", "bgcn_scatter_mean_fwd", "bgcn_scatter_mean_bwd",
    "bgcn_head_forward", "bgcn_head_backward",
    "bgcn_drop_edges_workspace_size", "bgcn_drop_edges",
    "bgcn_bigcn_workspace_size", "bgcn_bigcn_forward", "bgcn_bigcn_backward",
    "bgcn_keep_words", "bgcn_set_kernel_timing", "bgcn_kernel_timing", "bgcn_kernel_span", "bgcn_adam_step",
    "bgcn_prepare_workspace_size", "bgcn_prepare_batch", "bgcn_csr_to_dense",
    "bgcn_train_step_workspace_size", "bgcn_train_step", "bgcn_train_step_dw1", "bgcn_join_side",
    "bgcn_weight_images_size", "bgcn_train_step_saved", "bgcn_eval_step",
    "bgcn_loader_create", "bgcn_loader_slot_bytes", "bgcn_loader_len", "bgcn_loader_next", "bgcn_loader_destroy",
    "bgcn_loader_wait", "bgcn_loader_get_stats",
)


class SpmmPlan(Structure):
    """bgcn_spmm_plan (include/bgcn.h)."""
    _fields_ = [("bnd", c_void_p), ("longs", c_void_p), ("nlong", c_void_p)]


class GraphView(Structure):
    _fields_ = [
        ("t_ptr", c_void_p), ("t_row", c_void_p), ("t_col", c_void_p), ("t_w", c_void_p),
        ("s_ptr", c_void_p), ("s_row", c_void_p), ("s_col", c_void_p), ("s_w", c_void_p),
        ("capacity", c_int64), ("plan", SpmmPlan * 2), ("tree_status", c_void_p),
    ]


class CsrOut(Structure):
    _fields_ = [
        ("t_ptr", c_void_p), ("t_row", c_void_p), ("t_col", c_void_p), ("t_w", c_void_p),
        ("s_ptr", c_void_p), ("s_row", c_void_p), ("s_col", c_void_p), ("s_w", c_void_p),
    ]


class BiGCNArgs(Structure):
    _fields_ = [
        ("x", c_void_p), ("ldx", c_int64), ("num_nodes", c_int64), ("num_graphs", c_int64),
        ("in_feats", c_int64), ("hid", c_int64), ("batch", c_void_p), ("rootindex", c_void_p),
        ("td", GraphView), ("bu", GraphView),
        ("td_w1", c_void_p), ("td_b1", c_void_p), ("td_w2", c_void_p), ("td_b2", c_void_p),
        ("bu_w1", c_void_p), ("bu_b1", c_void_p), ("bu_w2", c_void_p), ("bu_b2", c_void_p),
        ("training", c_int), ("seed", c_uint64), ("keep_words", c_void_p),
        ("feat_mode", c_int), ("x_flags", c_void_p), ("x_nnz", c_void_p), ("x_cols", c_void_p),
        ("x_vals", c_void_p),
        ("tree_ptr", c_void_p), ("h1", c_void_p), ("h2", c_void_p), ("head_in", c_void_p),
        ("dhead_in", c_void_p),
        ("td_dw1", c_void_p), ("td_db1", c_void_p), ("td_dw2", c_void_p), ("td_db2", c_void_p),
        ("bu_dw1", c_void_p), ("bu_db1", c_void_p), ("bu_dw2", c_void_p), ("bu_db2", c_void_p),
        ("save_for_backward", c_int32), ("x_dtype", c_int32),
        ("prepared", c_void_p), ("prepared_bytes", c_size_t),
        ("td_num_edges", c_int64), ("bu_num_edges", c_int64),
    ]


BGCN_STEP_PARAMS = 10


class BatchDesc(Structure):
    """bgcn_batch (include/bgcn.h)."""
    _fields_ = [
        ("x", c_void_p), ("ldx", c_int64), ("num_nodes", c_int64), ("num_graphs", c_int64),
        ("batch", c_void_p), ("rootindex", c_void_p),
        ("td_edge_index", c_void_p), ("td_num_edges", c_int64),
        ("bu_edge_index", c_void_p), ("bu_num_edges", c_int64),
        ("td_droprate", c_double), ("bu_droprate", c_double), ("drop_seed", c_uint64),
        ("x_dtype", c_int32),
        ("x_row_ptr", c_void_p), ("x_col", c_void_p), ("x_val", c_void_p),
    ]


class StepArgs(Structure):
    """bgcn_step_args (include/bgcn.h)."""
    _fields_ = [
        ("cur", BatchDesc), ("in_feats", c_int64), ("num_classes", c_int64), ("y", c_void_p),
        ("degree_on", c_int32), ("training", c_int32), ("seed", c_uint64), ("feat_mode", c_int32),
        ("params", c_void_p * BGCN_STEP_PARAMS), ("grads", c_void_p * BGCN_STEP_PARAMS),
        ("loss", c_void_p), ("logp", c_void_p), ("status", c_void_p),
        ("prepared", c_void_p), ("prepared_bytes", c_size_t), ("prepared_ready", c_int32),
        ("next", POINTER(BatchDesc)), ("next_prepared", c_void_p), ("next_prepared_bytes", c_size_t),
        ("status_flag", c_void_p),
        ("images", c_void_p), ("images_current", c_int32),
        ("status_seen", c_void_p),
        ("defer_dw1", c_int32),
        ("adam", c_void_p),
    ]


_SIGS = {
    "bgcn_abi_version": (c_int, []),
    "bgcn_last_error": (c_char_p, []),
    "bgcn_graph_workspace_size": (c_size_t, [c_int64, c_int64]),
    "bgcn_build_graph": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int,
                                 c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_size_t, c_void_p]),
    "bgcn_graph_pair_workspace_size": (c_size_t, [c_int64, c_int64, c_int64]),
    "bgcn_graph_dinv": (c_int, [c_void_p, c_size_t, c_int64, c_int64, POINTER(c_void_p)]),
    "bgcn_edge_weight_grad_workspace_size": (c_size_t, [c_int64]),
    "bgcn_edge_weight_grad": (c_int, [c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_size_t, c_void_p]),
    "bgcn_build_graph_pair": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int,
                                      POINTER(CsrOut), POINTER(CsrOut), c_void_p, c_void_p, c_void_p,
                                      c_size_t, c_void_p]),
    "bgcn_spmm_workspace_size": (c_size_t, [c_int64, c_int32]),
    "bgcn_spmm": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                          c_int64, c_void_p, c_int64, c_int32, c_void_p, c_int, c_void_p,
                          c_size_t, c_void_p]),
    "bgcn_gemm_xwt": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                              c_int64, c_int64, c_int64, c_int64, c_void_p]),
    "bgcn_gemm_xw": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int64,
                             c_int64, c_int64, c_void_p]),
    "bgcn_gemm_tn_workspace_size": (c_size_t, [c_int64, c_int64, c_int64]),
    "bgcn_gemm_tn": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64,
                             c_int64, c_int64, c_int64, c_int64, c_void_p, c_size_t, c_void_p]),
    "bgcn_colsum_workspace_size": (c_size_t, [c_int64, c_int32]),
    "bgcn_colsum": (c_int, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p, c_size_t,
                            c_void_p]),
    "bgcn_scatter_mean_workspace_size": (c_size_t, [c_int64]),
    "bgcn_scatter_mean_fwd": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int32, c_int64,
                                      c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_size_t,
                                      c_void_p]),
    "bgcn_scatter_mean_bwd": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int32,
                                      c_int64, c_void_p, c_int64, c_void_p]),
    "bgcn_graph_pair_plans": (c_int, [c_void_p, c_size_t, c_int64, c_int64, c_int64, c_void_p, c_void_p]),
    "bgcn_head_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    "bgcn_head_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_void_p,
                                   c_void_p, c_void_p, c_void_p]),
    "bgcn_bigcn_workspace_size": (c_size_t, [c_int64, c_int64, c_int64, c_int64]),
    "bgcn_bigcn_forward": (c_int, [POINTER(BiGCNArgs), c_void_p, c_size_t, c_void_p]),
    "bgcn_bigcn_backward": (c_int, [POINTER(BiGCNArgs), c_void_p, c_size_t, c_void_p]),
    "bgcn_keep_words": (c_int, [c_uint64, c_int64, c_int32, c_void_p, c_void_p]),
    "bgcn_adam_step": (c_int, [c_void_p, c_void_p]),
    "bgcn_weight_images_size": (c_size_t, [c_int64]),
    "bgcn_drop_edges_workspace_size": (c_size_t, [c_int64]),
    "bgcn_drop_edges": (c_int, [c_void_p, c_int64, c_double, c_void_p, c_int64, c_void_p, c_int64, c_double,
                                c_void_p, c_int64, c_void_p, c_int64, c_int64, c_uint64, c_int32, c_void_p,
                                c_void_p, c_void_p, c_size_t, c_void_p]),
    "bgcn_prepare_workspace_size": (c_size_t, [c_int64, c_int64, c_int64, c_int64, c_int64]),
    "bgcn_prepare_batch": (c_int, [POINTER(BatchDesc), c_int64, c_int32, c_int32, c_void_p, c_size_t,
                                   c_void_p]),
    "bgcn_csr_to_dense": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32,
                                  c_void_p, c_void_p]),
    "bgcn_train_step_workspace_size": (c_size_t, [c_int64, c_int64, c_int64, c_int64, c_int64, c_int64]),
    "bgcn_train_step": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "bgcn_train_step_dw1": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "bgcn_eval_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "bgcn_join_side": (c_int, [c_void_p]),
    "bgcn_train_step_saved": (c_int, [c_void_p, c_size_t, c_int64, c_int64, c_int64, c_int64,
                                      POINTER(c_void_p), POINTER(c_void_p)]),
    "bgcn_loader_create": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int, c_int, c_uint64, c_int64,
                                   c_int, c_int, c_int, c_int, POINTER(c_void_p)]),
    "bgcn_loader_slot_bytes": (c_int64, [c_void_p]),
    "bgcn_loader_len": (c_int64, [c_void_p]),
    "bgcn_loader_next": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_int64,
                                 POINTER(c_void_p)]),
    "bgcn_loader_destroy": (None, [c_void_p]),
    "bgcn_loader_wait": (c_int, [c_void_p]),
    "bgcn_loader_get_stats": (c_int, [c_void_p, c_void_p, c_int]),
    "bgcn_set_kernel_timing": (c_int, [c_int]),
    "bgcn_kernel_timing": (c_int, [c_int, POINTER(c_float), POINTER(c_int64)]),
    "bgcn_kernel_span": (c_int, [c_int, POINTER(c_float), POINTER(c_int64)]),
}

_lock = threading.Lock()
_lib = None


class BGCNError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """Load and type the library (no GPU needed: used by the CPU symbol tests)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise ImportError(
                f"libbgcn.so not found at {path}: build it with `make -C bigcn_amd/csrc` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
        lib = ctypes.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.bgcn_abi_version() != ABI_VERSION:
            raise ImportError("libbgcn.so ABI version mismatch")
        _lib = lib
        return lib


_gpu_seen = False


def lib():
    """The library, for device work: requires a ROCm device (checked until one is seen)."""
    global _gpu_seen
    if not _gpu_seen:
        if not torch.cuda.is_available():
            raise BGCNError("the bigcn_amd HIP path needs a ROCm GPU (no CPU fallback exists)")
        _gpu_seen = True
    return _lib if _lib is not None else load_library()


def check(rc: int) -> None:
    if rc != 0:
        msg = load_library().bgcn_last_error().decode(errors="replace")
        raise BGCNError(f"libbgcn error {rc}: {msg}")


def stream_handle(device=None) -> int:
    """hipStream_t of the current torch stream (of `device`, default the current device).
    The per-call form reads torch's raw current stream (~0.1 us; the Stream object path
    costs ~3 us and runs several times per drop-in training step)."""
    if device is None and _raw_stream is not None:
        return _raw_stream(_cur_device())
    return torch.cuda.current_stream(device).cuda_stream


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)
if _cur_device is None:
    _raw_stream = None


def ptr(t) -> int:
    """Device pointer of a tensor (or 0 for None)."""
    if t is None:
        return 0
    return t.data_ptr()


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)
