"""ctypes binding of libgfd.so (include/gfd.h).  Fails loudly when missing.

There is deliberately no fallback: if the HIP library cannot be loaded, every
``gfd`` op raises ``RuntimeError`` -- the product path never silently runs a
CPU or PyTorch restatement.
"""
from __future__ import annotations

import ctypes as ct
import os
import threading

_LIB = None
_LOCK = threading.Lock()
# GFD_LIB_PATH: an alternative build of the same ABI (e.g. the -DGFD_PROF diagnostic build)
LIB_PATH = os.environ.get("GFD_LIB_PATH") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libgfd.so")

c_i32, c_i64, c_u64, c_f32, c_sz = ct.c_int32, ct.c_int64, ct.c_uint64, ct.c_float, ct.c_size_t
P = ct.c_void_p



class GfdEpilogue(ct.Structure):
    """``gfd_epilogue`` (include/gfd.h)."""
    _fields_ = [("scale_shift", P), ("relu", ct.c_int), ("residual", P),
                ("residual_stride", c_i64), ("head_weight", P), ("head_bias", P),
                ("head_out", P)]


class GfdPlan(ct.Structure):
    """``gfd_plan`` (include/gfd.h)."""
    _fields_ = [("row_order", P), ("slot_desc", P), ("slot_cols", P), ("hub_rank", P),
                ("hub_chunk", P), ("hub_chunk_ptr", P), ("hub_dst", P), ("class_split", P),
                ("num_hubs", c_i64), ("num_chunks", c_i64)]


# element types of x (GFD_DTYPE_*)
DTYPE_F32, DTYPE_BF16 = 0, 1


def x_dtype_code(t) -> int:
    """GFD_DTYPE_* of a feature tensor (fp32 or bf16); raises for anything else."""
    import torch
    if t.dtype == torch.float32:
        return DTYPE_F32
    if t.dtype == torch.bfloat16:
        return DTYPE_BF16
    raise TypeError(f"gfd: node features must be float32 or bfloat16 (got {t.dtype})")


PLAN = ct.POINTER(GfdPlan)

# name -> (restype, argtypes); mirrors include/gfd.h one to one
SIGNATURES = {
    "gfd_status_string": (ct.c_char_p, [c_i32]),
    "gfd_abi_version": (ct.c_int, []),
    "gfd_build_id": (ct.c_char_p, []),
    "gfd_csr_workspace_size": (c_sz, [c_i64, c_i64]),
    "gfd_csr_from_coo": (c_i32, [P, c_i64, c_i64, P, P, P, c_sz, P]),
    "gfd_coo_fingerprint": (c_i32, [P, c_i64, P, P]),
    "gfd_csc_workspace_size": (c_sz, [c_i64, c_i64]),
    "gfd_csc_from_csr": (c_i32, [P, P, c_i64, c_i64, P, P, P, P, c_sz, P]),
    "gfd_plan_workspace_size": (c_sz, [c_i64]),
    "gfd_plan_hubs": (c_i32, [P, c_i64, c_i32, c_i32, P, P, P, P, c_i64, c_i64,
                              ct.POINTER(c_i64), ct.POINTER(c_i64), P, c_sz, P]),
    "gfd_order_workspace_size": (c_sz, [c_i64, c_i32]),
    "gfd_plan_order": (c_i32, [P, c_i64, c_i32, P, P, c_sz, P]),
    "gfd_plan_desc": (c_i32, [P, P, c_i64, P, P, P, P, P, P]),
    "gfd_temporal_workspace_size": (c_sz, [c_i64, c_i64, c_i32]),
    "gfd_temporal_snapshots": (c_i32, [P, c_i64, P, c_i64, c_i64, c_i32, P, P, P, P, P, P, P, c_sz,
                                       P]),
    "gfd_sample_bounds": (c_i32, [c_i64, c_i64, P, c_i32, ct.POINTER(c_i64), ct.POINTER(c_i64)]),
    "gfd_sample_workspace_size": (c_sz, [c_i64, c_i64, P, c_i32]),
    "gfd_sample_neighbors": (c_i32, [P, P, c_i64, P, c_i64, P, c_i32, c_u64, P, P, P, P, P, P, P,
                                     P, c_sz, P]),
    "gfd_id_map_workspace_size": (c_sz, [c_i64]),
    "gfd_id_map_build": (c_i32, [P, c_i64, P, P, P, c_sz, P]),
    "gfd_id_map_lookup": (c_i32, [P, P, c_i64, P, c_i64, P, P]),
    "gfd_edges_from_ids_workspace_size": (c_sz, [c_i64]),
    "gfd_edges_from_ids": (c_i32, [P, P, c_i64, P, P, c_i64, P, P, P, c_sz, P]),
    "gfd_gat_packed_size": (c_sz, [ct.c_int, ct.c_int, ct.c_int]),
    "gfd_gat_pack_weights": (c_i32, [P, P, P, ct.c_int, ct.c_int, ct.c_int, P, P]),
    "gfd_gat_logits": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, ct.c_int, ct.c_int, P, P]),
    "gfd_gat_logits_ex": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, ct.c_int, ct.c_int, P,
                                  P, P]),
    "gfd_gat_logits_lone": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, ct.c_int, ct.c_int,
                                    P, P, c_f32, P, P, P, P, P]),
    "gfd_gat_fwd_workspace_size": (c_sz, [c_i64, c_i64, ct.c_int, ct.c_int, ct.c_int, c_i64,
                                          c_i64]),
    "gfd_gat_aggregate": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, c_i64, c_i64, P, P,
                                  P, ct.c_int, ct.c_int, c_f32, c_f32, c_u64, PLAN, ct.c_int, P,
                                  P, P, c_sz, P]),
    "gfd_gat_aggregate_ex": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, c_i64, c_i64, P,
                                     P, P, P, ct.c_int, ct.c_int, c_f32, c_f32, c_u64, PLAN,
                                     ct.c_int, P, P, P, c_sz, P]),
    "gfd_gat_aggregate_ep": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, c_i64, c_i64, P,
                                     P, P, P, ct.c_int, ct.c_int, c_f32, c_f32, c_u64, PLAN,
                                     ct.c_int, ct.POINTER(GfdEpilogue), P, P, P, c_sz, P]),
    "gfd_gat_aggregate_split": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, c_i64, c_i64,
                                        P, c_i64, P, c_i64, P, P, P, ct.c_int, ct.c_int, c_f32,
                                        c_f32, c_u64, PLAN, ct.c_int, ct.POINTER(GfdEpilogue), P,
                                        c_i64, P, P, c_sz, P]),
    "gfd_gat_logits_lone_split": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, ct.c_int,
                                          ct.c_int, P, P, c_f32, P, c_i64, P, c_i64, P, P, c_i64,
                                          P, P]),
    "gfd_gat_fwd": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, P, P, P, P, ct.c_int,
                            ct.c_int, c_f32, c_f32, c_u64, PLAN, P, P, P, P, c_sz, P]),
    "gfd_gat_fwd_ep": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, P, P, P, P, ct.c_int,
                               ct.c_int, c_f32, c_f32, c_u64, PLAN, ct.POINTER(GfdEpilogue), P, P,
                               P, P, c_sz, P]),
    "gfd_gat_fwd_ep_packed": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, P, P, ct.c_int,
                                      ct.c_int, c_f32, c_f32, c_u64, PLAN,
                                      ct.POINTER(GfdEpilogue), P, P, P, P, c_sz, P]),
    "gfd_gru_head": (c_i32, [P, c_i64, ct.c_int, c_i64, P, P, P, P, P, c_i64, P, P, ct.c_int, P,
                             P, P]),
    "gfd_gru_head_bwd": (c_i32, [P, c_i64, ct.c_int, c_i64, P, P, P, P, P, c_i64, P, ct.c_int, P,
                                 P, P, P, P, P, P]),
    "gfd_atb_workspace_size": (c_sz, [c_i64, ct.c_int]),
    "gfd_atb": (c_i32, [P, c_i64, ct.c_int, P, c_i64, c_i64, P, P, P, c_sz, P]),
    "gfd_rows_copy": (c_i32, [P, c_i64, P, P, c_i64, P, c_i64, ct.c_int, P]),
    "gfd_bn_workspace_size": (c_sz, []),
    "gfd_bn_relu_fwd": (c_i32, [P, P, c_i64, ct.c_int, P, P, c_f32, c_f32, P, P, ct.c_int, c_f32,
                                c_u64, P, P, P, P, c_sz, P]),
    "gfd_bn_relu_bwd": (c_i32, [P, P, c_i64, ct.c_int, P, P, P, P, ct.c_int, c_f32, c_u64, P, P, P,
                                P, c_sz, P]),
    "gfd_gat_bwd_workspace_size": (c_sz, [c_i64, c_i64, ct.c_int, ct.c_int, ct.c_int, c_i64,
                                          c_i64, c_i64]),
    "gfd_gat_bwd": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, PLAN, P, P, P, PLAN, c_i64,
                            P, P, P, ct.c_int, ct.c_int, c_f32, c_f32, c_u64, P, P, P, P, P, P, P,
                            P, P, c_sz, P]),
    "gfd_gat_bwd_ex": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, PLAN, P, P, P, PLAN,
                               c_i64, P, P, P, ct.c_int, ct.c_int, c_f32, c_f32, c_u64, P, P, P,
                               P, P, P, P, P, P, P, c_sz, P]),
    "gfd_gat_bwd_mode": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P, PLAN, P, P, P, PLAN,
                                 c_i64, P, P, P, ct.c_int, ct.c_int, c_f32, c_f32, c_u64, P, P, P,
                                 P, P, P, P, P, P, ct.c_int, P, c_sz, P]),
    "gfd_x_colmax": (c_i32, [P, ct.c_int, c_i64, ct.c_int, c_i64, P, P]),
}

STATUS = {0: "ok", 1: "invalid argument", 2: "edge index out of range", 3: "workspace too small",
          4: "HIP runtime error", 5: "unsupported configuration"}


class GfdError(RuntimeError):
    def __init__(self, fn: str, status: int):
        self.status = status
        super().__init__(f"{fn} failed: {STATUS.get(status, status)} (gfd_status={status})")


def load(path: str = LIB_PATH):
    """Load (once) and return the ctypes library. Raises if it is missing."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            if not os.path.exists(path):
                raise RuntimeError(
                    f"libgfd.so not found at {path}: build it with `python -m gfd.build` "
                    "(gnn-fraud-detection_amd/) or __graft_entry__.build(). gfd has no CPU fallback.")
            lib = ct.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _LIB = lib
    return _LIB


def open_variant(path: str):
    """A separately built library of the same ABI (e.g. the bounds-checked
    diagnostic build ``libgfd_checked.so``), with the signature table applied;
    does not replace the process-wide library of ``load()``."""
    lib = ct.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def call(name: str, *args):
    st = getattr(load(), name)(*args)
    if st != 0:
        raise GfdError(name, st)
    return st


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    return None if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
