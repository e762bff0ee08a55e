"""Bindings of the native libraries.

  * ``ops()`` -- the PyTorch-ROCm custom operators ``torch.ops.mlgate.*``
    (libmlgate_torch.so, csrc/torch_ops.cpp: TORCH_LIBRARY(mlgate) over the C ABI).
    Every compute call of the mlgate package goes through them.
  * ``lib()`` -- ctypes view of libmlgate.so, the C ABI declared in include/mlgate.h,
    kept for the op-level kernel tests and the ABI export checks.

The libraries are the only compute path of this package: there is no CPU or eager
PyTorch fallback.  ``ops()`` / ``lib()`` raise if a shared object is missing, and
``require_device()`` raises if no HIP device is visible.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmlgate.so")
TORCH_LIB_PATH = os.path.join(_HERE, "libmlgate_torch.so")
OPS = ("vit_forward_into", "salad_forward", "knn_gate", "knn_query", "row_normalize", "similarity", "xcorr_score", "xcorr_batch",
       "superpoint",
       "lightglue", "ransac_epipolar", "recover_pose", "resnet50", "loftr_features", "loftr_pack_tails", "loftr_coarse_layer", "loftr_match", "superglue", "pillow_resize_224", "plane_ransac", "proximity",
       "prof_enable", "prof_reset", "prof_read")


c_int, c_long, c_size_t, c_float, c_double, c_void_p = (
    ctypes.c_int, ctypes.c_long, ctypes.c_size_t, ctypes.c_float, ctypes.c_double, ctypes.c_void_p)

EXPORTS = {
    "mlg_abi_version": (c_int, []),
    "mlg_strerror": (ctypes.c_char_p, [c_int]),
    "mlg_vit_workspace_bytes": (c_size_t, [c_int, c_int]),
    "mlg_vit_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_long, c_int, c_int, c_void_p,
                                c_size_t, c_void_p, c_void_p, c_void_p]),
    "mlg_salad_workspace_bytes": (c_size_t, [c_int, c_int]),
    "mlg_salad_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_long, c_int,
                                  c_void_p, c_size_t, c_void_p, c_void_p]),
    "mlg_knn_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mlg_knn_workspace_bytes_k": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "mlg_knn_gate": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_double, c_float, c_int,
                             c_int, c_int, c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p]),
    "mlg_knn_query": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_double, c_int,
                              c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mlg_row_normalize_f32": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "mlg_similarity": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "mlg_xcorr_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mlg_xcorr_score": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p,
                                c_void_p]),
    "mlg_plane_ransac_workspace_bytes": (c_size_t, [c_int, c_int]),
    "mlg_plane_ransac": (c_int, [c_void_p, c_void_p, c_int, c_int, ctypes.c_uint64, c_double, c_void_p, c_size_t,
                                 c_void_p, c_void_p, c_void_p, c_void_p]),
    "mlg_proximity_workspace_bytes": (c_size_t, [c_int, c_int]),
    "mlg_proximity_count": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_double, c_int, c_int, c_void_p,
                                    c_size_t, c_void_p, c_void_p]),
    "mlg_proximity_emit": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_double, c_int, c_int, c_void_p,
                                   c_size_t, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mlg_ransac_workspace_bytes": (c_size_t, [c_int, c_long, c_int]),
    "mlg_ransac_epipolar": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_long, c_void_p, c_int, c_double, c_int,
                                    ctypes.c_uint64, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p]),
    "mlg_recover_pose": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                 c_void_p]),
    "mlg_resnet50_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mlg_resnet50_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_long, c_int, c_void_p,
                                     c_size_t, c_void_p, c_void_p]),
    "mlg_op_pillow_resize_224": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_long, c_void_p, c_size_t,
                                         c_void_p, c_void_p]),
    "mlg_superpoint_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mlg_superpoint": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_long, c_float, c_int, c_int, c_int,
                               c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mlg_lightglue_workspace_bytes": (c_size_t, [c_int, c_int]),
    "mlg_lightglue": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int,
                              c_float, c_float, c_float, c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p]),
    "mlg_op_gemm_f32out": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mlg_op_gemm_f32out_variant": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mlg_set_gemm_variant": (c_int, [c_int]),
    "mlg_set_loftr_similarity": (c_int, [c_int]),
    "mlg_op_gemm_bias_gelu": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mlg_op_gemm_residual": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                     c_void_p]),
    "mlg_op_layernorm_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "mlg_op_attention": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "mlg_op_attention_varlen": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                        c_void_p, c_int, c_int, c_void_p]),
    "mlg_op_lg_ffn": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int] + [c_void_p] * 8 + [c_void_p]),
    "mlg_op_lg_proj": (c_int, [c_int, c_void_p, c_int] + [c_void_p] * 8 + [c_int, c_void_p]),
    "mlg_op_conv2d_nhwc": (c_int, [c_void_p, c_void_p] + [c_int] * 6 + [c_void_p] * 3 + [c_int, c_void_p]),
    "mlg_op_preprocess_patches": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_long, c_int, c_void_p,
                                          c_void_p]),
    "mlg_prof_enable": (c_int, [c_int]),
    "mlg_prof_reset": (c_int, []),
    "mlg_prof_read": (c_int, [c_int, ctypes.POINTER(c_double), ctypes.POINTER(c_long)]),
    "mlg_prof_read_work": (c_int, [c_int, ctypes.POINTER(c_double)]),
    "mlg_lg_orient_matches": (c_int, [c_void_p] * 5 + [c_int, c_int] + [c_void_p] * 4),
    "mlg_xcorr_batch_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "mlg_xcorr_batch": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_size_t,
                                c_void_p, c_void_p]),
    "mlg_dbg_lg_trace_begin": (c_int, [c_void_p, c_size_t]),
    "mlg_dbg_lg_trace_end": (c_int, [c_void_p, c_void_p, c_int]),
    "mlg_dbg_fill_lds": (c_int, [ctypes.c_uint32, c_void_p, c_void_p]),
    "mlg_dbg_fill_regs": (c_int, [ctypes.c_uint32, c_void_p]),
    "mlg_dbg_ransac_poison_nsol": (c_int, [c_int, c_int]),
    "mlg_loftr_tails_bytes": (c_size_t, []),
    "mlg_loftr_pack_tails": (c_int, [c_void_p, c_void_p, c_void_p]),
    "mlg_op_loftr_coarse_layer_ws_bytes": (c_size_t, [c_int, c_int]),
    "mlg_op_loftr_coarse_layer": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_size_t,
                                          c_void_p]),
    "mlg_png_info": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mlg_png_decode_bgr": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mlg_png_load_bgr": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p]),
}

_lib = None
_ops = None


class MlgateError(RuntimeError):
    pass


def lib():
    """Load libmlgate.so (built by __graft_entry__.build / `make -C csrc`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MlgateError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                              "g.build()'` (hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def ops():
    """torch.ops.mlgate, after loading libmlgate_torch.so (built by __graft_entry__.build)."""
    global _ops
    if _ops is None:
        import torch
        if not os.path.exists(TORCH_LIB_PATH):
            raise MlgateError(f"{TORCH_LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                              "g.build()'`")
        lib()  # the C ABI library the operators link against
        torch.ops.load_library(TORCH_LIB_PATH)
        _ops = torch.ops.mlgate
    return _ops


def lightglue_workspace_bytes(pairs, kmax):
    """mlg_lightglue_workspace_bytes: HBM one LightGlue call of `pairs` pairs needs (a size
    query: DeviceGate sizes its pair chunks from it)."""
    return int(lib().mlg_lightglue_workspace_bytes(int(pairs), int(kmax)))


def check(rc, what=""):
    if rc != 0:
        msg = lib().mlg_strerror(rc).decode()
        raise MlgateError(f"{what} failed: {msg} (status {rc})")


def require_device(device="cuda"):
    """Raise unless a HIP device is usable for `device` (mlgate has no CPU path)."""
    import torch
    dev = torch.device(device)
    if dev.type != "cuda":
        raise MlgateError(f"mlgate runs its hot path on MI355X HIP kernels only; got device={device!r}. "
                          "Use device='cuda' (PyTorch-ROCm's name for the HIP device).")
    if not torch.cuda.is_available():
        raise MlgateError("no HIP device visible: mlgate's kernels need an MI355X (gfx950)")
    ops()
    return dev


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def stream_of(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
