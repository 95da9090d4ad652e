"""ctypes binding of the C ABI in include/picotron_hip.h (libpicotron_hip.so, built in-tree).

There is deliberately no fallback: if the library is missing, or no HIP device is visible,
every op raises.  torch must be imported (and its HIP runtime initialised) before the library is
loaded so that both share one runtime (see build.py).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libpicotron_hip.so")

_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f32 = ctypes.c_float
_vp = ctypes.c_void_p
_i64p = ctypes.POINTER(ctypes.c_int64)
_vpp = ctypes.POINTER(ctypes.c_void_p)

class GemmProblem(ctypes.Structure):
    """pt_gemm_problem (include/picotron_hip.h)."""
    _fields_ = [("A", _vp), ("lda", _i64), ("B", _vp * 4), ("ldb", _i64 * 4), ("b_bounds", _i64 * 5), ("nb", _i32),
                ("b_seg_dim", _i32), ("C", _vp * 4), ("ldc", _i64 * 4), ("c_bounds", _i64 * 5), ("nc", _i32),
                ("M", _i64), ("N", _i64), ("K", _i64), ("residual", _vp), ("ldr", _i64), ("ksplit", _i32),
                ("kpart_stride", _i64), ("A2", _vp), ("a_k2", _i64)]


# name -> (restype, argtypes); mirrors include/picotron_hip.h one to one
SIGNATURES = {
    "pt_rmsnorm_fwd": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _f32, _i32, _vp]),
    "pt_rmsnorm_bwd_partials": (_i32, [_i64, _i32]),
    "pt_gemm_grouped": (_i32, [ctypes.POINTER(GemmProblem), _i32, _i32, _i32, _i32, _i32, _vp]),
    "pt_gemm_splitk_sum": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp]),
    "pt_gemm_splitk_reduce": (_i32, [_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _i32, _i32, _vp, _i64, _vp]),
    "pt_gemm_dual": (_i32, [ctypes.POINTER(GemmProblem), _i32, _i32, _i32, _i32, ctypes.POINTER(GemmProblem), _i32,
                            _i32, _i32, _i32, _i32, _vp]),
    "pt_embedding_fwd": (_i32, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _vp]),
    "pt_embedding_bwd": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i32, _vp]),
    "pt_adamw_step": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _f32, _f32, _f32, _f32, _f32, _f32, _f32, _vp]),
    "pt_adamw_step_multi": (_i32, [_vp, _vp, _i32, _i64, _f32, _f32, _f32, _f32, _f32, _f32, _f32, _vp]),
    "pt_rmsnorm_bwd": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp]),
    "pt_rmsnorm_colsum_batch": (_i32, [_vp, _vp, _vp, _vp, _i32, _i64, _vp]),
    "pt_rmsnorm_bwd_splitk": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp]),
    "pt_rope": (_i32, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _i64, _i64, _i32, _vp]),
    "pt_swiglu_fwd": (_i32, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _vp]),
    "pt_swiglu_bwd": (_i32, [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _vp]),
    "pt_residual_add": (_i32, [_vp, _vp, _vp, _i64, _vp]),
    "pt_cross_entropy_fwd_bwd": (_i32, [_vp, _i64, _vp, _vp, _i64, _vp, _i64, _i64, _f32, _vp, _i64, _vp, _vp]),
    "pt_cross_entropy_fwd_lse": (_i32, [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp]),
    "pt_cross_entropy_bwd_lse": (_i32, [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _vp]),
    "pt_gemm": (_i32, [_vp, _i64, _i32, _vpp, _i64p, _i64p, _i32, _i32, _i32, _vpp, _i64p, _i64p, _i32,
                       _i64, _i64, _i64, _i32, _vp, _i64, _i32, _vp]),
    "pt_gemm_pick_tile": (_i32, [_i64, _i64, _i64p, _i32, _i64p, _i32]),
    "pt_attn_fwd": (_i32, [_vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64, _i64, _i64, _i64, _i64,
                           _i64, _f32, _i32, _i32, _i64, _vp]),
    "pt_attn_bwd_delta": (_i32, [_vp, _i64p, _vp, _i64p, _vp, _i64, _i64, _i64, _i64, _i64, _vp]),
    "pt_attn_bwd": (_i32, [_vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _vp, _vp, _i64p, _vp, _i64p,
                           _vp, _i64p, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _i32, _i32, _vp, _vp, _i64, _i64,
                           _vp]),
    "pt_attn_bwd_part": (_i32, [_vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _vp, _vp, _i64p, _vp, _i64p,
                                _vp, _i64p, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _i32, _i32, _i64, _i32, _vp]),
    "pt_attn_bwd_fused_delta": (_i32, [_vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _vp, _vp,
                                       _i64p, _vp, _i64p, _vp, _i64p, _i64, _i64, _i64, _i64, _i64, _i64, _f32,
                                       _i32, _vp, _vp, _i64, _i64, _vp]),
    "pt_attn_split_plan": (_i32, [_i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _vp]),
    "pt_attn_fwd_split": (_i32, [_vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64, _i64, _i64, _i64, _i64,
                                 _i64, _f32, _i32, _vp, _i64, _vp]),
    "pt_attn_bwd_split": (_i32, [_vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _i64p, _vp, _vp, _vp, _i64p,
                                 _vp, _i64p, _vp, _i64p, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _i32, _vp, _vp,
                                 _i64, _vp, _i64, _vp]),
    "pt_lse_merge": (_i32, [_vp, _vp, _i32, _vp, _vp, _i32, _vp, _vp, _i64, _i64, _vp]),
    "pt_gemm_ce_stats": (_i32, [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _vp]),
    "pt_cross_entropy_fwd_stats": (_i32, [_vp, _i64, _vp, _vp, _i64, _vp, _vp, _i64, _i64, _i64, _vp, _vp]),
    "pt_cross_entropy_mean": (_i32, [_vp, _vp, _i64, _i64, _vp, _vp, _vp, _i32, _i32, _vp]),
    "pt_cross_entropy_vp_partial": (_i32, [_vp, _i64, _vp, _vp, _i64, _vp, _i64, _i64, _i64, _vp]),
    "pt_cross_entropy_vp_combine": (_i32, [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp]),
    "pt_cross_entropy_bwd_lse_shard": (_i32, [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _i64, _i64,
                                              _vp]),
    "pt_embedding_sort": (_i32, [_vp, _i64, _i64, _i64, _i32, _i64, _vp, _vp, _vp]),
    "pt_set_variant": (_i32, [ctypes.c_char_p, _i32]),
    "pt_get_variant": (_i32, [ctypes.c_char_p]),
    "pt_gemm_rope": (_i32, [_vp, _i64, _vpp, _i64p, _i64p, _i32, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _i64, _i64,
                            _i64, _i64, _i32, _vp]),
}

ERRORS = {-1: "PT_EINVAL (bad size or null pointer)", -2: "PT_EALIGN (misaligned pointer/stride)",
          -3: "PT_EUNSUPPORTED (shape outside the kernel's tiling)"}

_lib = None          # the product library (LIB_PATH), used by every op
_alt_libs = {}       # other builds loaded for A/B tools, one entry per path; never become _lib


class HipKernelError(RuntimeError):
    pass


def load_library(path=LIB_PATH, strict=True):
    """dlopen the kernel library and bind every symbol; does not touch the GPU.  strict=False (A/B
    runs against another build) skips symbols that build does not export.  Only LIB_PATH becomes
    the library the ops call; another path is cached under its own name and returned."""
    global _lib
    path = os.path.abspath(path)
    is_main = path == os.path.abspath(LIB_PATH)
    if is_main and _lib is not None:
        return _lib
    if not is_main and path in _alt_libs:
        return _alt_libs[path]
    if not os.path.exists(path):
        raise HipKernelError(f"picotron_amd HIP library not built: {path} (run python -m picotron_amd.build)")
    import torch  # noqa: F401  -- its HIP runtime must be the one our SONAME binds to
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if not strict and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if is_main:
        from .switches import apply_native
        apply_native(lib)
        _lib = lib
    else:
        _alt_libs[path] = lib
    return lib


def use_library(path):
    """A/B tools only: make another build the library every op calls, explicitly (and say so)."""
    global _lib
    _lib = load_library(path, strict=False)
    print(f"[picotron_amd] ops now call {os.path.abspath(path)}", flush=True)
    return _lib


def lib():
    """The bound library, for compute calls: requires a visible HIP device."""
    if _lib is None:
        load_library()
    if not torch.cuda.is_available():
        raise HipKernelError("picotron_amd kernels need a HIP device (MI355X / gfx950); none is visible")
    return _lib


def check(rc, name):
    if rc != 0:
        msg = ERRORS.get(rc, f"hipError {rc}")
        raise HipKernelError(f"{name} failed: {msg}")


def stream_ptr(device=None):
    """torch's current stream on `device` (a tensor's device).  Kernels launch on the calling
    thread's current HIP device, so a tensor on another device is refused rather than handed to a
    kernel on the wrong GPU with foreign pointers."""
    if device is not None and getattr(device, "index", None) is not None and device.index != torch.cuda.current_device():
        raise HipKernelError(f"tensor on {device} but the current HIP device is cuda:{torch.cuda.current_device()}: "
                             f"call torch.cuda.set_device({device.index}) (train.py does) or use torch.cuda.device()")
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def i64arr(vals):
    return (ctypes.c_int64 * len(vals))(*[int(v) for v in vals])


def i32arr(vals):
    return (ctypes.c_int32 * len(vals))(*[int(v) for v in vals])


def ptrarr(vals):
    return (ctypes.c_void_p * len(vals))(*[int(v) for v in vals])
