"""ctypes binding of the C ABI in include/ghost_amd.h (libghost_amd.so, built in-tree).

There is no fallback: if the library is missing or the device is not a ROCm GPU,
every product entry point raises.  The CPU restatement under ``oracle/`` is test
infrastructure and is never reached from here.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import threading

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
# GHOST_TUNING=1 selects the A/B tuning build (python -m ghost_amd.build with GHOST_TUNING=1: the
# same sources with -DGHOST_TUNING, whose GHOST_KNOB switches read the environment)
# GHOST_LIB_FILE=<name> loads another in-tree build (same-box A/B against a saved library)
LIB_PATH = os.path.join(HERE, os.environ.get("GHOST_LIB_FILE") or
                        ("libghost_amd_tuning.so" if os.environ.get("GHOST_TUNING") == "1" else "libghost_amd.so"))
HEADER = os.path.join(os.path.dirname(HERE), "include", "ghost_amd.h")

F32, BF16, F16, U8 = 0, 1, 2, 3
_TORCH2G = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16, torch.uint8: U8}
_G2TORCH = {F32: torch.float32, BF16: torch.bfloat16, F16: torch.float16, U8: torch.uint8}

_lib = None
_lock = threading.Lock()

vp, i32, i64, f32 = C.c_void_p, C.c_int, C.c_int64, C.c_float
i64p = C.POINTER(C.c_int64)

_SIGS = {
    "ghost_version": (C.c_char_p, []),
    "ghost_last_error": (C.c_char_p, []),
    "ghost_aei_create": (i32, [C.c_char_p, i32, i32, i32, C.POINTER(vp)]),
    "ghost_aei_destroy": (None, [vp]),
    "ghost_aei_bind": (i32, [vp, C.c_char_p, vp, i64]),
    "ghost_aei_missing": (i32, [vp]),
    "ghost_aei_attr_geometry": (i32, [vp, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
    "ghost_aei_workspace_bytes": (i64, [vp, i32]),
    "ghost_aei_swap_workspace_bytes": (i64, [vp, i32]),
    "ghost_aei_forward": (i32, [vp, vp, i32, i64p, i32, vp, i32, i64, vp, vp, C.POINTER(vp), vp, i64, vp]),
    "ghost_aei_get_attr": (i32, [vp, vp, i32, i64p, i32, C.POINTER(vp), vp, i64, vp]),
    "ghost_aei_swap_u8": (i32, [vp, vp, i64, i32, vp, i32, i64, vp, vp, i64, vp]),
    "ghost_aei_up_stream": (i32, [vp, i32, C.POINTER(vp)]),
    "ghost_aei_identity_table_bytes": (i64, [vp, i32]),
    "ghost_aei_identity_table_workspace_bytes": (i64, [vp, i32]),
    "ghost_aei_identity_table": (i32, [vp, vp, i32, i64, i32, vp, i64, vp, i64, vp]),
    "ghost_aei_swap_u8_indexed": (i32, [vp, vp, i64, i32, vp, i32, i64, vp, vp, vp, i64, vp]),
    "ghost_aei_profile": (i32, [vp, i32]),
    "ghost_aei_profile_read": (i32, [vp, i32, C.POINTER(C.c_double), C.POINTER(i64), C.POINTER(C.c_double),
                                     C.POINTER(C.c_double)]),
    "ghost_aei_profile_clock": (i32, [vp, C.POINTER(C.c_double), C.POINTER(i64), C.POINTER(i32)]),
    "ghost_conv2d_nhwc": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp,
                                f32, vp, i32, i32, vp, i32, vp, i64, vp]),
    "ghost_arc_create": (i32, [C.POINTER(i32), i32, i32, C.POINTER(vp)]),
    "ghost_arc_destroy": (None, [vp]),
    "ghost_arc_bind": (i32, [vp, C.c_char_p, vp, i64]),
    "ghost_arc_missing": (i32, [vp]),
    "ghost_arc_workspace_bytes": (i64, [vp, i32]),
    "ghost_arc_forward": (i32, [vp, vp, i32, i64p, i32, vp, vp, i64, vp]),
    "ghost_arc_embed_u8": (i32, [vp, vp, i64, i32, i32, i32, vp, vp, i64, vp]),
    "ghost_arc_set_taps": (i32, [vp, C.POINTER(vp), i32]),
    "ghost_arc_match": (i32, [vp, i32, vp, i32, i32, f32, vp, vp, vp, vp]),
    "ghost_blend_swaps_u8": (i32, [vp, i64, i32, i32, i32, vp, i64, i32, i32, vp, i64, vp, vp, vp]),
    "ghost_resize_u8_linear": (i32, [vp, i64, i32, i32, i32, vp, i64, i32, i32, vp]),
    "ghost_blend_image_u8": (i32, [vp, i32, i32, vp, i64, i32, i32, vp, i64, vp, vp]),
    "ghost_mask_polygons": (i32, [vp, i32, i32, vp, vp, vp]),
    "ghost_face_masks_workspace_bytes": (i64, [i32, i32, i32]),
    "ghost_face_masks": (i32, [vp, vp, vp, i32, i32, i32, vp, i64, vp, i64, vp]),
    "ghost_conv2d_ex_nhwc": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp,
                                   i32, vp, i64, vp]),
    "ghost_conv_transpose4x4s2_nhwc": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, vp, vp, f32, vp,
                                             i32, vp, i32, vp, i64, vp]),
    "ghost_linear_f32": (i32, [vp, i32, i32, vp, i32, i32, i32, vp, i32, vp, i32, vp, i64, vp]),
    "ghost_instnorm_stats_nhwc": (i32, [i32, vp, i32, i32, i32, i32, vp, vp, i64, vp]),
    "ghost_instnorm_stats_up2x_nhwc": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, vp, i64, vp]),
    "ghost_aad_layer_nhwc": (i32, [i32, vp, i32, vp, i32, i32, i32, i32, i32, i32, vp, i32, i32, vp, vp, vp, vp,
                                   i32, f32, vp, i32, vp, i64, vp]),
    "ghost_upsample2x_nhwc": (i32, [i32, vp, i32, vp, i32, i32, i32, i32, i32, vp]),
    "ghost_nhwc_to_nchw": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, vp]),
    "ghost_crops_to_input_nhwc": (i32, [vp, i64, i32, i32, i32, i32, vp, vp]),
    "ghost_aei_set_option": (i32, [vp, i32, i32]),
    "ghost_aei_get_option": (i32, [vp, i32, C.POINTER(i32)]),
    "ghost_aei_set_taps": (i32, [vp, C.POINTER(vp)]),
    "ghost_aad_layers_v3_nhwc": (i32, [vp, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32, C.POINTER(vp), C.POINTER(vp),
                                       C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), i32, f32, C.POINTER(vp),
                                       C.POINTER(i32), vp, i64, vp]),
    "ghost_conv3x3_narrow_nhwc": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, i32, i32, vp, i32, i32, vp, i32, vp,
                                        vp]),
}


class ConvEpi(C.Structure):
    """struct ghost_conv_epi (include/ghost_amd.h)."""
    _fields_ = [("scale", vp), ("shift", vp), ("slope", f32), ("prelu", vp), ("res", vp), ("ldres", i32),
                ("res_first", i32), ("tanh_out", i32), ("y2", vp), ("ldy2", i32), ("scale2", vp), ("shift2", vp), ("split_k", i32)]


def header_symbols():
    """Function names declared in include/ghost_amd.h."""
    with open(HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ghost_[a-z0-9_]+)\s*\(", text)))


def load(path: str = LIB_PATH):
    """Load libghost_amd.so (raises if absent: there is no fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(f"ghost_amd: native library not built ({path}); run `python -m ghost_amd.build`")
        lib = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().ghost_last_error().decode(errors="replace")
        raise RuntimeError(f"ghost_amd{(' ' + what) if what else ''} failed (rc={rc}): {msg}")


def gdtype(t: torch.dtype) -> int:
    try:
        return _TORCH2G[t]
    except KeyError as e:
        raise TypeError(f"ghost_amd: unsupported dtype {t}") from e


def tdtype(g: int) -> torch.dtype:
    return _G2TORCH[g]


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"ghost_amd: {what} runs only on a ROCm GPU (MI355X); got a {t.device} tensor. "
                           "The CPU path of the reference is not shipped by this package.")


def require_same_device(t: torch.Tensor, dev: torch.device, what: str) -> None:
    """The reference raises torch's device-mismatch error for a host embedding next to device crops;
    the native path would read a host pointer on the GPU, so refuse it here."""
    if t.device != dev:
        raise RuntimeError(f"ghost_amd: {what} must be on {dev}, got a {t.device} tensor")
