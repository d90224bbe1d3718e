"""ctypes binding of libtik.so (the C ABI in include/tik.h).

There is no CPU or PyTorch fallback: if the HIP library is missing or no
MI355X is visible, every op raises. torch is imported first so that the HIP
runtime torch ships (soname libamdhip64.so.7) is the one libtik.so binds to,
and device pointers from torch allocations are valid in our kernels.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Iterable, Tuple

import numpy as np
import torch  # noqa: F401  (must precede loading libtik.so)

LIB_PATH = os.environ.get("TIK_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtik.so")

TIK_OK, TIK_E_INVALID, TIK_E_HIP, TIK_E_MISSING, TIK_E_NOMEM = 0, -1, -2, -3, -4


class TikTensor(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.POINTER(ctypes.c_float)),
                ("ndim", ctypes.c_int), ("shape", ctypes.c_int64 * 4)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.POINTER(ctypes.c_float)

# name -> (restype, argtypes); every symbol include/tik.h declares
SIGNATURES: Dict[str, Tuple[object, Tuple]] = {
    "tik_last_error": (ctypes.c_char_p, ()),
    "tik_version": (ctypes.c_char_p, ()),
    "tik_debug_check_guards": (_I, ()),
    "tik_debug_checksums": (_I, (ctypes.c_char_p, _I)),
    "tik_model_create": (_I, (ctypes.POINTER(TikTensor), _I, ctypes.POINTER(_P))),
    "tik_model_destroy": (_I, (_P,)),
    "tik_model_out_frames": (_I, (_P, _I)),
    "tik_model_reserve": (_I, (_P, _I, _I)),
    "tik_ik_forward": (_I, (_P, _P, _I, _I, _P, _P)),
    "tik_backbone_forward": (_I, (_P, _P, _I, _I, _P, _P)),
    "tik_model_set_precision": (_I, (_P, _I)),
    "tik_model_get_precision": (_I, (_P,)),
    "tik_block_set_precision": (_I, (_P, _I)),
    "tik_fk_set_precision": (_I, (_P, _I)),
    "tik_model_profile": (_I, (_P, _I)),
    "tik_model_profile_count": (_I, (_P,)),
    "tik_model_profile_read": (_I, (_P, _I, ctypes.c_char_p, _I, ctypes.POINTER(ctypes.c_float),
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double))),
    "tik_block_create": (_I, (ctypes.POINTER(TikTensor), _I, _I, _I, _I, _I, _F, _I, ctypes.POINTER(_P))),
    "tik_block_destroy": (_I, (_P,)),
    "tik_stgcn_block_fwd": (_I, (_P, _P, _I, _I, _P, _P)),
    "tik_gconv_fwd": (_I, (_P, _I, _I, _I, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P, _P)),
    "tik_aa_to_rotmat": (_I, (_P, _I, _P, _P)),
    "tik_window_gather": (_I, (_P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P)),
    "tik_moveai_to_coco": (_I, (_P, _I, _I, ctypes.POINTER(ctypes.c_int), _P, _P)),
    "tik_stream_create": (_I, (_P, _I, _I, ctypes.POINTER(_P))),
    "tik_stream_destroy": (_I, (_P,)),
    "tik_stream_reset": (_I, (_P,)),
    "tik_stream_push": (_I, (_P, _F, _F)),
    "tik_stream_path": (_I, (_P,)),
    "tik_rotate_root_z": (_I, (_P, _I, _I, ctypes.c_double, _P)),
    "tik_train_windows": (_I, (_P, _I, _P, _I, _P, _P, _P, _P, _I, _I, _P, _P, _I, _I, ctypes.c_ulonglong, _P, _P, _P)),
    "tik_debug_stream_trace": (_I, (_P, ctypes.POINTER(ctypes.c_longlong), _I)),
    "tik_debug_stream_inject_error": (_I, (_P,)),
    "tik_debug_stream_set_count": (_I, (_P, _I)),
    "tik_fk_create": (_I, (ctypes.POINTER(TikTensor), _I, _I, ctypes.POINTER(_P))),
    "tik_fk_destroy": (_I, (_P,)),
    "tik_fk_num_joints": (_I, (_P,)),
    "tik_fk_num_verts": (_I, (_P,)),
    "tik_fk_reserve": (_I, (_P, _I)),
    "tik_fk_forward": (_I, (_P, _P, _P, _P, _P, _I, _P, _P, _P)),
    "tik_fk_profile": (_I, (_P, _I)),
    "tik_fk_profile_count": (_I, (_P,)),
    "tik_fk_profile_read": (_I, (_P, _I, ctypes.c_char_p, _I, ctypes.POINTER(ctypes.c_float),
                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double))),
    "tik_trainer_create": (_I, (ctypes.POINTER(TikTensor), _I, ctypes.c_float, ctypes.POINTER(_P))),
    "tik_trainer_destroy": (_I, (_P,)),
    "tik_trainer_step": (_I, (_P, _P, _I, _I, _P, _P, ctypes.c_ulonglong, _P, _P)),
    "tik_trainer_out_frames": (_I, (_P, _I)),
    "tik_trainer_count": (_I, (_P,)),
    "tik_trainer_tensor": (_I, (_P, _I, ctypes.c_char_p, _I, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(_I),
                                ctypes.POINTER(_I))),
    "tik_trainer_read": (_I, (_P, _I, _I, _P, _P)),
    "tik_trainer_steps": (ctypes.c_longlong, (_P,)),
    "tik_trainer_debug": (_I, (_P, _I, _I, _P, ctypes.c_longlong, _P)),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load libtik.so (raises RuntimeError if it is absent: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libtik.so not found at {path}: build it with "
                           f"`python -m temporal_inverse_kinematics_amd._build` (there is no CPU fallback)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = list(args)
    _lib = lib
    return lib


PRECISIONS = {"fp32": 0, "f32": 0, "bf16x3": 2}


def precision_code(name: str) -> int:
    """'fp32' = exact f32 MFMA; 'bf16x3' = 6-product bf16 split MFMA, fp32 range
    (the default; see include/tik.h)."""
    if name not in PRECISIONS:
        raise ValueError(f"unknown precision {name!r}; expected one of {sorted(PRECISIONS)}")
    return PRECISIONS[name]


def last_error() -> str:
    return load().tik_last_error().decode(errors="replace")


def check(rc: int, what: str = "") -> int:
    if rc >= 0:
        return rc
    msg = f"{what}: {last_error()}" if what else last_error()
    if rc == TIK_E_INVALID:
        raise ValueError(msg)
    if rc == TIK_E_MISSING:
        raise KeyError(msg)
    if rc == TIK_E_NOMEM:
        raise MemoryError(msg)
    raise RuntimeError(msg)


def require_gpu(*tensors: torch.Tensor) -> None:
    """The product path runs only on the MI355X; refuse CPU tensors loudly."""
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("temporal_inverse_kinematics_amd ops run on the GPU only "
                               "(got a CPU tensor; there is no CPU fallback)")
        if t.dtype != torch.float32:
            raise TypeError(f"expected float32 tensor, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError("expected a contiguous tensor")


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def pack_tensors(named: Iterable[Tuple[str, np.ndarray]]):
    """-> (ctypes array of TikTensor, keep-alive list)."""
    items = []
    keep = []
    for name, arr in named:
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32))
        if a.ndim > 4:
            raise ValueError(f"tensor {name} has ndim {a.ndim} > 4")
        bname = name.encode()
        keep += [a, bname]
        shape = (ctypes.c_int64 * 4)(*([int(s) for s in a.shape] + [1] * (4 - a.ndim)))
        items.append(TikTensor(bname, a.ctypes.data_as(_F), a.ndim, shape))
    arr_t = (TikTensor * len(items))(*items)
    return arr_t, keep
