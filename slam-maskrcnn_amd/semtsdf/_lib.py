"""ctypes binding of libsemtsdf.so (the C ABI in include/semtsdf.h).

The product path has no fallback: if the HIP library is missing or fails to load, every
entry point raises `SemTSDFError` (the reference's pybind11 module would equally fail at
import, src/TSDF_Python/tsdf.py:7).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsemtsdf.so")

MAX_OBJECTS = 32

OK = 0
ERR_INVALID = -1
ERR_HIP = -2
ERR_OOM = -3
ERR_LABEL = -4
ERR_STATE = -5
ERR_COMM = -6
ERR_UNSUPPORTED = -7

F_SEMANTIC = 0x1
F_GATE_COLOR = 0x2
F_COLOR_I32 = 0x4
F_VOTE = 0x8
F_NO_CULL = 0x10
F_ID_SATURATE = 0x20

PLACE_SFM = 0
PLACE_PYTHON = 1

RENDER_LABEL = 0
RENDER_COLOR = 1
RAY_ASSOC = 2
ASSOC_PARTIAL_LEN = 3168
ASSOC_PIXEL_WORDS = 34
NEED_PIXELS = 1
EXCHANGE_ALLGATHER = 0
EXCHANGE_MIN = 1


class SemTSDFError(RuntimeError):
    """Raised for every non-zero status of the C ABI (reference: RuntimeError from a
    pybind11-translated std::string throw, TSDF_Python/tsdf.cu:119-124)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"semtsdf error {code}: {msg}")
        self.code = code


class Params(C.Structure):
    _fields_ = [
        ("dim", C.c_int32 * 3),
        ("vol_start", C.c_float * 3),
        ("vol_end", C.c_float * 3),
        ("voxel", C.c_float * 3),
        ("mu", C.c_float),
        ("K", C.c_float * 16),
        ("Kinv", C.c_float * 16),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("depth_scale", C.c_float),
        ("gate", C.c_float),
        ("box_thresh", C.c_float),
        ("prior_mrcnn_err_rate", C.c_float),
        ("duplicate_thresh", C.c_float),
        ("flags", C.c_uint32),
        ("z_shard", C.c_int32),
        ("z_nshards", C.c_int32),
        ("z_chunk", C.c_int32),
    ]


class State(C.Structure):
    _fields_ = [
        ("n_obs", C.c_uint32),
        ("num_objs", C.c_int32),
        ("local_dim", C.c_int32 * 3),
        ("local_voxels", C.c_uint64),
        ("device_bytes", C.c_uint64),
        ("label_votes_dropped", C.c_uint64),
    ]


class AssocStats(C.Structure):
    _fields_ = [
        ("max_obj_now", C.c_int32),
        ("num_objs", C.c_int32),
        ("assigned_prev", C.c_int32 * MAX_OBJECTS),
        ("assigned_prob", C.c_float * MAX_OBJECTS),
        ("lut", C.c_uint8 * 256),
        ("exact_rows", C.c_uint32),
        ("reject_rows", C.c_uint32),
    ]


class SurfacePoint(C.Structure):
    _fields_ = [("x", C.c_uint32), ("y", C.c_uint32), ("z", C.c_uint32), ("sdf", C.c_float),
                ("r", C.c_uint8), ("g", C.c_uint8), ("b", C.c_uint8), ("label", C.c_uint8)]


class Timing(C.Structure):
    _fields_ = [
        ("integrate_ms", C.c_double),
        ("assoc_ms", C.c_double),
        ("render_ms", C.c_double),
        ("n_integrate", C.c_uint64),
        ("n_assoc", C.c_uint64),
        ("n_render", C.c_uint64),
        ("touched", C.c_uint64),
        ("gated", C.c_uint64),
        ("bricks", C.c_uint64),
        ("prep_ms", C.c_double),
        ("n_prep", C.c_uint64),
        ("free_units", C.c_uint64),
        ("full_units", C.c_uint64),
        ("lazy_voxels", C.c_uint64),
        ("assoc_exact_frames", C.c_uint64),
        ("assoc_exact_rows", C.c_uint64),
        ("touched_lines", C.c_uint64),
        ("assoc_pos_max", C.c_double),
    ]


_P = C.c_void_p
_I = C.c_int
_F = C.c_float
_D = C.c_double
_PP = C.POINTER(C.c_void_p)

# name -> (restype, argtypes); the complete export list of include/semtsdf.h
SIGNATURES = {
    "semtsdf_last_error": (C.c_char_p, []),
    "semtsdf_abi_version": (_I, []),
    "semtsdf_build_key": (C.c_char_p, []),
    "semtsdf_device_count": (_I, [C.POINTER(C.c_int)]),
    "semtsdf_set_device": (_I, [_I]),
    "semtsdf_stream_create": (_I, [_PP]),
    "semtsdf_stream_destroy": (_I, [_P]),
    "semtsdf_stream_sync": (_I, [_P]),
    "semtsdf_dev_malloc": (_I, [_PP, C.c_size_t]),
    "semtsdf_dev_free": (_I, [_P]),
    "semtsdf_memcpy": (_I, [_P, _P, C.c_size_t, _I, _P]),
    "semtsdf_params_default": (_I, [C.POINTER(Params), _I, _P, _I, _I]),
    "semtsdf_place_from_frame": (_I, [C.POINTER(Params), _P, _D, _I]),
    "semtsdf_create": (_I, [C.POINTER(Params), _I, _PP]),
    "semtsdf_destroy": (_I, [_P]),
    "semtsdf_get_params": (_I, [_P, C.POINTER(Params)]),
    "semtsdf_get_state": (_I, [_P, C.POINTER(State)]),
    "semtsdf_set_state": (_I, [_P, C.c_uint32, C.c_int32]),
    "semtsdf_get_stream": (_P, [_P]),
    "semtsdf_reset": (_I, [_P, _P]),
    "semtsdf_integrate": (_I, [_P, _P, _P, _P, _P, _P]),
    "semtsdf_integrate_dev": (_I, [_P, _P, _P, _P, _P, _P]),
    "semtsdf_integrate_dev_async": (_I, [_P, _P, _P, _P, _P, _P, _P]),
    "semtsdf_integrate_vote_dev": (_I, [_P, _P, _P, _P, _P, _P]),
    "semtsdf_associate": (_I, [_P, _P, _P, C.POINTER(AssocStats), _P]),
    "semtsdf_associate_dev": (_I, [_P, _P, _P, C.POINTER(AssocStats), _P]),
    "semtsdf_assoc_probs": (_I, [_P, _P, _P, _P, _P]),
    "semtsdf_filter_overlaps_dev": (_I, [_P, _P, _P, _P, C.POINTER(AssocStats), _P]),
    "semtsdf_libm_eval": (_I, [_I, _P, _P, C.c_size_t, _P]),
    "semtsdf_parse_frame": (_I, [_P, _P, _P, _P, _P, C.POINTER(AssocStats), _P]),
    "semtsdf_parse_frame_dev": (_I, [_P, _P, _P, _P, _P, _P]),
    "semtsdf_parse_frame_dev_after": (_I, [_P, _P, _P, _P, _P, _P, _P]),
    "semtsdf_parse_frame_view_dev": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P]),
    "semtsdf_orbit_camera": (_I, [_P, _F, _F, _P, _P]),
    "semtsdf_raycast": (_I, [_P, _P, _P, _I, _P, _P, _P]),
    "semtsdf_raycast_dev": (_I, [_P, _P, _P, _I, _P, _P, _P]),
    "semtsdf_shard_ray_begin": (_I, [_P, _I, _P, _P, _I, C.POINTER(C.c_size_t), C.POINTER(C.c_int)]),
    "semtsdf_shard_ray_step": (_I, [_P, _I, _P, _P, _P]),
    "semtsdf_shard_render_finish": (_I, [_P, _P, _P, _P, _P]),
    "semtsdf_shard_assoc_partial": (_I, [_P, _P, _P, _P, _P]),
    "semtsdf_shard_assoc_apply": (_I, [_P, _P, _P, C.POINTER(AssocStats), _P]),
    "semtsdf_shard_assoc_pixels": (_I, [_P, _P, _P, _P]),
    "semtsdf_shard_assoc_apply_exact": (_I, [_P, _P, _P, _P, C.POINTER(AssocStats), _P]),
    "semtsdf_shard_note_integrated": (_I, [_P, _P, _P]),
    "semtsdf_min_i64": (_I, [_P, _P, C.c_size_t, _P]),
    "semtsdf_masks_to_labels": (_I, [_P, _I, _I, _I, _I, _P, C.POINTER(C.c_int), _P]),
    "semtsdf_copy_bandwidth": (_I, [_I, C.c_size_t, _I, C.POINTER(C.c_double)]),
    "semtsdf_download": (_I, [_P, _P, _P, _P, _P, _P, _P]),
    "semtsdf_download_slab": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _P]),
    "semtsdf_upload": (_I, [_P, _P, _P, _P, _P, _P, _P]),
    "semtsdf_export_surface": (_I, [_P, _F, C.c_int32, _P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "semtsdf_map_words": (_I, [_P, _P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "semtsdf_set_instrumentation": (_I, [_P, _I]),
    "semtsdf_get_timing": (_I, [_P, C.POINTER(Timing)]),
    "semtsdf_reset_timing": (_I, [_P]),
    "semtsdf_tsdf_update": (_I, [_P, _P, _P, _P, _P, _I, _P, _F, _F, _P, _P, _P, _P, _P, _I, _I]),
}

_lib = None
_load_error = None


def _bind_torch_runtime():
    """PyTorch-ROCm ships its own copy of the HIP runtime (torch/lib/libamdhip64.so, same
    SONAME as /opt/rocm's) and loads it by path.  Two HIP runtimes in one process do not
    work: the second one to initialise finds no device.  Importing torch (no GPU call)
    before the library makes the library's libamdhip64.so.7 dependency resolve to torch's
    copy, so a process that also uses torch (torch.distributed shard groups, the bench's
    pinned buffers and streams) has a single runtime.  SEMTSDF_NO_TORCH=1 skips it."""
    if os.environ.get("SEMTSDF_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except Exception:  # torch absent: the library uses the system ROCm runtime alone
        pass


def load(path: str | None = None):
    """Load libsemtsdf.so once.  Raises SemTSDFError (loudly) if it is missing."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    _bind_torch_runtime()
    p = path or os.environ.get("SEMTSDF_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise SemTSDFError(ERR_STATE, f"HIP library not built: {p} (run __graft_entry__.build())")
    try:
        lib = C.CDLL(p)
    except OSError as e:  # pragma: no cover - depends on the box
        _load_error = str(e)
        raise SemTSDFError(ERR_HIP, f"cannot load {p}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        if p != LIB_PATH and not hasattr(lib, name):  # an older build under A/B (SEMTSDF_LIB)
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int):
    if rc != OK:
        msg = load().semtsdf_last_error()
        raise SemTSDFError(rc, msg.decode() if msg else "")
    return rc


def ptr(a) -> C.c_void_p | None:
    """Raw pointer of a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, int):
        return C.c_void_p(a)
    if isinstance(a, C.Array):
        return C.cast(a, C.c_void_p)
    assert isinstance(a, np.ndarray), type(a)
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return C.c_void_p(a.ctypes.data)


def f32(a, n=None) -> np.ndarray:
    out = np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1))
    if n is not None and out.size != n:
        raise ValueError(f"expected {n} float32 values, got {out.size}")
    return out
