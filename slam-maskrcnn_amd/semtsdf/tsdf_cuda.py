"""Drop-in replacement for the pybind11 module `tsdf_cuda` of src/TSDF_Python
(tsdf.cpp:11-37).  `import semtsdf.tsdf_cuda as tsdf_cuda` makes the reference's
`tsdf_cuda.tsdf_update(...)` call in tsdf.py:63-64 run on the gfx950 kernels.

Argument order, meaning and in-place semantics are the reference's: the five volume arrays
are updated in place.  pybind11's `array_t<T>` force-casts a wrongly typed or
non-contiguous argument into a temporary, so the reference silently loses the update of
such an in/out array; that behaviour is kept here (with a RuntimeWarning so the loss is at
least visible).  Input arrays are cast the same way (e.g. the u8 HxWx3 masks of
main.py:101 become an int32 array whose first H*W elements are read as `cls`).
"""
from __future__ import annotations

import warnings

import numpy as np

from . import _lib as L


def _inout(a, dt, name):
    if isinstance(a, np.ndarray) and a.dtype == dt and a.flags["C_CONTIGUOUS"] and a.flags["WRITEABLE"]:
        return a
    warnings.warn(f"tsdf_update: '{name}' is not a contiguous {np.dtype(dt).name} array; like pybind11's "
                  f"force-cast the update goes to a temporary copy and is lost", RuntimeWarning, stacklevel=3)
    return np.ascontiguousarray(np.array(a, dtype=dt))


def _in(a, dt):
    return np.ascontiguousarray(np.asarray(a, dtype=dt))


def tsdf_update(tsdf_diff, tsdf_color, tsdf_wt, tsdf_cls, tsdf_cls_cnt, vol_dim, vol_start, voxel, miu, intrinsic,
                depth, color, cls, extrinsic2init, width, height):
    d = _inout(tsdf_diff, np.float32, "tsdf_diff")
    c = _inout(tsdf_color, np.int32, "tsdf_color")
    w = _inout(tsdf_wt, np.int32, "tsdf_wt")
    k = _inout(tsdf_cls, np.int32, "tsdf_cls")
    kc = _inout(tsdf_cls_cnt, np.int32, "tsdf_cls_cnt")
    n = int(vol_dim) ** 3
    for a, m, name in ((d, 1, "tsdf_diff"), (c, 3, "tsdf_color"), (w, 1, "tsdf_wt"), (k, 1, "tsdf_cls"),
                       (kc, 1, "tsdf_cls_cnt")):
        if a.size < n * m:
            # the reference would read/write past the end of the buffer
            raise ValueError(f"{name} has {a.size} elements, needs {n * m} for vol_dim={vol_dim}")
    vs = _in(vol_start, np.float32)
    K = _in(intrinsic, np.float32)
    dep = _in(depth, np.uint16)
    col = _in(color, np.uint8)
    cl = _in(cls, np.int32)
    E = _in(extrinsic2init, np.float32)
    npx = int(width) * int(height)
    if dep.size < npx or col.size < 3 * npx or cl.size < npx or K.size < 16 or E.size < 16 or vs.size < 3:
        raise ValueError("frame or matrix arguments are too small")
    L.check(L.load().semtsdf_tsdf_update(L.ptr(d), L.ptr(c), L.ptr(w), L.ptr(k), L.ptr(kc), int(vol_dim), L.ptr(vs),
                                         float(voxel), float(miu), L.ptr(K), L.ptr(dep), L.ptr(col), L.ptr(cl),
                                         L.ptr(E), int(width), int(height)))
