"""Mask producer contract: Mask R-CNN detection masks -> the u8
instance-label mask the fusion consumes, on the GPU (semtsdf_masks_to_labels, restating
Mask_RCNN/dmask.py:21-59 mask_detect: filter_tiny_objects, preserve_small_objs, label
i + 1).  The detector itself (COCO-weight Mask R-CNN) is not part of this package: its
weights are not available offline; any producer that yields masks[H, W, N] can feed it.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .volume import DeviceBuffer

MIN_AREA = 2000  # dmask.py:42 (area > 2000)


def masks_to_labels_dev(masks_ptr: int, width: int, height: int, n: int, labels_ptr: int, min_area: int = MIN_AREA,
                        stream=None, want_count: bool = False):
    """Device masks [H][W][n] bytes -> device labels [H][W] u8 (async unless want_count)."""
    k = C.c_int()
    L.check(L.load().semtsdf_masks_to_labels(C.c_void_p(masks_ptr) if n else None, int(width), int(height), int(n),
                                             int(min_area), C.c_void_p(labels_ptr),
                                             C.byref(k) if want_count else None, stream))
    return k.value if want_count else None


def masks_to_labels(masks: np.ndarray, min_area: int = MIN_AREA):
    """Host convenience: masks bool/u8 [H, W, N] -> (labels u8 [H, W], kept detections)."""
    m = np.ascontiguousarray(masks)
    if m.ndim != 3:
        raise ValueError("masks must be [H, W, N]")
    m = m.view(np.uint8) if m.dtype == np.bool_ else np.ascontiguousarray(m, dtype=np.uint8)
    H, W, n = m.shape
    out = np.zeros((H, W), np.uint8)
    mb = DeviceBuffer(max(m.nbytes, 1))
    ob = DeviceBuffer(H * W)
    try:
        if n:
            mb.upload(m)
        kept = masks_to_labels_dev(mb.ptr, W, H, n, ob.ptr, min_area, want_count=True)
        ob.download(out)
        L.check(L.load().semtsdf_stream_sync(None))
    finally:
        mb.free()
        ob.free()
    return out, kept
