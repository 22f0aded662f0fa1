"""Headless orbit viewer: the reference's endless view loop
(src/SfM_CUDA/kernel.cpp:101-107 -> Viewer::show_tsdf, viewer.cu:137-179) without the window.
Every view is the same orbit camera (angle += 0.01 per view around the volume at the mean
depth) raycast on the GPU; instead of cv::imshow (viewer.cu:176) the views are written as PNG
files, or handed to a callback (a display or an encoder).

    python -m semtsdf.orbit CHECKPOINT.npz OUT_DIR [--views 60] [--mode label|color]

writes OUT_DIR/view_00000.png ... from a checkpoint saved by TSDF.save.
"""
from __future__ import annotations

import argparse
import os

import numpy as np

from . import _lib as L
from .tsdf import orbit_angle_sequence
from .volume import DeviceBuffer, orbit_camera


def orbit_views(vol, kinv, dist: float, n: int, mode: str = "label", step: float = 0.01, start: float = 0.0,
                out_dir: str | None = None, callback=None):
    """Render n orbit views of `vol` (a semtsdf.Volume) at angles start + step*(k+1)
    (kernel.cpp:104 increments before the first view).  Each view is a BGR u8 [H, W, 3] image
    (viewer.cu:81-83 writes B, G, R).  The raycast of view k+1 is queued before view k is
    encoded, so the GPU does not wait for the host's PNG encoding.
    Returns the list of written paths (out_dir) or of images (no out_dir, no callback)."""
    m = L.RENDER_LABEL if mode == "label" else L.RENDER_COLOR
    H, W = vol.H, vol.W
    buf = DeviceBuffer(W * H * 3)
    angles = [start + a for a in orbit_angle_sequence(n, step)]
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
    out = []
    try:
        if n:
            vol.raycast_dev(*orbit_camera(kinv, angles[0], dist), m, buf.ptr)
        for k in range(n):
            img = np.empty((H, W, 3), np.uint8)
            buf.download(img, vol.stream)
            vol.sync()
            if k + 1 < n:  # the next view renders while the host encodes this one
                vol.raycast_dev(*orbit_camera(kinv, angles[k + 1], dist), m, buf.ptr)
            if callback is not None:
                callback(k, angles[k], img)
            if out_dir:
                from PIL import Image

                path = os.path.join(out_dir, f"view_{k:05d}.png")
                Image.fromarray(img[:, :, ::-1]).save(path)  # BGR -> RGB file: the colours imshow shows
                out.append(path)
            elif callback is None:
                out.append(img)
    finally:
        vol.sync()
        buf.free()
    return out


def main(argv=None):
    from .tsdf import TSDF

    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("checkpoint")
    ap.add_argument("out_dir")
    ap.add_argument("--views", type=int, default=60)
    ap.add_argument("--mode", choices=["label", "color"], default="label")
    ap.add_argument("--step", type=float, default=0.01)
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    t = TSDF.load(a.checkpoint, device=a.device)
    try:
        paths = orbit_views(t.vol, t.intrinsic_inv, t.mean_depth, a.views, a.mode, a.step, out_dir=a.out_dir)
    finally:
        t.close()
    print(f"wrote {len(paths)} views to {a.out_dir}")


if __name__ == "__main__":
    main()
