"""Surface export of a fused volume (the reference keeps no export of its
own -- its volume layout is src/TSDF_Python/tsdf.py:48-52 and the voxel position rule
src/SfM_CUDA/tsdf.cu:30): the labelled surface voxels as a point cloud, written as PLY."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

# the palette of the label render (viewer.cu:93-126), RGB
PALETTE = np.array([
    230, 25, 75, 60, 180, 75, 255, 225, 25, 0, 130, 200, 245, 130, 48, 145, 30, 180, 70, 240, 240, 240, 50, 230,
    210, 245, 60, 250, 190, 190, 0, 128, 128, 230, 190, 255, 170, 110, 40, 255, 250, 200, 128, 0, 0, 170, 255, 195,
    230, 25, 75, 60, 180, 75, 255, 225, 25, 0, 130, 200, 245, 130, 48, 145, 30, 180, 70, 240, 240, 240, 50, 230,
    210, 245, 60, 250, 190, 190, 0, 128, 128, 230, 190, 255, 170, 110, 40, 255, 250, 200, 128, 0, 0, 170, 255, 195,
], np.uint8).reshape(32, 3)


def export_surface(vol, sdf_max: float = 0.2, min_weight: int = 1) -> dict:
    """Surface voxels of `vol` (a Volume; a shard exports its owned planes): weight >= min_weight
    and |sdf| < sdf_max.  Returns index [n, 3] u32 (global voxel index, the reference's flat
    order), xyz [n, 3] f32 world position vol_start + index * voxel rounded once (tsdf.cu:30's
    fmaf), sdf [n] f32, rgb [n, 3] u8, label [n] u8."""
    lib = L.load()
    n = C.c_uint64()
    L.check(lib.semtsdf_export_surface(vol.handle, float(sdf_max), int(min_weight), None, 0, C.byref(n)))
    pts = (L.SurfacePoint * max(int(n.value), 1))()
    if n.value:
        L.check(lib.semtsdf_export_surface(vol.handle, float(sdf_max), int(min_weight), C.cast(pts, C.c_void_p),
                                           int(n.value), C.byref(n)))
    a = np.frombuffer(pts, dtype=np.dtype([("x", "<u4"), ("y", "<u4"), ("z", "<u4"), ("sdf", "<f4"),
                                           ("r", "u1"), ("g", "u1"), ("b", "u1"), ("label", "u1")]))[:int(n.value)]
    idx = np.stack([a["x"], a["y"], a["z"]], axis=1).astype(np.uint32)
    p = vol.params
    start = np.array(list(p.vol_start), np.float32).astype(np.float64)
    voxel = np.array(list(p.voxel), np.float32).astype(np.float64)
    # idx * voxel + start is exact in double (a 16-bit index times a 24-bit float, plus a float):
    # rounding it once to f32 is the fused multiply-add of tsdf.cu:30
    xyz = (idx.astype(np.float64) * voxel + start).astype(np.float32)
    return {"index": idx, "xyz": xyz, "sdf": a["sdf"].copy(), "rgb": np.stack([a["r"], a["g"], a["b"]], axis=1),
            "label": a["label"].copy()}


def write_ply(path: str, xyz: np.ndarray, rgb: np.ndarray, label: np.ndarray | None = None,
              color_by_label: bool = False) -> None:
    """Binary little-endian PLY: float x, y, z; uchar red, green, blue; uchar label.  With
    color_by_label the colours are the label render's palette (label 0 keeps its colour)."""
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    n = xyz.shape[0]
    rgb = np.ascontiguousarray(rgb, np.uint8).reshape(n, 3)
    lab = np.zeros(n, np.uint8) if label is None else np.ascontiguousarray(label, np.uint8).reshape(n)
    if color_by_label:
        rgb = np.where((lab > 0)[:, None], PALETTE[lab % 32], rgb).astype(np.uint8)
    rec = np.zeros(n, dtype=np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("red", "u1"), ("green", "u1"),
                                      ("blue", "u1"), ("label", "u1")]))
    rec["x"], rec["y"], rec["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    rec["red"], rec["green"], rec["blue"] = rgb[:, 0], rgb[:, 1], rgb[:, 2]
    rec["label"] = lab
    header = ("ply\nformat binary_little_endian 1.0\ncomment semtsdf surface export\n"
              f"element vertex {n}\nproperty float x\nproperty float y\nproperty float z\n"
              "property uchar red\nproperty uchar green\nproperty uchar blue\nproperty uchar label\nend_header\n")
    with open(path, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(rec.tobytes())


def read_ply(path: str) -> dict:
    """Reads back what write_ply writes (tests, tools)."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    head = data[:end].decode("ascii").splitlines()
    n = int(next(ln for ln in head if ln.startswith("element vertex")).split()[-1])
    rec = np.frombuffer(data[end:], dtype=np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("red", "u1"),
                                                    ("green", "u1"), ("blue", "u1"), ("label", "u1")]), count=n)
    return {"xyz": np.stack([rec["x"], rec["y"], rec["z"]], axis=1), "rgb": np.stack([rec["red"], rec["green"],
                                                                                        rec["blue"]], axis=1),
            "label": rec["label"].copy()}
