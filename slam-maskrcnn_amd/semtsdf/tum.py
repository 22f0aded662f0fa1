"""TUM RGB-D ingest: trajectory reading, frame association and
pose lookup, replacing the reference's host drivers.

Two selectable behaviours:
  * mode="sfm"    — src/SfM_CUDA/kernel.cpp:44-99 + utils.cu:62-91: timestamps parsed from
                    `name[5:]` and returned as *float32* by the lambda (kernel.cpp:52,56: ~4 ms
                    rounding), depth i paired with the first mask j whose time >= depth time,
                    rgb indexed by the mask index, pose = first trajectory key >= ts
                    (std::map::lower_bound on fmod(ts, 1e5)), mean depth in metres.
  * mode="python" — src/TSDF_Python/main.py:59-140 + tsdf_utils.py:23-29: float64
                    timestamps, depth paired with rgb, pose lerp/slerp interpolated,
                    mean depth in raw units.
"""
from __future__ import annotations

import glob
import os
from dataclasses import dataclass

import numpy as np

from . import pose as P


def read_traj(filename: str) -> np.ndarray:
    """tsdf_utils.py:23-29: rows [t, tx, ty, tz, qx, qy, qz, qw]; t = float(stamp[5:])."""
    rows = []
    with open(filename) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            parts = line.strip("\n").split(" ")
            parts[0] = parts[0][5:]
            rows.append([float(x) for x in parts[:8]])
    return np.array(rows, dtype=np.float64)


def read_trajactory(filename: str) -> dict:
    """utils.cu:62-75 (name kept): {fmod(ts, 1e5): [tx ty tz qx qy qz qw]}; lines that do
    not parse as 8 numbers are skipped."""
    out = {}
    with open(filename) as f:
        for line in f:
            parts = line.split()
            try:
                vals = [float(x) for x in parts[:8]]
            except ValueError:
                continue
            if len(vals) < 8:
                continue
            out.setdefault(float(np.fmod(vals[0], 1e5)), vals[1:8])
    return dict(sorted(out.items()))


def lower_bound_pose(traj_map: dict, ts: float):
    """std::map::lower_bound (kernel.cpp:97): first key >= ts."""
    for k, v in traj_map.items():
        if k >= ts:
            return v
    raise KeyError(f"no trajectory entry at or after {ts}")


def stamp_of(fn: str, as_float32: bool) -> float:
    base = os.path.basename(fn)
    stem = base[: base.rfind(".")] if "." in base else base
    v = float(stem[5:])
    return float(np.float32(v)) if as_float32 else v


def mean_depth_m(depth: np.ndarray, depth_scale: float = 5000.0) -> float:
    """utils.cu:77-91: mean of d/5000 over d > 0, accumulated in float64, returned float32."""
    d = depth[depth > 0].astype(np.float64)
    return float(np.float32((d / depth_scale).sum() / d.size))


def mean_depth_raw(depth: np.ndarray) -> float:
    """main.py:124: np.mean(depth[depth > 0]) in raw units."""
    return float(np.mean(depth[depth > 0]))


@dataclass
class FrameRef:
    depth_fn: str
    rgb_fn: str
    mask_fn: str | None
    ts: float
    pose: np.ndarray  # [tx ty tz qx qy qz qw]


def associate(root: str, mode: str = "sfm", begin: float = 68164.0, end: float = 68170.0,
              max_frames: int = 100) -> list[FrameRef]:
    """Frame list of a TUM directory `root` with rgb/, depth/, mask/ and groundtruth.txt."""
    rgb_fn = sorted(glob.glob(os.path.join(root, "rgb", "*.png")))
    depth_fn = sorted(glob.glob(os.path.join(root, "depth", "*.png")))
    mask_fn = sorted(glob.glob(os.path.join(root, "mask", "*.png")))
    gt = os.path.join(root, "groundtruth.txt")
    f32 = mode == "sfm"
    dts = [stamp_of(f, f32) for f in depth_fn]
    pair_fn = mask_fn if mode == "sfm" else rgb_fn
    pts = [stamp_of(f, f32) for f in pair_fn]
    out: list[FrameRef] = []
    if mode == "sfm":
        traj_map = read_trajactory(gt)
    else:
        traj = read_traj(gt)
    i, j = 0, 0
    while i < len(dts):
        if dts[i] < begin or dts[i] > end:
            i += 1
            continue
        while i < len(dts) and j < len(pts) and dts[i] < pts[j]:
            i += 1
        while i < len(dts) and j < len(pts) and pts[j] < dts[i]:
            j += 1
        if i >= len(dts) or j >= len(pts):
            break
        ts = dts[i]
        if mode == "sfm":
            pose = np.array(lower_bound_pose(traj_map, ts), dtype=np.float64)
            out.append(FrameRef(depth_fn[i], rgb_fn[j] if j < len(rgb_fn) else "", mask_fn[j], ts, pose))
        else:
            pose = P.interpolate_pose(traj, ts)
            out.append(FrameRef(depth_fn[i], rgb_fn[j], mask_fn[j] if j < len(mask_fn) else None, ts, pose))
        if len(out) >= max_frames:
            break
        i += 1
    return out


def load_png(fn: str) -> np.ndarray:
    """PNG reader (16-bit depth, 8-bit mask, RGB).  PIL stands in for cv2.imread."""
    from PIL import Image

    im = Image.open(fn)
    a = np.array(im)
    if a.ndim == 3 and a.shape[2] == 4:
        a = a[:, :, :3]
    return np.ascontiguousarray(a)
