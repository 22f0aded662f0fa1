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
    """utils.cu:77-91: `sum += ptr[i] / 5000.` over the nonzero pixels in pixel order (double,
    left to right), divided by their count, returned as float32 (NaN for an all-zero frame,
    the reference's 0/0)."""
    d = np.asarray(depth).reshape(-1)
    d = d[d > 0].astype(np.float64) / depth_scale
    if d.size == 0:
        return float("nan")
    s = float(np.cumsum(d)[-1])  # sequential accumulation, as the C loop (not pairwise)
    return float(np.float32(s / d.size))


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
    i: int = -1       # depth index
    j: int = -1       # mask (sfm) / rgb (python) index


def _pairs_sfm(dts, pts, begin, end, max_frames):
    """kernel.cpp:64-74: one index i that the inner loops advance (the for-loop's i++ keeps
    them), frames counted before the cap `cnt > 100`."""
    out = []
    j = 0
    i = 0
    cnt = 0
    while i < 10000:
        if i >= len(dts):
            break
        if dts[i] < begin or dts[i] > end:
            i += 1
            continue
        while i < len(dts) and j < len(pts) and dts[i] < pts[j]:
            i += 1
        while i < len(dts) and j < len(pts) and pts[j] < dts[i]:
            j += 1
        if i >= len(dts) or j >= len(pts):
            break  # the reference reads past the end here
        cnt += 1
        if cnt > max_frames:
            break
        out.append((i, j))
        i += 1
    return out


def _pairs_python(dts, pts, begin, end, max_frames):
    """main.py:83-91: `for i in range(3000)` rebinds i every iteration, so the inner loops'
    advances do not carry over and a depth frame can be processed more than once."""
    out = []
    j = 0
    for i0 in range(3000):
        i = i0
        if i >= len(dts):
            break
        if dts[i] < begin or dts[i] > end:
            continue
        while i < len(dts) and j < len(pts) and dts[i] < pts[j]:
            i += 1
        while i < len(dts) and j < len(pts) and pts[j] < dts[i]:
            j += 1
        if i >= len(dts) or j >= len(pts):
            break  # the reference raises IndexError here
        out.append((i, j))
        if max_frames is not None and len(out) >= max_frames:
            break
    return out


def associate(root: str, mode: str = "sfm", begin: float | None = None, end: float | None = None,
              max_frames: int | None = None) -> list[FrameRef]:
    """Frame list of a TUM directory `root` with rgb/, depth/, mask/ and groundtruth.txt.

    mode "sfm"    (kernel.cpp:44-99): float32 time stamps, depth i paired with the first
                  mask j whose stamp is >= the depth stamp, rgb by the mask index, pose =
                  lower_bound of fmod(ts, 1e5) (no interpolation); window [68164, 68170],
                  at most 100 frames.
    mode "python" (main.py:59-142): float64 stamps, depth paired with rgb, mask by the rgb
                  index, pose lerp/slerp-interpolated; window [68164, 68164.37], no cap."""
    if mode not in ("sfm", "python"):
        raise ValueError(f"mode must be 'sfm' or 'python', got {mode!r}")
    sfm = mode == "sfm"
    begin = (68164.0 if begin is None else begin)
    end = (68170.0 if sfm else 68164.37) if end is None else end
    rgb_fn = sorted(glob.glob(os.path.join(root, "rgb", "*.png")))
    depth_fn = sorted(glob.glob(os.path.join(root, "depth", "*.png")))
    mask_fn = sorted(glob.glob(os.path.join(root, "mask", "*.png")))
    gt = os.path.join(root, "groundtruth.txt")
    dts = [stamp_of(f, sfm) for f in depth_fn]
    pair_fn = mask_fn if sfm else rgb_fn
    pts = [stamp_of(f, sfm) for f in pair_fn]
    out: list[FrameRef] = []
    if sfm:
        traj_map = read_trajactory(gt)
        for i, j in _pairs_sfm(dts, pts, begin, end, 100 if max_frames is None else max_frames):
            pose = np.array(lower_bound_pose(traj_map, dts[i]), dtype=np.float64)
            out.append(FrameRef(depth_fn[i], rgb_fn[j] if j < len(rgb_fn) else "", mask_fn[j], dts[i], pose, i, j))
    else:
        traj = read_traj(gt)
        for i, j in _pairs_python(dts, pts, begin, end, max_frames):
            pose = P.interpolate_pose(traj, dts[i])
            out.append(FrameRef(depth_fn[i], rgb_fn[j], mask_fn[j] if j < len(mask_fn) else None, dts[i], pose, i, j))
    return out


def load_png(fn: str) -> np.ndarray:
    """PNG reader (16-bit depth, 8-bit mask, RGB).  PIL stands in for cv2.imread."""
    from PIL import Image

    im = Image.open(fn)
    a = np.array(im)
    if a.ndim == 3 and a.shape[2] == 4:
        a = a[:, :, :3]
    return np.ascontiguousarray(a)
