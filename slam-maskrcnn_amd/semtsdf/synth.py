"""Seeded synthetic RGB-D + instance-mask stream.

Scene in frame-0 camera coordinates (= volume coordinates):
  * back wall plane z = 3.0 m (instance 0 / background);
  * 6 spheres, radius U(0.15, 0.35) m, centres uniform inside the frustum at z in
    [1.2, 2.4] m; sphere k is instance k+1;
  * per-object base colour U{0..255}^3 with a +-16 checker texture (u8);
  * depth = analytic ray-hit z, round(z * 5000) as u16; 2 % seeded dropout pixels = 0;
    optional Gaussian noise sigma = 1.5 mm * z^2 (bench) — parity runs use none;
  * camera k: yaw 0.004 k rad about y, translation (0.01 k, 0, 0.005 k) m (C2W, frame 0 = I).
Per-frame masks follow the Mask R-CNN contract of Mask_RCNN/dmask.py:127-165: objects with
<= 2000 px are dropped (filter_tiny_objects), overlaps resolved by depth (nearest surface
wins, which is what a visible-instance mask shows) and labels are a per-frame permutation of
the visible objects (i+1 for the i-th detection), so the association has real work to do.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from . import pose as P
from .config import DEPTH_SCALE, FRAME_H, FRAME_W, TUM_INTRINSICS


@dataclass
class Frame:
    depth: np.ndarray      # u16 [H, W]
    rgb: np.ndarray        # u8 [H, W, 3]
    mask: np.ndarray       # u8 [H, W] per-frame instance labels
    gt_ids: np.ndarray     # u8 [H, W] ground-truth global instance ids (1 + sphere index)
    c2w: np.ndarray        # f64 4x4
    w2c: np.ndarray        # f64 4x4 (extrinsic)
    ts: float


class SyntheticStream:
    def __init__(self, seed: int = 0, width: int = FRAME_W, height: int = FRAME_H,
                 intrinsics=TUM_INTRINSICS, n_spheres: int = 6, noise: bool = False,
                 dropout: float = 0.02, min_area: int = 2000, permute_labels: bool = True,
                 yaw_step: float = 0.004, trans_step=(0.01, 0.0, 0.005)):
        self.seed = seed
        self.W, self.H = width, height
        self.fx, self.fy, self.cx, self.cy = intrinsics
        rng = np.random.default_rng(seed)
        self.radius = rng.uniform(0.15, 0.35, n_spheres)
        zc = rng.uniform(1.2, 2.4, n_spheres)
        u = rng.uniform(0.15 * width, 0.85 * width, n_spheres)
        v = rng.uniform(0.15 * height, 0.85 * height, n_spheres)
        self.centres = np.stack([(u - self.cx) / self.fx * zc, (v - self.cy) / self.fy * zc, zc], axis=1)
        self.colours = rng.integers(0, 256, (n_spheres + 1, 3))
        self.wall_z = 3.0
        self.noise = noise
        self.dropout = dropout
        self.min_area = min_area
        self.permute = permute_labels
        self.yaw_step = yaw_step
        self.trans_step = np.asarray(trans_step, dtype=np.float64)
        self.n_spheres = n_spheres
        j, i = np.meshgrid(np.arange(width), np.arange(height))
        self._rays = np.stack([(j - self.cx) / self.fx, (i - self.cy) / self.fy, np.ones_like(j, dtype=np.float64)],
                              axis=-1)
        self._checker = (((j // 8) + (i // 8)) % 2 * 32 - 16).astype(np.int64)

    def c2w(self, k: int) -> np.ndarray:
        a = self.yaw_step * k
        m = np.eye(4)
        m[:3, :3] = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
        m[:3, 3] = self.trans_step * k
        return m

    def frame(self, k: int) -> Frame:
        c2w = self.c2w(k)
        R, t = c2w[:3, :3], c2w[:3, 3]
        dirs = self._rays @ R.T             # world directions (unnormalised, camera z = 1)
        fwd = R[:, 2]                        # camera z axis in world
        best = np.full(dirs.shape[:2], np.inf)
        obj = np.zeros(dirs.shape[:2], dtype=np.int64)
        # wall z = wall_z (world): t + s * d, s = (wall - t_z) / d_z
        with np.errstate(divide="ignore", invalid="ignore"):
            s_wall = (self.wall_z - t[2]) / dirs[..., 2]
        s_wall = np.where(s_wall > 0, s_wall, np.inf)
        best = s_wall
        for n in range(self.n_spheres):
            oc = t - self.centres[n]
            a = np.einsum("hwc,hwc->hw", dirs, dirs)
            b = 2.0 * np.einsum("hwc,c->hw", dirs, oc)
            c = float(oc @ oc) - self.radius[n] ** 2
            disc = b * b - 4 * a * c
            ok = disc > 0
            sq = np.sqrt(np.where(ok, disc, 0.0))
            s0 = (-b - sq) / (2 * a)
            hit = ok & (s0 > 0) & (s0 < best)
            best = np.where(hit, s0, best)
            obj = np.where(hit, n + 1, obj)
        # camera-space depth of the hit = s * (d . fwd) with d the unnormalised ray (z_cam = s)
        z = best * np.einsum("hwc,c->hw", dirs, fwd)
        rng = np.random.default_rng(self.seed * 1000003 + k)
        if self.noise:
            z = z + rng.normal(0.0, 1.0, z.shape) * (0.0015 * z * z)
        depth = np.where(np.isfinite(z) & (z > 0), np.round(z * DEPTH_SCALE), 0)
        depth = np.clip(depth, 0, 65535).astype(np.uint16)
        drop = rng.random(depth.shape) < self.dropout
        depth[drop] = 0
        base = self.colours[obj]
        rgb = np.clip(base + self._checker[..., None], 0, 255).astype(np.uint8)
        gt = obj.astype(np.uint8)
        gt[depth == 0] = 0
        # Mask R-CNN-like per-frame labels
        mask = np.zeros_like(gt)
        present = [n for n in range(1, self.n_spheres + 1) if int((gt == n).sum()) > self.min_area]
        order = list(present)
        if self.permute:
            rng.shuffle(order)
        for lab, n in enumerate(order, start=1):
            mask[gt == n] = lab
        w2c = np.linalg.inv(c2w)
        return Frame(depth, np.ascontiguousarray(rgb), mask, gt, c2w, w2c, self.stamp(k))

    # TUM stamps of the fr2 sequences (1311868164.xxxx); the reference drivers drop the first
    # five characters (kernel.cpp:53, tsdf_utils.py:27), leaving 68164.xxxx
    STAMP0 = 1311868164.0

    def stamp(self, k: int) -> float:
        return self.STAMP0 + 0.033 * k

    def tum_lines(self, n: int) -> list[str]:
        """groundtruth.txt lines (camera-to-world) of frames 0..n-1, '# ...' header first."""
        return ["# timestamp tx ty tz qx qy qz qw"] + [P.c2w_to_tum(self.stamp(k), self.c2w(k)) for k in range(n)]
