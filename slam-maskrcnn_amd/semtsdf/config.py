"""Configuration knobs of the fusion path.

`Configuration` keeps the reference's two static knobs with the same names and values
(src/SfM_CUDA/configuration.h:2-9).  `duplicate_thresh` is declared there but never read
by the reference; it is kept (and passed through the C ABI) for drop-in compatibility and
is unused here too.  The remaining constants are the hard-coded values SURVEY.md §8a
(row a10) lists, each with its reference location.
"""
from __future__ import annotations

from dataclasses import dataclass, field


class Configuration:
    """Drop-in for `class Configuration` (configuration.h:2-6)."""

    prior_mrcnn_err_rate: float = 0.05  # configuration.h:8
    duplicate_thresh: float = 0.5       # configuration.h:9 (unused by the reference)


MAX_OBJECTS = 32                 # tsdf.cuh:4
DEFAULT_VOL_DIM = 256            # tsdf.cuh:52, tsdf.py:21
DEPTH_SCALE = 5000.0             # tsdf.cu:49, tsdf.py:38,101
GATE = 0.99                      # tsdf.cu:57
BOX_THRESH = 0.3                 # tsdf.cu:128
MU_VOXELS = 5.0                  # tsdf.cu:199, tsdf.py:47
TUM_INTRINSICS = (520.9, 521.0, 325.1, 249.7)  # kernel.cpp:39, TSDF_Python/main.py:72
FRAME_W, FRAME_H = 640, 480


@dataclass
class FusionConfig:
    """Every constant of the hot path in one place (SURVEY.md §5 'Config / flags')."""

    vol_dim: int = DEFAULT_VOL_DIM
    intrinsics: tuple = TUM_INTRINSICS
    width: int = FRAME_W
    height: int = FRAME_H
    depth_scale: float = DEPTH_SCALE
    gate: float = GATE
    box_thresh: float = BOX_THRESH
    prior_mrcnn_err_rate: float = field(default_factory=lambda: Configuration.prior_mrcnn_err_rate)
    duplicate_thresh: float = field(default_factory=lambda: Configuration.duplicate_thresh)
    semantic: bool = True            # SfM design A: 32-bin histogram
    gate_color: bool = True          # SfM: colour/histogram only for f < gate
    color_i32: bool = False          # TSDF_Python stores int32 colour
    vote: bool = False               # TSDF_Python design B label vote
    integrate_first_frame: bool = False  # SfM places only; TSDF_Python integrates frame 0
    placement: str = "sfm"           # "sfm" (f32, metres) | "python" (f64, raw units)
    cull: bool = True
