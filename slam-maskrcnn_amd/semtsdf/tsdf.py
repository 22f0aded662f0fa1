"""Host-side `TSDF` class: the drop-in surface of src/TSDF_Python/tsdf.py (attributes and
`parse_frame` signature of tsdf.py:10-178) driving the SfM_CUDA semantics of
src/SfM_CUDA/tsdf.cu:137-540 (instance histogram, association, relabel) through the C ABI.

Differences from the reference, by design:
  * the intrinsic matrix is built with a tuple index (tsdf.py:13 relies on pre-1.23 NumPy
    list-index semantics and yields a singular K on NumPy 2);
  * the volume lives on the GPU; `tsdf_diff`, `tsdf_wt`, `tsdf_color`, `tsdf_cnt`,
    `tsdf_cls`, `tsdf_cls_cnt` are read-only views downloaded on access, in the TSDF_Python
    2-D layout `[tex_dim, tex_dim]` when D^3 is a perfect square and flat `[D^3]` otherwise
    (tsdf.py:22 truncates when it is not);
  * first-frame behaviour is a flag: SfM places without integrating (tsdf.cu:173-214),
    TSDF_Python integrates frame 0 (tsdf.py:55-57).
"""
from __future__ import annotations

import dataclasses
import json
import math

import numpy as np

from . import _lib as L
from . import pose as P
from .config import Configuration, FusionConfig
from .volume import Volume, default_params, orbit_camera, place_from_frame


def bounding_rect_nonzero(a: np.ndarray):
    """cv2.boundingRect(cv2.findNonZero(a)) -> (x, y, w, h)."""
    ys, xs = np.nonzero(a)
    if xs.size == 0:
        raise ValueError("no non-zero pixel")
    x0, x1, y0, y1 = int(xs.min()), int(xs.max()), int(ys.min()), int(ys.max())
    return x0, y0, x1 - x0 + 1, y1 - y0 + 1


class TSDF:
    def __init__(self, intrinsics, vol_dim: int | None = None, config: FusionConfig | None = None, device: int = 0):
        cfg = config or FusionConfig()
        if vol_dim is not None:
            cfg.vol_dim = int(vol_dim)
        cfg.intrinsics = tuple(float(x) for x in intrinsics)
        self.config = cfg
        self.device = device
        self.intrinsic = np.eye(4, dtype=np.float32)
        self.intrinsic[(0, 1, 0, 1), (0, 1, 2, 2)] = np.array(intrinsics, dtype=np.float32)
        self.init = False
        self.mu = 0
        self.vol_dim = cfg.vol_dim
        self.tex_dim = int(np.sqrt(pow(self.vol_dim, 3)))
        self.voxel = [0] * 3
        self.vol_start = None
        self.vol_end = None
        self.intrinsic_inv = np.linalg.inv(self.intrinsic)
        self.init_extrinsic_inv = None
        self.mean_depth = 0
        self.num_cls = 0
        self.N = 0
        self.vol: Volume | None = None
        self.last_assoc: L.AssocStats | None = None

    # ------------------------------------------------------------------ placement (a1)
    def _flags(self) -> int:
        c = self.config
        f = 0
        if c.vote:
            f |= L.F_VOTE | L.F_COLOR_I32
        else:
            if c.semantic:
                f |= L.F_SEMANTIC
            if c.gate_color:
                f |= L.F_GATE_COLOR
            if c.color_i32:
                f |= L.F_COLOR_I32
        if not c.cull:
            f |= L.F_NO_CULL
        return f

    def init_vars(self, depth, color, extrinsic, mean_depth):
        """tsdf.py:32-52 (placement="python": mean_depth in raw units, float64) or
        tsdf.cu:173-212 (placement="sfm": mean_depth in metres, float32)."""
        c = self.config
        depth = np.ascontiguousarray(depth, dtype=np.uint16)
        self.init = True
        self.init_extrinsic_inv = np.linalg.inv(np.asarray(extrinsic, dtype=np.float64))
        p = default_params(c.vol_dim, c.intrinsics, depth.shape[1], depth.shape[0])
        p.depth_scale = c.depth_scale
        p.gate = c.gate
        p.box_thresh = c.box_thresh
        p.prior_mrcnn_err_rate = c.prior_mrcnn_err_rate
        p.duplicate_thresh = c.duplicate_thresh
        p.flags = self._flags()
        if c.placement == "python":
            rect = bounding_rect_nonzero(depth.astype(np.uint8))
            kinv = self.intrinsic_inv
            tl = np.dot(kinv[:3, :3], [rect[0], rect[1], 1])
            br = np.dot(kinv[:3, :3], [rect[0] + rect[2], rect[1] + rect[3], 1])
            tl *= mean_depth / 5000
            br *= mean_depth / 5000
            self.mean_depth = mean_depth / 5000
            half_side = np.sqrt(np.dot(tl[:2] - br[:2], tl[:2] - br[:2])) / 2
            center = (tl + br) / 2
            self.vol_start = center - half_side
            self.vol_end = center + half_side
            self.voxel = (self.vol_end - self.vol_start) / (self.vol_dim - 1)
            self.mu = 5 * self.voxel[0]
            for i in range(3):
                p.vol_start[i] = self.vol_start[i]
                p.vol_end[i] = self.vol_end[i]
                p.voxel[i] = self.voxel[i]
            p.mu = self.mu
            for i in range(16):
                p.Kinv[i] = float(self.intrinsic_inv.reshape(-1)[i])
        else:
            place_from_frame(p, depth, float(mean_depth), L.PLACE_SFM)
            self.mean_depth = float(mean_depth)
            self.vol_start = np.array(p.vol_start[:], dtype=np.float32)
            self.vol_end = np.array(p.vol_end[:], dtype=np.float32)
            self.voxel = np.array(p.voxel[:], dtype=np.float32)
            self.mu = float(p.mu)
            self.intrinsic_inv = np.array(p.Kinv[:], dtype=np.float32).reshape(4, 4)
        self.vol = Volume(p, self.device)

    # ------------------------------------------------------------------ per frame (a7)
    def parse_frame(self, depth, color, extrinsic, mean_depth, masks=None):
        """tsdf.py:54 signature.  Returns the association decision (or None)."""
        if not self.init:
            self.init_vars(depth, color, extrinsic, mean_depth)
            if self.config.integrate_first_frame:
                return self.parse_frame(depth, color, extrinsic, mean_depth, masks)
            return None
        E = P.relative_pose(extrinsic, self.init_extrinsic_inv)
        v = self.vol
        if self.config.vote:
            cls = np.ascontiguousarray(np.asarray(masks), dtype=np.int32).reshape(-1)[: v.W * v.H]
            self._vote_frame(depth, color, cls, E)
            self.N += 1
            return None
        m = None
        if self.config.semantic:
            if masks is None:
                raise ValueError("semantic fusion needs a mask")
            m = np.asarray(masks)
            if m.ndim == 3:  # cv2.imread default loads a label PNG as 3 equal channels
                m = m[:, :, 0]
            m = np.ascontiguousarray(m, dtype=np.uint8)
            self.num_cls = int(m.max()) if m.size else 0
        st = v.parse_frame(depth, color, m, E)
        if m is not None and masks is not None and isinstance(masks, np.ndarray) and masks.dtype == np.uint8 \
                and masks.shape == m.shape and masks.flags["C_CONTIGUOUS"]:
            masks[...] = m  # relabelled in place (tsdf.cu:376-386: Mat& masks)
        self.N += 1
        self.last_assoc = st
        return st

    def _vote_frame(self, depth, color, cls, E):
        from .volume import DeviceBuffer

        v = self.vol
        d = np.ascontiguousarray(depth, dtype=np.uint16)
        r = np.ascontiguousarray(color, dtype=np.uint8)
        bufs = [DeviceBuffer(d.nbytes), DeviceBuffer(r.nbytes), DeviceBuffer(cls.nbytes)]
        bufs[0].upload(d, v.stream)
        bufs[1].upload(r, v.stream)
        bufs[2].upload(cls, v.stream)
        v.integrate_vote_dev(bufs[0].ptr, bufs[1].ptr, bufs[2].ptr, E)
        v.sync()
        for b in bufs:
            b.free()

    # ------------------------------------------------------------------ views
    @property
    def n_obs(self) -> int:
        return int(self.vol.state().n_obs) if self.vol else 0

    @property
    def num_objs(self) -> int:
        return int(self.vol.state().num_objs) if self.vol else 0

    def _shape(self, a, ch=None):
        D = self.vol_dim
        if self.tex_dim * self.tex_dim == D ** 3:
            shp = (self.tex_dim, self.tex_dim)
        else:
            shp = (D ** 3,)
        return a.reshape(shp + ((ch,) if ch else ()))

    @property
    def tsdf_diff(self):
        return None if self.vol is None else self._shape(self.vol.download(wt=False, color=False)["sdf"])

    @property
    def tsdf_wt(self):
        return None if self.vol is None else self._shape(self.vol.download(sdf=False, color=False)["wt"])

    @property
    def tsdf_color(self):
        return None if self.vol is None else self._shape(self.vol.download(sdf=False, wt=False)["color"], 3)

    @property
    def tsdf_cnt(self):
        if self.vol is None or not (self.vol.params.flags & L.F_SEMANTIC):
            return None
        return self.vol.download(sdf=False, wt=False, color=False, hist=True)["hist"].reshape(-1, L.MAX_OBJECTS)

    @property
    def tsdf_cls(self):
        if self.vol is None or not (self.vol.params.flags & L.F_VOTE):
            return None
        return self._shape(self.vol.download(sdf=False, wt=False, color=False, cls=True)["cls"])

    @property
    def tsdf_cls_cnt(self):
        if self.vol is None or not (self.vol.params.flags & L.F_VOTE):
            return None
        return self._shape(self.vol.download(sdf=False, wt=False, color=False, cls=True)["cls_cnt"])

    # ------------------------------------------------------------------ raycast (a8)
    def render(self, angle: float, mode: str = "label", dist: float | None = None):
        """Viewer::show_tsdf (viewer.cu:137-179) without the window: BGR u8 image."""
        s2w, c = orbit_camera(self.intrinsic_inv, angle, self.mean_depth if dist is None else dist)
        return self.vol.raycast(s2w, c, L.RENDER_LABEL if mode == "label" else L.RENDER_COLOR)

    def orbit(self, n: int, out_dir: str | None = None, mode: str = "label", step: float = 0.01, callback=None):
        """The reference's view loop (kernel.cpp:101-107: angle += 0.01 per view at the mean
        depth) headless: n views written as PNG files to out_dir, or handed to callback(k,
        angle, bgr), or returned (semtsdf.orbit.orbit_views)."""
        from .orbit import orbit_views

        return orbit_views(self.vol, self.intrinsic_inv, self.mean_depth, n, mode, step, out_dir=out_dir,
                           callback=callback)

    # ------------------------------------------------------------------ checkpoint (§8f rank 3)
    def save(self, path: str):
        v = self.vol
        sem = bool(v.params.flags & L.F_SEMANTIC)
        vote = bool(v.params.flags & L.F_VOTE)
        data = v.download(hist=sem, cls=vote)
        st = v.state()
        # every field of the volume's semtsdf_params (placement, intrinsics and their inverse,
        # frame size, thresholds, knobs, flags, shard), so a reloaded volume integrates,
        # associates and renders exactly like the saved one
        params = {f"p_{name}": np.array(getattr(v.params, name)[:] if hasattr(getattr(v.params, name), "__len__")
                                        else getattr(v.params, name)) for name, _ in L.Params._fields_}
        np.savez_compressed(
            path, vol_start=np.asarray(self.vol_start, np.float64), vol_end=np.asarray(self.vol_end, np.float64),
            voxel=np.asarray(self.voxel, np.float64), mu=np.float64(self.mu), vol_dim=np.int64(self.vol_dim),
            n_obs=np.int64(st.n_obs), num_objs=np.int64(st.num_objs), N=np.int64(self.N),
            mean_depth=np.float64(self.mean_depth), init_extrinsic_inv=self.init_extrinsic_inv,
            intrinsic=self.intrinsic, intrinsic_inv=np.asarray(self.intrinsic_inv), flags=np.int64(v.params.flags),
            config=np.str_(json.dumps(dataclasses.asdict(self.config))), **params, **data)

    @classmethod
    def load(cls, path: str, config: FusionConfig | None = None, device: int = 0) -> "TSDF":
        """Restores a checkpoint written by save(): the volume's full parameter block (not the
        defaults), the host attributes and the configuration it was saved with (`config`, if
        given, overrides the saved one for future host-side choices only)."""
        z = np.load(path, allow_pickle=False)
        K = z["intrinsic"]
        if config is None and "config" in z:
            d = json.loads(str(z["config"]))
            d["intrinsics"] = tuple(d["intrinsics"])
            config = FusionConfig(**d)
        t = cls((float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])), int(z["vol_dim"]), config, device)
        t.init = True
        t.vol_start, t.vol_end, t.voxel = z["vol_start"], z["vol_end"], z["voxel"]
        t.mu = float(z["mu"])
        t.mean_depth = float(z["mean_depth"])
        t.init_extrinsic_inv = z["init_extrinsic_inv"]
        t.N = int(z["N"])
        if "intrinsic_inv" in z:
            t.intrinsic_inv = z["intrinsic_inv"]
        p = L.Params()
        if "p_flags" in z:
            for name, ctype in L.Params._fields_:
                val = z[f"p_{name}"]
                if hasattr(getattr(p, name), "__len__"):
                    getattr(p, name)[:] = [x.item() for x in val.reshape(-1)]
                else:
                    setattr(p, name, val.item())
        else:  # checkpoints of ABI 2: geometry and flags only, defaults for the rest
            p = default_params(t.vol_dim, t.config.intrinsics, t.config.width, t.config.height)
            for i in range(3):
                p.vol_start[i], p.vol_end[i], p.voxel[i] = t.vol_start[i], t.vol_end[i], t.voxel[i]
            p.mu = t.mu
            p.flags = int(z["flags"])
        t.vol = Volume(p, device)
        t.vol.upload(sdf=z["sdf"], wt=z["wt"], color=z["color"], hist=z["hist"] if "hist" in z else None,
                     cls=z["cls"] if "cls" in z else None, cls_cnt=z["cls_cnt"] if "cls_cnt" in z else None)
        t.vol.set_state(int(z["n_obs"]), int(z["num_objs"]))
        return t

    def close(self):
        if self.vol is not None:
            self.vol.close()
            self.vol = None


def orbit_angle_sequence(n: int, step: float = 0.01):
    """kernel.cpp:101-107: angle += 0.01 per view."""
    return [step * (k + 1) for k in range(n)]


__all__ = ["TSDF", "Configuration", "FusionConfig", "bounding_rect_nonzero", "orbit_angle_sequence", "math"]
