"""Thin object wrapper over one `semtsdf_vol` handle of the C ABI.

All compute goes through libsemtsdf.so (HIP kernels for gfx950); this module only
marshals arguments.  Device buffers for resident frames (bench, multi-frame pipelines) are
allocated through the library too, so no second allocator is involved.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def default_params(dim, intrinsics, width, height) -> L.Params:
    lib = L.load()
    p = L.Params()
    intr = L.f32(intrinsics, 4)
    L.check(lib.semtsdf_params_default(C.byref(p), int(dim), L.ptr(intr), int(width), int(height)))
    return p


def place_from_frame(p: L.Params, depth: np.ndarray, mean_depth: float, mode: int) -> L.Params:
    lib = L.load()
    d = np.ascontiguousarray(depth, dtype=np.uint16)
    if d.size != p.width * p.height:
        raise ValueError("depth size does not match params")
    L.check(lib.semtsdf_place_from_frame(C.byref(p), L.ptr(d), float(mean_depth), int(mode)))
    return p


def orbit_camera(Kinv, angle: float, dist: float):
    lib = L.load()
    ki = L.f32(Kinv, 16)
    s2w = np.zeros(16, np.float32)
    c = np.zeros(3, np.float32)
    L.check(lib.semtsdf_orbit_camera(L.ptr(ki), float(angle), float(dist), L.ptr(s2w), L.ptr(c)))
    return s2w, c


class DeviceBuffer:
    """A device allocation owned by the library's allocator (hipMalloc)."""

    def __init__(self, nbytes: int):
        lib = L.load()
        self.nbytes = int(nbytes)
        self._p = C.c_void_p()
        L.check(lib.semtsdf_dev_malloc(C.byref(self._p), self.nbytes))

    @property
    def ptr(self) -> int:
        return self._p.value

    def upload(self, a: np.ndarray, stream=None, offset: int = 0):
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        L.check(L.load().semtsdf_memcpy(C.c_void_p(self.ptr + offset), L.ptr(a), a.nbytes, 1, stream))

    def copy_from(self, src_ptr: int, nbytes: int, stream=None, offset: int = 0):
        """Device-to-device copy into this buffer (asynchronous on ``stream``)."""
        assert offset + nbytes <= self.nbytes
        L.check(L.load().semtsdf_memcpy(C.c_void_p(self.ptr + offset), C.c_void_p(src_ptr), int(nbytes), 3, stream))

    def download(self, out: np.ndarray, stream=None, offset: int = 0):
        assert out.flags["C_CONTIGUOUS"] and offset + out.nbytes <= self.nbytes
        L.check(L.load().semtsdf_memcpy(L.ptr(out), C.c_void_p(self.ptr + offset), out.nbytes, 2, stream))

    def free(self):
        if self._p.value:
            L.check(L.load().semtsdf_dev_free(self._p))
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Volume:
    def __init__(self, params: L.Params, device: int = 0):
        lib = L.load()
        self.params = params
        self._h = C.c_void_p()
        L.check(lib.semtsdf_create(C.byref(params), int(device), C.byref(self._h)))
        self.W, self.H = params.width, params.height
        st = self.state()
        self.local_dim = tuple(st.local_dim)
        self.nvox = int(st.local_voxels)  # reference layout (dense rows of local_dim[2] planes)

    # ---- lifecycle
    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        return L.load().semtsdf_get_stream(self._h)

    def close(self):
        if self._h and self._h.value:
            L.check(L.load().semtsdf_destroy(self._h))
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        L.check(L.load().semtsdf_reset(self._h, None))

    def get_params(self) -> L.Params:
        p = L.Params()
        L.check(L.load().semtsdf_get_params(self._h, C.byref(p)))
        return p

    def state(self) -> L.State:
        st = L.State()
        L.check(L.load().semtsdf_get_state(self._h, C.byref(st)))
        return st

    def set_state(self, n_obs: int, num_objs: int):
        L.check(L.load().semtsdf_set_state(self._h, int(n_obs), int(num_objs)))

    def sync(self):
        L.check(L.load().semtsdf_stream_sync(C.c_void_p(self.stream)))

    # ---- frames (host pointers)
    def _frame(self, depth, rgb, mask):
        d = np.ascontiguousarray(depth, dtype=np.uint16)
        r = np.ascontiguousarray(rgb, dtype=np.uint8)
        if d.size != self.W * self.H or r.size != self.W * self.H * 3:
            raise ValueError(f"frame must be {self.H}x{self.W} (depth u16, rgb u8x3)")
        m = None
        if mask is not None:
            m = np.ascontiguousarray(mask, dtype=np.uint8)
            if m.size != self.W * self.H:
                raise ValueError("mask must be HxW u8")
        return d, r, m

    def integrate(self, depth, rgb, mask, E):
        d, r, m = self._frame(depth, rgb, mask)
        e = L.f32(E, 16)
        L.check(L.load().semtsdf_integrate(self._h, L.ptr(d), L.ptr(r), L.ptr(m), L.ptr(e), None))

    def associate(self, mask: np.ndarray, E) -> L.AssocStats:
        """Relabels `mask` (u8, C-contiguous) in place and returns the decision."""
        assert mask.dtype == np.uint8 and mask.flags["C_CONTIGUOUS"] and mask.size == self.W * self.H
        st = L.AssocStats()
        e = L.f32(E, 16)
        L.check(L.load().semtsdf_associate(self._h, L.ptr(mask), L.ptr(e), C.byref(st), None))
        return st

    def parse_frame(self, depth, rgb, mask, E) -> L.AssocStats:
        d, r, m = self._frame(depth, rgb, None)
        st = L.AssocStats()
        e = L.f32(E, 16)
        if mask is not None:
            assert mask.dtype == np.uint8 and mask.flags["C_CONTIGUOUS"] and mask.size == self.W * self.H
        L.check(L.load().semtsdf_parse_frame(self._h, L.ptr(d), L.ptr(r), L.ptr(mask), L.ptr(e), C.byref(st), None))
        return st

    def assoc_probs(self, E):
        n = self.W * self.H * L.MAX_OBJECTS
        probs = np.zeros(n, np.float32)
        box = np.zeros(n, np.uint8)
        e = L.f32(E, 16)
        L.check(L.load().semtsdf_assoc_probs(self._h, L.ptr(e), L.ptr(probs), L.ptr(box), None))
        return probs.reshape(self.H, self.W, L.MAX_OBJECTS), box.reshape(self.H, self.W, L.MAX_OBJECTS)

    # ---- device-resident frames
    def integrate_dev(self, depth_ptr: int, rgb_ptr: int, mask_ptr: int | None, E, stream=None):
        e = L.f32(E, 16)
        L.check(L.load().semtsdf_integrate_dev(self._h, C.c_void_p(depth_ptr), C.c_void_p(rgb_ptr),
                                               C.c_void_p(mask_ptr) if mask_ptr else None, L.ptr(e), stream))

    def integrate_dev_async(self, depth_ptr: int, rgb_ptr: int, mask_ptr: int | None, E, inputs_ready=None,
                            stream=None):
        """integrate_dev with the frame prepass on the volume's prep stream, overlapping the
        previous frame's integrate; inputs_ready: a raw hipEvent_t marking the inputs complete
        (None: they already are).  The inputs must not change until this frame has run."""
        e = L.f32(E, 16)
        L.check(L.load().semtsdf_integrate_dev_async(self._h, C.c_void_p(depth_ptr), C.c_void_p(rgb_ptr),
                                                     C.c_void_p(mask_ptr) if mask_ptr else None, L.ptr(e),
                                                     C.c_void_p(inputs_ready) if inputs_ready else None, stream))

    def integrate_vote_dev(self, depth_ptr: int, rgb_ptr: int, cls_ptr: int, E, stream=None):
        e = L.f32(E, 16)
        L.check(L.load().semtsdf_integrate_vote_dev(self._h, C.c_void_p(depth_ptr), C.c_void_p(rgb_ptr),
                                                    C.c_void_p(cls_ptr), L.ptr(e), stream))

    def parse_frame_dev(self, depth_ptr: int, rgb_ptr: int, mask_ptr: int | None, E, stream=None,
                        integrate_after_event: int | None = None):
        """integrate_after_event: a raw hipEvent_t (e.g. torch.cuda.Event.cuda_event) the
        frame's integrate waits for (readers of the previous state on other streams)."""
        e = L.f32(E, 16)
        L.check(L.load().semtsdf_parse_frame_dev_after(self._h, C.c_void_p(depth_ptr), C.c_void_p(rgb_ptr),
                                                       C.c_void_p(mask_ptr) if mask_ptr else None, L.ptr(e),
                                                       C.c_void_p(integrate_after_event) if integrate_after_event
                                                       else None, stream))

    def parse_frame_view_dev(self, depth_ptr: int, rgb_ptr: int, mask_ptr: int | None, E, s2w, c, mode,
                             out_ptr: int, t_ptr: int | None = None, stream=None):
        """parse_frame_dev plus one live view of the volume as it stands before this frame (the
        view shown after the previous frame), rendered in the same launch as this frame's
        association march (semtsdf_parse_frame_view_dev)."""
        e = L.f32(E, 16)
        s = L.f32(s2w, 16)
        cc = L.f32(c, 3)
        L.check(L.load().semtsdf_parse_frame_view_dev(self._h, C.c_void_p(depth_ptr), C.c_void_p(rgb_ptr),
                                                      C.c_void_p(mask_ptr) if mask_ptr else None, L.ptr(e),
                                                      L.ptr(s), L.ptr(cc), int(mode), C.c_void_p(out_ptr),
                                                      C.c_void_p(t_ptr) if t_ptr else None, stream))

    def associate_dev(self, mask_ptr: int, E, stream=None, want_stats=False):
        e = L.f32(E, 16)
        st = L.AssocStats() if want_stats else None
        L.check(L.load().semtsdf_associate_dev(self._h, C.c_void_p(mask_ptr), L.ptr(e),
                                               C.byref(st) if st is not None else None, stream))
        return st

    # ---- render
    def raycast(self, s2w, c, mode=L.RENDER_LABEL, want_t=False):
        out = np.zeros((self.H, self.W, 3), np.uint8)
        t = np.zeros((self.H, self.W), np.float32) if want_t else None
        s = L.f32(s2w, 16)
        cc = L.f32(c, 3)
        L.check(L.load().semtsdf_raycast(self._h, L.ptr(s), L.ptr(cc), int(mode), L.ptr(out), L.ptr(t), None))
        return (out, t) if want_t else out

    def raycast_dev(self, s2w, c, mode, out_ptr: int, t_ptr: int | None = None, stream=None):
        s = L.f32(s2w, 16)
        cc = L.f32(c, 3)
        L.check(L.load().semtsdf_raycast_dev(self._h, L.ptr(s), L.ptr(cc), int(mode), C.c_void_p(out_ptr),
                                             C.c_void_p(t_ptr) if t_ptr else None, stream))

    # ---- state transfer (reference layouts)
    def download(self, sdf=True, wt=True, color=True, hist=False, cls=False):
        n = self.nvox
        ci32 = bool(self.params.flags & L.F_COLOR_I32)
        out = {}
        a_sdf = np.zeros(n, np.float32) if sdf else None
        a_wt = np.zeros(n, np.int32) if wt else None
        a_col = np.zeros(n * 3, np.int32 if ci32 else np.uint8) if color else None
        a_hist = np.zeros(n * L.MAX_OBJECTS, np.uint32) if hist else None
        a_cls = np.zeros(n, np.int32) if cls else None
        a_cnt = np.zeros(n, np.int32) if cls else None
        L.check(L.load().semtsdf_download(self._h, L.ptr(a_sdf), L.ptr(a_wt), L.ptr(a_col), L.ptr(a_hist),
                                          L.ptr(a_cls), L.ptr(a_cnt)))
        for k, v in (("sdf", a_sdf), ("wt", a_wt), ("color", a_col), ("hist", a_hist), ("cls", a_cls),
                     ("cls_cnt", a_cnt)):
            if v is not None:
                out[k] = v
        return out

    def download_slab(self, x0: int, x1: int, sdf=True, wt=True, color=True, hist=False, cls=False):
        """The x-planes [x0, x1) of download() (semtsdf_download_slab)."""
        n = (int(x1) - int(x0)) * int(self.local_dim[1]) * int(self.local_dim[2])
        ci32 = bool(self.params.flags & L.F_COLOR_I32)
        arrs = {"sdf": np.zeros(n, np.float32) if sdf else None, "wt": np.zeros(n, np.int32) if wt else None,
                "color": np.zeros(n * 3, np.int32 if ci32 else np.uint8) if color else None,
                "hist": np.zeros(n * L.MAX_OBJECTS, np.uint32) if hist else None,
                "cls": np.zeros(n, np.int32) if cls else None, "cls_cnt": np.zeros(n, np.int32) if cls else None}
        L.check(L.load().semtsdf_download_slab(self._h, int(x0), int(x1), *[L.ptr(arrs[k]) for k in
                                                                             ("sdf", "wt", "color", "hist", "cls",
                                                                              "cls_cnt")]))
        return {k: v for k, v in arrs.items() if v is not None}

    def upload(self, sdf=None, wt=None, color=None, hist=None, cls=None, cls_cnt=None):
        ci32 = bool(self.params.flags & L.F_COLOR_I32)

        def c(a, dt):
            return None if a is None else np.ascontiguousarray(a, dtype=dt).reshape(-1)

        arrs = [c(sdf, np.float32), c(wt, np.int32), c(color, np.int32 if ci32 else np.uint8), c(hist, np.uint32),
                c(cls, np.int32), c(cls_cnt, np.int32)]
        L.check(L.load().semtsdf_upload(self._h, *[L.ptr(a) for a in arrs]))

    # ---- instrumentation
    def set_instrumentation(self, events: bool = True, count: bool = False, force_exact: bool = False,
                            other_map_passes: bool = False, frame_fold: bool = False):
        """events: HIP-event kernel timing; count: touched/gated voxel counters; force_exact: every
        association row decided from its exact f32 pixel-order sums (tests, cost measurement);
        other_map_passes: the octant maps by the other of their two implementations (tests: same maps);
        frame_fold: parse_frame_view_dev folds the frame's mask statistics and depth pyramid into its
        march launch (tests: same results)."""
        flags = ((1 if events else 0) | (2 if count else 0) | (4 if force_exact else 0) | (8 if other_map_passes else 0)
                 | (16 if frame_fold else 0))
        L.check(L.load().semtsdf_set_instrumentation(self._h, flags))

    def map_words(self):
        """The octant distance map of the current state (numpy uint64 per 8^3 brick, x-major, z
        fastest; byte o = octant o's distance in bricks), or None without octant maps."""
        import numpy as np
        n = C.c_uint64(0)
        L.check(L.load().semtsdf_map_words(self._h, None, 0, C.byref(n)))
        if n.value == 0:
            return None
        out = np.zeros(n.value, dtype=np.uint64)
        L.check(L.load().semtsdf_map_words(self._h, C.c_void_p(out.ctypes.data), n.value, C.byref(n)))
        return out

    def filter_overlaps_dev(self, probs_ptr: int, box_ptr: int, mask_ptr: int, stream=None) -> L.AssocStats:
        """TSDF::filter_overlaps (tsdf.cu:304-416) on device arrays: probs f32 [H*W][32], box u8
        [H*W][32], mask u8 [H*W] relabelled in place; uses this handle's n_obs and num_objs."""
        st = L.AssocStats()
        L.check(L.load().semtsdf_filter_overlaps_dev(self._h, C.c_void_p(probs_ptr), C.c_void_p(box_ptr),
                                                     C.c_void_p(mask_ptr), C.byref(st), stream))
        return st

    def timing(self) -> L.Timing:
        t = L.Timing()
        L.check(L.load().semtsdf_get_timing(self._h, C.byref(t)))
        return t

    def reset_timing(self):
        L.check(L.load().semtsdf_reset_timing(self._h))
