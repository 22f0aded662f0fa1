"""ORACLE — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline.  The product (libsemtsdf.so and
the `semtsdf` host package) never imports it.

Contents
  * ctypes loader of liboracle.so, the scalar C restatement in semtsdf_oracle.c (bit-level
    reference for the HIP kernels: integrate, association raycast, filter_overlaps,
    render, placement).
  * `numpy_integrate` — a NumPy restatement of the reference's vectorised integrate, the
    commented block src/TSDF_Python/tsdf.py:78-120 (float64 arithmetic, results stored
    to the array dtypes), extended with the SfM_CUDA semantic gate + instance histogram
    (src/SfM_CUDA/tsdf.cu:57-62) for semantic mode, and chunked along x so 512^3 fits in
    RAM.  It is pinned against golden vectors produced by executing the reference block
    itself (tests/golden/gen_golden.py, tests/test_oracle_golden.py).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "semtsdf_oracle.c")
# ORACLE_SANITIZE=1: an AddressSanitizer + UndefinedBehaviorSanitizer build (host code only;
# the Python process needs libasan preloaded, tests/test_oracle_sanitize.py does that)
SANITIZE = os.environ.get("ORACLE_SANITIZE") == "1"
LIB = os.path.join(HERE, "liboracle_san.so" if SANITIZE else "liboracle.so")
SAN_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"]
OMAX = 32


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        opt = SAN_FLAGS if SANITIZE else ["-O2"]
        cmd = ["gcc", *opt, "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", "-std=c11", SRC, "-o", LIB,
               "-lm"]
        subprocess.check_call(cmd)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        P = C.c_void_p
        _lib.oracle_integrate.argtypes = [P, P, P, P, C.c_int, C.c_int, C.c_uint32, P, P, P, P, P, P, P, P, P, P,
                                          C.c_int, C.c_int, P, P, C.c_int]
        _lib.oracle_integrate.restype = None
        _lib.oracle_integrate_slab.argtypes = [P, P, P, P, C.c_int, C.c_int, C.c_uint32, P, P, P, P, P, P, P, P, P,
                                               P, C.c_int, C.c_int, P]
        _lib.oracle_integrate_slab.restype = None
        _lib.oracle_march_probs.argtypes = [P, P, P, P, C.c_int, C.c_int, P, P, C.c_float, P, P, C.c_int, C.c_int]
        _lib.oracle_march_probs.restype = None
        _lib.oracle_filter_overlaps.argtypes = [P, P, P, C.c_int, C.c_int, C.c_uint32, C.c_float, C.c_int, P, P, P, P,
                                                C.c_int]
        _lib.oracle_filter_overlaps.restype = C.c_int
        _lib.oracle_render.argtypes = [P, P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, P, C.c_int,
                                       C.c_int]
        _lib.oracle_render.restype = None
        _lib.oracle_shard_render_step.argtypes = [P, P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, C.c_int,
                                                  C.c_int, C.c_int, C.c_int, P, P, P, P, P]
        _lib.oracle_shard_render_step.restype = None
        _lib.oracle_div_rcp_mismatches.argtypes = [P, C.c_int, C.c_float]
        _lib.oracle_div_rcp_mismatches.restype = C.c_int
        _lib.oracle_place.argtypes = [P, C.c_int, C.c_int, P, P, C.c_double, C.c_int, P]
        _lib.oracle_place.restype = C.c_int
        _lib.oracle_orbit_camera.argtypes = [P, C.c_float, C.c_float, P, P]
        _lib.oracle_orbit_camera.restype = None
        _lib.oracle_project.argtypes = [P, P, P, P, C.c_int, C.c_int, P, C.c_int, C.c_int]
        _lib.oracle_project.restype = None
        _lib.oracle_libm_mismatches.argtypes = [C.c_int, P, P, C.c_long, C.c_uint32]
        _lib.oracle_libm_mismatches.restype = C.c_long
        _lib.oracle_logf_ulp_max.argtypes = [P, C.c_long, C.c_uint32]
        _lib.oracle_logf_ulp_max.restype = C.c_double
    return _lib


def _p(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be contiguous"
    return C.c_void_p(a.ctypes.data)


class OGeom:
    """Volume geometry for the C oracle (f32 values exactly as given to the kernels)."""

    def __init__(self, dims, vol_start, voxel, mu, vol_end=None, depth_scale=5000.0, gate=0.99):
        self.dims = np.ascontiguousarray(np.asarray(dims, np.int32).reshape(3))
        vs = np.asarray(vol_start, np.float32).reshape(3)
        vx = np.asarray(voxel, np.float32).reshape(3)
        ve = np.asarray(vol_end, np.float32).reshape(3) if vol_end is not None else \
            (vs + vx * (self.dims - 1).astype(np.float32)).astype(np.float32)
        self.geo = np.zeros(12, np.float32)
        self.geo[0:3] = vs
        self.geo[3:6] = vx
        self.geo[6] = np.float32(mu)
        self.geo[7] = np.float32(depth_scale)
        self.geo[8] = np.float32(gate)
        self.geo[9:12] = ve

    @classmethod
    def from_params(cls, p):
        return cls(list(p.dim), list(p.vol_start), list(p.voxel), p.mu, list(p.vol_end), p.depth_scale, p.gate)


def k9(K16):
    K = np.asarray(K16, np.float32).reshape(4, 4)
    return np.ascontiguousarray(K[:3, :3].reshape(9))


class OState:
    """Reference-layout volume state for the C oracle."""

    def __init__(self, dims, mu, semantic=False, color_i32=False, vote=False, lz=None):
        n = int(dims[0]) * int(dims[1]) * int(dims[2] if lz is None else lz)
        self.sdf = np.full(n, np.float32(mu), np.float32)
        self.wt = np.zeros(n, np.int32)
        self.color = np.zeros(n * 3, np.int32 if color_i32 else np.uint8)
        self.hist = np.zeros(n * OMAX, np.uint32) if semantic else None
        self.cls = np.zeros(n, np.int32) if vote else None
        self.cls_cnt = np.zeros(n, np.int32) if vote else None


def integrate(g: OGeom, st: OState, K16, E16, depth, rgb, mask=None, cls=None, flags=0x3, x_range=None, zmap=None):
    """zmap: global z of each local plane (a Z-slab shard); st must then be sized
    dims[0] x dims[1] x len(zmap)."""
    H, W = depth.shape[:2]
    x0, x1 = (0, int(g.dims[0])) if x_range is None else x_range
    counts = np.zeros(3, np.uint64)
    zm = None if zmap is None else np.ascontiguousarray(zmap, np.int32)
    lib().oracle_integrate(_p(g.dims), _p(g.geo), _p(k9(K16)), _p(np.ascontiguousarray(E16, np.float32).reshape(16)),
                           W, H, flags, _p(st.sdf), _p(st.wt), _p(st.color), _p(st.hist), _p(st.cls), _p(st.cls_cnt),
                           _p(np.ascontiguousarray(depth, np.uint16)), _p(np.ascontiguousarray(rgb, np.uint8)),
                           _p(None if mask is None else np.ascontiguousarray(mask, np.uint8)),
                           _p(None if cls is None else np.ascontiguousarray(cls, np.int32)), x0, x1, _p(counts),
                           _p(zm), 0 if zm is None else int(zm.size))
    return counts


def project(g: OGeom, K16, E16, W, H, x_range=None):
    """Pixel index (y*W + x, -1 off-image) of every voxel under the f32 contract."""
    x0, x1 = (0, int(g.dims[0])) if x_range is None else x_range
    out = np.full(int(np.prod(g.dims)), -1, np.int32)
    lib().oracle_project(_p(g.dims), _p(g.geo), _p(k9(K16)), _p(np.ascontiguousarray(E16, np.float32).reshape(16)),
                         int(W), int(H), _p(out), x0, x1)
    return out


def numpy_pixels(vol_dim, vol_start, voxel, K, E, W, H, n_flat=None):
    """Pixel index (-1 where rejected) of every flat voxel under the float64 reference block
    (tsdf.py:86-97: f64 pose, f32 K, truncation toward zero, bounds on the truncated value)."""
    D = int(vol_dim)
    n = D ** 3 if n_flat is None else int(n_flat)
    flat = np.arange(n, dtype=np.int64)
    xi = flat // (D * D)
    yi = flat // D - xi * D
    zi = flat % D
    vs = np.asarray(vol_start, np.float64)
    vx = np.asarray(voxel, np.float64) * np.ones(3)
    pos = np.stack([vs[0] + xi * vx[0], vs[1] + yi * vx[1], vs[2] + zi * vx[2], np.ones(n)], axis=0)
    proj = np.dot(np.asarray(E, np.float64), pos)
    pixel = np.dot(np.asarray(K, np.float32), proj)
    pixel /= pixel[2, :]
    px = pixel[0].astype(np.int64)
    py = pixel[1].astype(np.int64)
    ok = (px >= 0) & (px <= W - 1) & (py >= 0) & (py <= H - 1)
    return np.where(ok, py * W + px, -1)


def integrate_slab(g: OGeom, st: OState, K16, E16, depth, rgb, x_range, mask=None, flags=0x3):
    """Integrate x-planes [x0, x1) into a state holding only those planes (OState with
    dims (x1 - x0, Dy, Dz)), with the global voxel coordinates."""
    H, W = depth.shape[:2]
    counts = np.zeros(3, np.uint64)
    lib().oracle_integrate_slab(_p(g.dims), _p(g.geo), _p(k9(K16)),
                                _p(np.ascontiguousarray(E16, np.float32).reshape(16)), W, H, flags, _p(st.sdf),
                                _p(st.wt), _p(st.color), _p(st.hist), _p(st.cls), _p(st.cls_cnt),
                                _p(np.ascontiguousarray(depth, np.uint16)), _p(np.ascontiguousarray(rgb, np.uint8)),
                                _p(None if mask is None else np.ascontiguousarray(mask, np.uint8)), None,
                                int(x_range[0]), int(x_range[1]), _p(counts))
    return counts


def march_probs(g: OGeom, Kinv16, E16, W, H, sdf, hist, box_thresh=0.3):
    probs = np.zeros(W * H * OMAX, np.float32)
    box = np.zeros(W * H * OMAX, np.uint8)
    lib().oracle_march_probs(_p(g.dims), _p(g.geo), _p(k9(Kinv16)), _p(np.ascontiguousarray(E16, np.float32).reshape(16)),
                             W, H, _p(sdf), _p(hist), box_thresh, _p(probs), _p(box), 0, H)
    return probs, box


def filter_overlaps(probs, box, mask, n_obs, num_objs, eps=0.05, precision=0, table=None, id_policy=0):
    """Relabels a copy of mask; returns (mask, num_objs, max_obj_now, assigned_prev, assigned_prob).
    id_policy 0: the reference's unbounded new ids (held in the u8 mask modulo 256); 1: new ids
    >= 32 become background (the engine's opt-in SEMTSDF_F_ID_SATURATE).
    precision 0: the reference's f32 rule (logf terms summed in pixel order, expf of the f32
    mean, tsdf.cu:312-349), which the device reproduces; 1: double accumulation (tests only).
    table: optional float64 [32, 32] that receives every candidate probability (row = current
    label, column = previous id)."""
    H, W = mask.shape
    m = np.ascontiguousarray(mask, np.uint8).copy()
    no = C.c_int(int(num_objs))
    prev = np.zeros(OMAX, np.int32)
    prob = np.zeros(OMAX, np.float32)
    if table is not None:
        assert table.dtype == np.float64 and table.shape == (OMAX, OMAX) and table.flags["C_CONTIGUOUS"]
        table[:] = 0.0
    mx = lib().oracle_filter_overlaps(_p(np.ascontiguousarray(probs, np.float32)),
                                      _p(np.ascontiguousarray(box, np.uint8)), _p(m), W, H, int(n_obs), eps,
                                      int(precision), C.byref(no), _p(prev), _p(prob), _p(table),
                                      int(id_policy))
    return m, no.value, mx, prev, prob


def render(g: OGeom, s2w, c, W, H, mode, sdf, hist=None, color=None, color_i32=False):
    out = np.zeros(W * H * 3, np.uint8)
    t = np.zeros(W * H, np.float32)
    lib().oracle_render(_p(g.dims), _p(g.geo), _p(np.ascontiguousarray(s2w, np.float32).reshape(16)),
                        _p(np.ascontiguousarray(c, np.float32).reshape(3)), W, H, int(mode), int(color_i32), _p(sdf),
                        _p(hist), _p(color), _p(out), _p(t), 0, H)
    return out.reshape(H, W, 3), t.reshape(H, W)


def shard_render_step(g: OGeom, s2w, c, W, H, mode, sdf, hist, color, step, shard, nshards, chunk, gathered,
                      send, state, out=None, out_t=None, color_i32=False):
    """One step of the Z-sharded render protocol for virtual shard `shard` (see
    oracle_shard_render_step).  gathered/send: int32 [.., H*W*2]; state int32 [6*H*W]."""
    lib().oracle_shard_render_step(_p(g.dims), _p(g.geo), _p(np.ascontiguousarray(s2w, np.float32).reshape(16)),
                                   _p(np.ascontiguousarray(c, np.float32).reshape(3)), W, H, int(mode),
                                   int(color_i32), _p(sdf), _p(hist), _p(color), int(step), int(shard),
                                   int(nshards), int(chunk), _p(gathered), _p(send), _p(state), _p(out), _p(out_t))


def div_rcp_mismatches(a, b: float) -> int:
    a = np.ascontiguousarray(a, np.float32)
    return int(lib().oracle_div_rcp_mismatches(_p(a), a.size, float(b)))


def place(depth, Kinv16, dims, mean_depth, mode):
    out = np.zeros(10, np.float32)
    H, W = depth.shape
    rc = lib().oracle_place(_p(np.ascontiguousarray(depth, np.uint16)), W, H,
                            _p(np.ascontiguousarray(Kinv16, np.float32).reshape(16)),
                            _p(np.ascontiguousarray(dims, np.int32)), float(mean_depth), int(mode), _p(out))
    if rc != 0:
        raise ValueError("no valid depth")
    return dict(vol_start=out[0:3].copy(), vol_end=out[3:6].copy(), voxel=out[6:9].copy(), mu=float(out[9]))


def orbit_camera(Kinv16, angle, dist):
    s2w = np.zeros(16, np.float32)
    c = np.zeros(3, np.float32)
    lib().oracle_orbit_camera(_p(np.ascontiguousarray(Kinv16, np.float32).reshape(16)), angle, dist, _p(s2w), _p(c))
    return s2w, c


# ------------------------------------------------------------------------------------
# NumPy restatement of src/TSDF_Python/tsdf.py:78-120 (+ SfM gate/histogram)
# ------------------------------------------------------------------------------------
def numpy_integrate(sdf, wt, color, vol_dim, vol_start, voxel, mu, K, E, depth, rgb, x_range=None,
                    semantic=False, gate=0.99, mask=None, hist=None, n_flat=None):
    """In-place update of flat x-major state arrays (sdf f32 [N], wt i32 [N], color i32/u8
    [N, 3], hist u32 [N, 32]) over x-planes `x_range` (default all).  float64 arithmetic as
    the reference block: projection with the f64 pose and the f32 intrinsic, pixel by
    truncation toward zero (astype int), depth/5000 - z, clamp to +-mu, reject f <= -1,
    running means (colour truncated on store).  With semantic=True the colour and the
    histogram are updated only where f < gate (tsdf.cu:57-62).  Returns (touched, gated).
    `n_flat` limits the visited flat indices (the reference's tex_dim^2 truncation)."""
    D = int(vol_dim)
    H, W = depth.shape[:2]
    x0, x1 = (0, D) if x_range is None else x_range
    lo, hi = x0 * D * D, x1 * D * D
    if n_flat is not None:
        hi = min(hi, n_flat)
    if hi <= lo:
        return 0, 0
    flat = np.arange(lo, hi, dtype=np.int64)
    xi = flat // (D * D)
    yi = flat // D - xi * D
    zi = flat % D
    vs = np.asarray(vol_start, np.float64)
    vx = np.asarray(voxel, np.float64) * np.ones(3)
    pos = np.stack([vs[0] + xi * vx[0], vs[1] + yi * vx[1], vs[2] + zi * vx[2], np.ones(flat.size)], axis=0)
    proj = np.dot(np.asarray(E, np.float64), pos)
    pixel = np.dot(np.asarray(K, np.float32), proj)
    pixel /= pixel[2, :]
    px = pixel[0].astype(np.int64)
    py = pixel[1].astype(np.int64)
    ok = (px >= 0) & (px <= W - 1) & (py >= 0) & (py <= H - 1)
    iy = np.minimum(np.maximum(py, 0), H - 1)
    ix = np.minimum(np.maximum(px, 0), W - 1)
    d = depth[iy, ix]
    diff = d / 5000 - proj[2, :]
    ok &= d > 0
    diff = np.maximum(np.minimum(diff, mu), -mu) / mu
    ok &= diff > -1
    sl = slice(lo, hi)
    s_sdf, s_wt, s_col = sdf[sl], wt[sl], color.reshape(-1, 3)[sl]
    wm = s_wt > 0
    c_img = rgb[iy, ix].astype(np.float64)
    a = ok & wm
    b = ok & ~wm
    s_sdf[a] = (s_sdf[a] * s_wt[a] + diff[a]) / (s_wt[a] + 1)
    s_sdf[b] = diff[b]
    cg_a, cg_b = a, b
    gated = ok
    if semantic:
        gated = ok & (diff < gate)
        cg_a, cg_b = a & gated, b & gated
    s_col[cg_a] = (s_col[cg_a] * s_wt[cg_a][:, None] + c_img[cg_a]) / (s_wt[cg_a] + 1)[:, None]
    s_col[cg_b] = c_img[cg_b]
    if semantic and hist is not None and mask is not None:
        lab = mask[iy, ix].astype(np.int64)
        h = hist.reshape(-1, OMAX)[sl]
        sel = np.nonzero(gated)[0]
        np.add.at(h, (sel, lab[sel]), 1)
    s_wt[ok] += 1
    return int(ok.sum()), int(gated.sum())


# ------------------------------------------------------------------------------------
# NumPy restatement of Mask_RCNN/dmask.py:21-59 (mask_detect, depth_image=None as
# mask_process.py:100 calls it)
# ------------------------------------------------------------------------------------
def masks_to_labels(masks, min_area=2000):
    """masks bool [H, W, N] -> (labels u8 [H, W], kept).  filter_tiny_objects (:34-45) keeps
    detections with area > min_area; preserve_small_objs (:21-32) leaves each pixel to the
    first detection in ascending-area order that covers it (the sequential removal reduces
    to that); :56-58 writes 1 + index among the kept.  Equal areas: the stable order (lower
    index first) -- dmask.py's np.argsort (quicksort) leaves that order unspecified."""
    m = np.asarray(masks).astype(bool)
    H, W, n = m.shape
    areas = m.sum(axis=(0, 1))
    kept = np.nonzero(areas > min_area)[0]
    out = np.zeros((H, W), np.uint8)
    if kept.size == 0:
        return out, 0
    order = np.argsort(areas[kept], kind="stable")
    mk = m[:, :, kept[order]]
    any_ = mk.any(axis=2)
    first = mk.argmax(axis=2)
    out[any_] = (order[first[any_]] + 1).astype(np.uint8)
    return out, int(kept.size)


def non_max_suppression(boxes, scores, threshold):
    """Greedy NMS, Mask_RCNN/mrcnn/utils.py:116-150 (with compute_iou utils.py:58-76), in f32: indices of
    the kept boxes, highest score first (a restatement for the tests; the product runs the HIP kernels
    of libsemtsdf_det.so)."""
    boxes = np.asarray(boxes, dtype=np.float32)
    scores = np.asarray(scores)
    y1, x1, y2, x2 = boxes[:, 0], boxes[:, 1], boxes[:, 2], boxes[:, 3]
    area = (y2 - y1) * (x2 - x1)
    ixs = scores.argsort(kind="stable")[::-1]
    pick = []
    while len(ixs) > 0:
        i = ixs[0]
        pick.append(i)
        rest = ixs[1:]
        yy1 = np.maximum(y1[i], y1[rest])
        yy2 = np.minimum(y2[i], y2[rest])
        xx1 = np.maximum(x1[i], x1[rest])
        xx2 = np.minimum(x2[i], x2[rest])
        inter = np.maximum(xx2 - xx1, np.float32(0)) * np.maximum(yy2 - yy1, np.float32(0))
        with np.errstate(invalid="ignore", divide="ignore"):
            iou = inter / (area[i] + area[rest] - inter)
        ixs = np.delete(ixs, np.where(iou > threshold)[0] + 1)
        ixs = np.delete(ixs, 0)
    return np.array(pick, dtype=np.int32)


def nms_sorted_cpu(boxes, iou_threshold, max_out):
    """The product's nms_sorted contract (boxes sorted by descending score; keep [max_out] with -1
    past the count, count [1]) on CPU torch tensors, from non_max_suppression above: for CPU tests of
    the detector graph."""
    import torch

    b = boxes.detach().float().cpu().numpy()
    n = b.shape[0]
    pick = non_max_suppression(b, -np.arange(n, dtype=np.float64), iou_threshold)[:max_out] if n else np.zeros(0, np.int32)
    keep = np.full(max(max_out, 1), -1, np.int32)
    keep[:len(pick)] = pick
    return torch.from_numpy(keep[:max_out]), torch.tensor([len(pick)], dtype=torch.int32)
