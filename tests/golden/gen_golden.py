"""Generate golden vectors by executing the reference's own Python code (run here only).

This script needs /root/reference (absent on the GPU box); its OUTPUT (tests/golden/*.npz)
is committed and is what the tests read.  Nothing of the reference's text is stored.

What runs from the reference:
  * src/TSDF_Python/tsdf.py  `TSDF.init_vars` (volume placement, tsdf.py:32-52), called on
    an instance whose constructor state is set by hand because tsdf.py:13 builds a singular
    K on NumPy >= 1.23 (list index); the K used is the intended one (tuple index);
  * the commented vectorised integrate, tsdf.py:78-120, extracted from the file at run time,
    comment markers stripped, with two NumPy-2 shims: `np.int = int` (tsdf.py:92-93) and
    `idx = tuple(idx)` after tsdf.py:99-100 (a list of index arrays is no longer a tuple);
  * src/TSDF_Python/tsdf_utils.py `transform44`, `slerp` (pure NumPy) and `parse_pos`
    (with the in-memory cv2 stub below providing Rodrigues).
Frames: the real 640x480 TUM fr2 depth/RGB files that ship in the reference
(Mask_RCNN/1311871922.983782.png + 1311871923.004312.png, and
Mask_RCNN/samples/1311871965.993806.png + 1311871965.975433.png), with synthetic poses.
The first frame is integrated with E = extrinsic * inv(extrinsic) (tsdf.py:55-57 recursion).
"""
from __future__ import annotations

import math
import os
import sys
import textwrap
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _stub_modules():
    cv2 = types.ModuleType("cv2")

    def findNonZero(a):
        ys, xs = np.nonzero(a)
        return np.stack([xs, ys], axis=1).reshape(-1, 1, 2).astype(np.int32)

    def boundingRect(pts):
        p = np.asarray(pts).reshape(-1, 2)
        x0, y0 = p.min(axis=0)
        x1, y1 = p.max(axis=0)
        return int(x0), int(y0), int(x1 - x0 + 1), int(y1 - y0 + 1)

    def Rodrigues(rvec, out=None):
        r = np.asarray(rvec, np.float64).reshape(3)
        th = float(np.linalg.norm(r))
        if th < 1e-300:
            R = np.eye(3)
        else:
            k = r / th
            K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
            R = math.cos(th) * np.eye(3) + (1 - math.cos(th)) * np.outer(k, k) + math.sin(th) * K
        if out is not None:
            out[...] = R
        return R, None

    cv2.findNonZero = findNonZero
    cv2.boundingRect = boundingRect
    cv2.Rodrigues = Rodrigues
    cv2.imshow = lambda *a, **k: None
    cv2.waitKey = lambda *a, **k: 0
    sys.modules["cv2"] = cv2
    for name in ("sdl2", "OpenGL", "OpenGL.GL", "OpenGL.GL.shaders"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["OpenGL"].GL = sys.modules["OpenGL.GL"]
    sys.modules["OpenGL.GL"].shaders = sys.modules["OpenGL.GL.shaders"]
    viewer = types.ModuleType("TSDF_Python.viewer")
    viewer.Viewer = object
    sys.modules["TSDF_Python.viewer"] = viewer


def _integrate_block() -> str:
    with open(os.path.join(REF, "src/TSDF_Python/tsdf.py")) as f:
        lines = f.read().split("\n")
    blk = lines[77:120]  # tsdf.py:78-120
    out = []
    for ln in blk:
        s = ln.lstrip()
        ind = ln[: len(ln) - len(s)]
        if s.startswith("# "):
            s = s[2:]
        elif s.startswith("#"):
            s = s[1:]
        out.append(ind + s)
    code = textwrap.dedent("\n".join(out))
    # shim 2: a list of index arrays is no longer a tuple index on NumPy >= 1.23
    fixed = []
    for ln in code.split("\n"):
        fixed.append(ln)
        if "color.shape[1] - 1)]" in ln:
            fixed.append("idx = tuple(idx)")
    return "\n".join(fixed)


def _png(path):
    from PIL import Image

    return np.array(Image.open(os.path.join(REF, path)))


def make_tsdf(TSDF, intrinsics, vol_dim):
    t = TSDF.__new__(TSDF)
    t.intrinsic = np.eye(4, dtype=np.float32)
    t.intrinsic[(0, 1, 0, 1), (0, 1, 2, 2)] = np.array(intrinsics)
    t.init = False
    t.tsdf_diff = t.tsdf_wt = t.tsdf_color = t.tsdf_cls = t.tsdf_cls_cnt = None
    t.mu = 0
    t.vol_dim = vol_dim
    t.tex_dim = int(np.sqrt(pow(t.vol_dim, 3)))
    t.voxel = [0] * 3
    t.vol_start = t.vol_end = None
    t.intrinsic_inv = np.linalg.inv(t.intrinsic)
    t.init_extrinsic_inv = None
    t.mean_depth = 0
    t.num_cls = 0
    t.N = 0
    return t


def run_case(TSDF, block, frames, vol_dim, intrinsics=(520.9, 521.0, 325.1, 249.7)):
    t = make_tsdf(TSDF, intrinsics, vol_dim)
    np.int = int  # shim 1 (tsdf.py:92-93)
    outs = []
    for k, (depth, color, extrinsic) in enumerate(frames):
        mean_depth = np.mean(depth[depth > 0])
        if not t.init:
            t.init_vars(depth, color, extrinsic, mean_depth)  # reference code, tsdf.py:32-52
            place = dict(vol_start=np.array(t.vol_start), vol_end=np.array(t.vol_end), voxel=np.array(t.voxel),
                         mu=np.float64(t.mu), mean_depth=np.float64(mean_depth), intrinsic_inv=t.intrinsic_inv,
                         sdf_dtype=str(t.tsdf_diff.dtype))
        ns = {"self": t, "depth": depth, "color": color, "extrinsic": extrinsic, "np": np}
        exec(block, ns)  # reference code, tsdf.py:78-120
        outs.append(dict(sdf=t.tsdf_diff.reshape(-1).copy(), wt=t.tsdf_wt.reshape(-1).copy(),
                         color=t.tsdf_color.reshape(-1, 3).copy(),
                         E=np.matmul(extrinsic, t.init_extrinsic_inv)))
    return place, outs


def main():
    sys.path.insert(0, os.path.join(REF, "src"))
    _stub_modules()
    from TSDF_Python import tsdf_utils
    from TSDF_Python.tsdf import TSDF

    block = _integrate_block()
    dA = _png("Mask_RCNN/1311871922.983782.png").astype(np.uint16)
    cA = _png("Mask_RCNN/1311871923.004312.png")[:, :, :3].copy()
    dB = _png("Mask_RCNN/samples/1311871965.993806.png").astype(np.uint16)
    cB = _png("Mask_RCNN/samples/1311871965.975433.png")[:, :, :3].copy()

    # synthetic TUM poses (tx ty tz qx qy qz qw), camera-to-world
    poses = [
        [0.10, -0.05, 0.02, 0.01, 0.02, 0.005, 1.0],
        [0.12, -0.04, 0.03, 0.012, 0.025, 0.004, 1.0],
        [0.09, -0.06, 0.00, 0.008, 0.015, 0.010, 1.0],
    ]
    poses = [np.array(p[:3] + list(np.array(p[3:]) / np.linalg.norm(p[3:]))) for p in poses]
    extr = [tsdf_utils.parse_pos(p) for p in poses]
    degenerate = np.array([0.1, -0.2, 0.3, 0.0, 0.0, 1e-5, 0.0])  # |q|^2 < 1e-7: tsdf_utils.py:46-52
    pose_fix = dict(
        poses=np.array(poses),
        parse_pos=np.array(extr),
        transform44=np.array([tsdf_utils.transform44(p) for p in poses]),
        degenerate_pose=degenerate,
        transform44_degenerate=tsdf_utils.transform44(degenerate),
        slerp=np.array([tsdf_utils.slerp(poses[0][3:], poses[1][3:], t) for t in (0.0, 0.25, 0.5, 1.0)] +
                       [tsdf_utils.slerp(poses[0][3:], -poses[2][3:], 0.3)]),
    )
    np.savez_compressed(os.path.join(OUT, "pose_golden.npz"), **pose_fix)

    cases = {
        "d64": (64, [(dA, cA, extr[0]), (dA, cA, extr[1]), (dB, cB, extr[2])]),
        "d128": (128, [(dA, cA, extr[0])]),
    }
    for name, (D, frames) in cases.items():
        place, outs = run_case(TSDF, block, frames, D)
        rec = {f"place_{k}": v for k, v in place.items()}
        rec["vol_dim"] = np.int64(D)
        rec["n_frames"] = np.int64(len(frames))
        for k, o in enumerate(outs):
            touched = np.nonzero(o["wt"])[0].astype(np.int64)
            rec[f"f{k}_idx"] = touched
            rec[f"f{k}_sdf"] = o["sdf"][touched]
            rec[f"f{k}_wt"] = o["wt"][touched]
            rec[f"f{k}_color"] = o["color"][touched]
            rec[f"f{k}_E"] = o["E"]
            rec[f"f{k}_nflat"] = np.int64(o["wt"].size)
            rec[f"f{k}_extrinsic"] = frames[k][2]
        np.savez_compressed(os.path.join(OUT, f"integrate_{name}.npz"), **rec)
        print(name, D, [int(np.count_nonzero(o["wt"])) for o in outs], place["sdf_dtype"])
    # the frames themselves (data files of the reference, stored as arrays)
    np.savez_compressed(os.path.join(OUT, "frames_tum_fr2.npz"), depth_a=dA, rgb_a=cA, depth_b=dB, rgb_b=cB)

    # placement (tsdf.py:32-52, init_vars) on both real frames at several volume sizes
    place = {}
    for fname, (d, c) in (("a", (dA, cA)), ("b", (dB, cB))):
        for D in (64, 128, 256):
            t = make_tsdf(TSDF, (520.9, 521.0, 325.1, 249.7), D)
            mean_depth = np.mean(d[d > 0])
            t.init_vars(d, c, np.eye(4), mean_depth)
            for k, val in (("vol_start", t.vol_start), ("vol_end", t.vol_end), ("voxel", t.voxel), ("mu", t.mu),
                           ("mean_depth", mean_depth), ("intrinsic_inv", t.intrinsic_inv)):
                place[f"{fname}{D}_{k}"] = np.asarray(val)
    np.savez_compressed(os.path.join(OUT, "placement_golden.npz"), **place)
    print("placement", sorted({k.split('_')[0] for k in place}))

    c1_case(TSDF, tsdf_utils, block)


def c1_case(TSDF, tsdf_utils, block, n_frames=20, D=128):
    """C1 (BASELINE.json configs[0]): the NumPy integrate at 128^3 over 20 frames, no masks.
    fr2_desk is not in the container, so the frames are the seeded synthetic stream (seed 0,
    regenerated by the tests) and its poses go through the reference's own pose path:
    groundtruth lines -> tsdf_utils.read_traj -> parse_pos.  Frame 0 places the volume and is
    integrated with E = extrinsic * inv(extrinsic) (tsdf.py:55-57); the final state is stored."""
    import tempfile

    sys.path.insert(0, os.path.join(os.path.dirname(OUT), "..", "slam-maskrcnn_amd"))
    from semtsdf.synth import SyntheticStream

    from semtsdf import pose as P

    st = SyntheticStream(seed=0)
    # the stream's frame 0 is the identity pose, whose zero rotation axis parse_pos divides by
    # (tsdf_utils.py:67-68 -> NaN); a fixed world offset B keeps every relative pose
    # E = inv(B c2w_k) B c2w_0 = inv(c2w_k) c2w_0 and avoids it
    B = np.eye(4)
    B[:3, :3] = P.rodrigues([0.02, -0.03, 0.01])
    B[:3, 3] = (0.3, -0.1, 0.2)
    lines = [P.c2w_to_tum(st.stamp(k), B @ st.c2w(k)) for k in range(n_frames)]
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        f.write("# timestamp tx ty tz qx qy qz qw\n" + "\n".join(lines) + "\n")
        gt = f.name
    traj = tsdf_utils.read_traj(gt)  # reference code
    os.unlink(gt)
    t = make_tsdf(TSDF, (520.9, 521.0, 325.1, 249.7), D)
    np.int = int
    Es, sums = [], []
    for k in range(n_frames):
        fr = st.frame(k)
        extrinsic = tsdf_utils.parse_pos(traj[k, 1:])  # reference code (cv2.Rodrigues stubbed)
        if not t.init:
            t.init_vars(fr.depth, fr.rgb, extrinsic, np.mean(fr.depth[fr.depth > 0]))
        exec(block, {"self": t, "depth": fr.depth, "color": fr.rgb, "extrinsic": extrinsic, "np": np})
        Es.append(np.matmul(extrinsic, t.init_extrinsic_inv))
        sums.append(int(fr.depth.astype(np.int64).sum()) ^ (int(fr.rgb.astype(np.int64).sum()) << 1))
    wt = t.tsdf_wt.reshape(-1)
    idx = np.nonzero(wt)[0]
    col = t.tsdf_color.reshape(-1, 3)[idx]
    assert wt.max() <= 255 and col.min() >= 0 and col.max() <= 255
    np.savez_compressed(
        os.path.join(OUT, "integrate_c1_d128.npz"), vol_dim=np.int64(D), n_frames=np.int64(n_frames),
        n_flat=np.int64(wt.size), place_vol_start=np.array(t.vol_start), place_voxel=np.array(t.voxel),
        place_mu=np.float64(t.mu), place_intrinsic_inv=t.intrinsic_inv, E=np.array(Es), frame_sums=np.array(sums),
        world_offset=B, idx=idx.astype(np.uint32), sdf=t.tsdf_diff.reshape(-1)[idx].astype(np.float32), wt=wt[idx].astype(np.uint8),
        color=col.astype(np.uint8), sdf_dtype=np.str_(str(t.tsdf_diff.dtype)))
    print("c1", D, n_frames, "touched", idx.size)


if __name__ == "__main__":
    main()
