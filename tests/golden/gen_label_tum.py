"""Golden vectors for the label histogram and the Python driver's frame association, made by
executing the reference's own Python text (run here only; /root/reference is absent on the
GPU box).  The OUTPUT (tests/golden/hist_golden.npz, tum_assoc_golden.npz) is committed and
is what the tests read; nothing of the reference's text is stored.

* Instance histogram (the label path): src/TSDF_Python/tsdf.py:122-130 is the
  commented first-frame class count.  It runs here right after the commented integrate
  (tsdf.py:78-120, exactly as gen_golden.py executes it), in the same namespace, so it sees
  that block's `idx` (the clamped pixel of every voxel) and `mask` (the touched voxels).  The
  masks are a synthetic non-overlapping multi-channel [H, W, C] array on the real TUM frame
  (channel k <-> instance label k + 1).  Shims: `np.int = int` and the tuple index, as in
  gen_golden.py.  The reference's `masks[..][idx] > 0 & mask` parses as `> (0 & mask)`, so its
  count ignores the touch mask; the comparable set is the touched voxels (stored), where the
  count is 1 exactly when the voxel's pixel carries channel k.
* Frame association + pose interpolation (§8 a3, f2): src/TSDF_Python/main.py:63-64 (stamps
  from the file names), :69-70, :75-76 (window), :83-91 (the association loop) and :127-140
  (lerp + slerp of the bracketing ground-truth rows, then parse_pos), executed with a hook
  that records (i, j) and the pose in place of the image reads; the file lists are synthetic
  Windows-style paths (the reference splits on '\\'), the trajectory a synthetic
  groundtruth.txt read by the reference's read_traj.
"""
from __future__ import annotations

import os
import sys
import tempfile
import textwrap

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "..", "slam-maskrcnn_amd"))
import gen_golden as G  # noqa: E402

REF = G.REF


def _uncomment(lines):
    out = []
    for ln in lines:
        s = ln.lstrip()
        ind = ln[: len(ln) - len(s)]
        if s.startswith("# "):
            s = s[2:]
        elif s.startswith("#"):
            s = s[1:]
        out.append(ind + s)
    return textwrap.dedent("\n".join(out))


def _hist_block() -> str:
    with open(os.path.join(REF, "src/TSDF_Python/tsdf.py")) as f:
        lines = f.read().split("\n")
    return _uncomment(lines[121:130])  # tsdf.py:122-130


def label_image(H, W, n_cls, seed):
    """Non-overlapping instance labels 0..n_cls (ellipses, first drawn wins)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    lab = np.zeros((H, W), np.uint8)
    for k in range(n_cls):
        cy, cx = rng.uniform(0.1 * H, 0.9 * H), rng.uniform(0.1 * W, 0.9 * W)
        ry, rx = rng.uniform(0.08 * H, 0.3 * H), rng.uniform(0.08 * W, 0.3 * W)
        inside = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0
        lab[inside & (lab == 0)] = k + 1
    return lab


def hist_cases(TSDF, tsdf_utils, block):
    hb = _hist_block()
    dA = G._png("Mask_RCNN/1311871922.983782.png").astype(np.uint16)
    cA = G._png("Mask_RCNN/1311871923.004312.png")[:, :, :3].copy()
    pose = np.array([0.10, -0.05, 0.02, 0.01, 0.02, 0.005, 1.0])
    pose[3:] /= np.linalg.norm(pose[3:])
    extrinsic = tsdf_utils.parse_pos(pose)
    rec = {}
    n_cls = 6
    lab = label_image(480, 640, n_cls, seed=21)
    masks = np.stack([(lab == k + 1).astype(np.uint8) for k in range(n_cls)], axis=2)
    rec["labels"] = lab
    rec["n_cls"] = np.int64(n_cls)
    np.int = int
    for D in (64, 128):
        t = G.make_tsdf(TSDF, (520.9, 521.0, 325.1, 249.7), D)
        mean_depth = np.mean(dA[dA > 0])
        t.init_vars(dA, cA, extrinsic, mean_depth)  # reference code, tsdf.py:32-52
        ns = {"self": t, "depth": dA, "color": cA, "extrinsic": extrinsic, "masks": masks, "np": np}
        exec(block, ns)   # reference code, tsdf.py:78-120
        exec(hb, ns)      # reference code, tsdf.py:122-130 (N == 0: first-frame class count)
        wt = t.tsdf_wt.reshape(-1)
        cnt = t.tsdf_cls_cnt.reshape(-1, n_cls)
        touched = np.nonzero(wt)[0]
        untouched_counted = int((cnt[wt == 0] > 0).any(axis=1).sum())
        rec[f"d{D}_vol_start"] = np.array(t.vol_start)
        rec[f"d{D}_voxel"] = np.array(t.voxel)
        rec[f"d{D}_mu"] = np.float64(t.mu)
        rec[f"d{D}_nflat"] = np.int64(wt.size)
        rec[f"d{D}_E"] = np.matmul(extrinsic, t.init_extrinsic_inv)
        rec[f"d{D}_idx"] = touched.astype(np.int64)
        rec[f"d{D}_cls_cnt"] = cnt[touched].astype(np.uint8)
        rec[f"d{D}_untouched_counted"] = np.int64(untouched_counted)
        print(f"hist d{D}: touched {touched.size}, counted {int((cnt[touched] > 0).sum())}, "
              f"untouched voxels with a count (the precedence quirk) {untouched_counted}")
    np.savez_compressed(os.path.join(HERE, "hist_golden.npz"), **rec)


def _main_lines():
    with open(os.path.join(REF, "src/TSDF_Python/main.py")) as f:
        return f.read().split("\n")


def tum_case(tsdf_utils, name, depth_st, rgb_st, gt_lines):
    """Execute main.py's stamp parsing, association loop and pose interpolation on synthetic
    file lists; returns the recorded (i, j) pairs and poses."""
    L = _main_lines()
    body_assoc = "\n".join(L[82:91])      # main.py:83-91 (for-loop header + association)
    body_pose = "\n".join(L[126:140])     # main.py:127-140 (pose interpolation + parse_pos)
    hook1 = "        rec_pairs.append((i, j))"
    hook2 = "        rec_poses.append(extrinsic)"
    code = "\n".join([L[62], L[63], L[68], L[69], L[74], L[75], body_assoc, hook1, body_pose, hook2])
    code = textwrap.dedent(code)
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        f.write("\n".join(gt_lines) + "\n")
        gt = f.name
    try:
        ns = {
            "np": np, "tsdf_utils": tsdf_utils,
            "depth_fn": [f"D:\\rgb-datasets\\desk\\depth\\{s}.png" for s in depth_st],
            "rgb_fn": [f"D:\\rgb-datasets\\desk\\rgb\\{s}.png" for s in rgb_st],
            "TRAJ_PATH": gt, "rec_pairs": [], "rec_poses": [],
        }
        exec(code, ns)  # reference code, main.py:63-64,69-70,75-76,83-91,127-140
    finally:
        os.unlink(gt)
    print(f"tum {name}: {len(ns['rec_pairs'])} frames, pairs {ns['rec_pairs'][:6]}...")
    return np.array(ns["rec_pairs"], np.int64).reshape(-1, 2), np.array(ns["rec_poses"], np.float64).reshape(-1, 4, 4)


def tum_cases(tsdf_utils):
    from semtsdf import pose as P
    from semtsdf.synth import SyntheticStream

    st = SyntheticStream(seed=0, yaw_step=0.02)
    rng = np.random.default_rng(4)
    rec = {}
    # ground truth at 100 Hz with jitter from 68163.8 s on; depth and rgb at ~30 Hz, offset
    t_gt = 1311868163.8 + np.cumsum(rng.uniform(0.008, 0.012, 160))
    gt_lines = ["# ground truth trajectory", "# timestamp tx ty tz qx qy qz qw"]
    gt_lines += [P.c2w_to_tum(float(t), st.c2w(k)) for k, t in enumerate(t_gt)]
    cases = {}
    t_d = 1311868163.95 + np.cumsum(rng.uniform(0.028, 0.038, 36))
    t_r = t_d + rng.uniform(-0.012, 0.012, t_d.size)  # rgb close to depth, either side
    cases["jitter"] = ([f"{t:.6f}" for t in t_d], [f"{t:.6f}" for t in np.sort(t_r)])
    # rgb at half the rate: the Python loop's rebinding of i fuses a depth frame repeatedly
    t_d2 = 1311868163.95 + 0.033 * np.arange(1, 30)
    t_r2 = 1311868163.96 + 0.066 * np.arange(1, 16)
    cases["half_rate_rgb"] = ([f"{t:.6f}" for t in t_d2], [f"{t:.6f}" for t in t_r2])
    for name, (ds, rs) in cases.items():
        pairs, poses = tum_case(tsdf_utils, name, ds, rs, gt_lines)
        rec[f"{name}_depth"] = np.array(ds)
        rec[f"{name}_rgb"] = np.array(rs)
        rec[f"{name}_pairs"] = pairs
        rec[f"{name}_extrinsic"] = poses
    rec["gt_lines"] = np.array(gt_lines)
    np.savez_compressed(os.path.join(HERE, "tum_assoc_golden.npz"), **rec)


def main():
    sys.path.insert(0, os.path.join(REF, "src"))
    G._stub_modules()
    from TSDF_Python import tsdf_utils
    from TSDF_Python.tsdf import TSDF

    hist_cases(TSDF, tsdf_utils, G._integrate_block())
    tum_cases(tsdf_utils)


if __name__ == "__main__":
    main()
