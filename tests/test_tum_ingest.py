"""TUM RGB-D ingest of the host (§8f rank 2): trajectory
readers, both frame-association drivers, pose lookup/interpolation and mean depth, on a
temporary TUM directory written by the test.  The expected pairings are worked out from
the reference loops (src/SfM_CUDA/kernel.cpp:51-99, src/TSDF_Python/main.py:59-140)."""
import math
import os

import numpy as np
import pytest
from PIL import Image

from semtsdf import pose as P
from semtsdf import tum
from semtsdf.synth import SyntheticStream


def _write_dir(root, depth_stamps, pair_stamps, gt_lines, shape=(6, 8)):
    for sub in ("depth", "rgb", "mask"):
        os.makedirs(os.path.join(root, sub), exist_ok=True)
    rng = np.random.default_rng(7)
    for st in depth_stamps:
        d = rng.integers(0, 9000, shape).astype(np.uint16)
        Image.fromarray(d).save(os.path.join(root, "depth", f"{st}.png"))
    for st in pair_stamps:
        Image.fromarray(rng.integers(0, 256, shape + (3,)).astype(np.uint8)).save(os.path.join(root, "rgb", f"{st}.png"))
        Image.fromarray(rng.integers(0, 5, shape).astype(np.uint8)).save(os.path.join(root, "mask", f"{st}.png"))
    with open(os.path.join(root, "groundtruth.txt"), "w") as f:
        f.write("\n".join(gt_lines) + "\n")


def _gt(n=40, t0=1311868164.0, dt=0.01):
    st = SyntheticStream(seed=0, yaw_step=0.02)
    lines = ["# ground truth trajectory", "# timestamp tx ty tz qx qy qz qw"]
    for k in range(n):
        lines.append(P.c2w_to_tum(t0 + dt * k, st.c2w(k)))
    return lines


def test_read_traj_and_read_trajactory(tmp_path):
    lines = _gt(5) + ["1311868164.0100 9 9 9 0 0 0 1"]  # duplicate key: std::map::insert keeps the first
    p = tmp_path / "gt.txt"
    p.write_text("\n".join(lines) + "\n")
    traj = tum.read_traj(str(p))  # tsdf_utils.py:23-29: name[5:] as float64
    assert traj.shape == (6, 8)
    assert np.allclose(traj[:5, 0], 68164.0 + 0.01 * np.arange(5), atol=1e-9)
    m = tum.read_trajactory(str(p))  # utils.cu:62-75: key fmod(ts, 1e5), first insert wins
    keys = list(m)
    assert len(keys) == 5 and keys == sorted(keys)
    assert abs(keys[1] - math.fmod(1311868164.01, 1e5)) < 1e-9
    assert m[keys[1]][0] != 9.0 and list(m.values())[1] == [float(x) for x in lines[3].split()[1:8]]


def test_lower_bound_pose():
    m = {1.0: [1], 2.0: [2], 3.0: [3]}
    assert tum.lower_bound_pose(m, 2.0) == [2]  # equal key
    assert tum.lower_bound_pose(m, 2.5) == [3]  # first key after
    assert tum.lower_bound_pose(m, 0.1) == [1]
    with pytest.raises(KeyError):
        tum.lower_bound_pose(m, 3.5)  # end(): the reference dereferences it


def test_stamp_rounding_of_the_sfm_driver():
    # kernel.cpp:52,56: stod of name[5:] returned as float -> 2^-7 s spacing at 68164 s
    f = "/x/depth/1311868164.3640.png"
    assert tum.stamp_of(f, True) == float(np.float32(68164.364)) == 68164.3671875
    assert tum.stamp_of(f, False) == 68164.364


def test_associate_float32_quirk_pairs_differently(tmp_path):
    """Depth .3640 and mask/rgb .3635: the float32 stamps of the SfM driver are equal, so it
    pairs them; in float64 the mask is earlier and the Python driver moves to the next one."""
    depth = ["1311868164.3640", "1311868164.4100"]
    pair = ["1311868164.3635", "1311868164.4000"]
    _write_dir(str(tmp_path), depth, pair, _gt())
    sfm = tum.associate(str(tmp_path), "sfm", begin=68164.0, end=68170.0)
    assert [(f.i, f.j) for f in sfm] == [(0, 0)]
    assert sfm[0].mask_fn.endswith(pair[0] + ".png") and sfm[0].rgb_fn.endswith(pair[0] + ".png")
    assert sfm[0].ts == 68164.3671875
    py = tum.associate(str(tmp_path), "python", begin=68164.0, end=68170.0)
    assert [(f.i, f.j) for f in py] == [(0, 1)]


def test_associate_python_driver_repeats_frames(tmp_path):
    """main.py:83 `for i in range(3000)` rebinds i, so the inner loop's advance is lost and the
    same depth frame is fused once per earlier index; kernel.cpp's size_t i keeps it."""
    depth = ["1311868164.1000", "1311868164.2000", "1311868164.3000"]
    pair = ["1311868164.3000", "1311868164.4000"]
    _write_dir(str(tmp_path), depth, pair, _gt(n=80, dt=0.007))
    py = tum.associate(str(tmp_path), "python")  # window [68164, 68164.37] (main.py:75-76)
    assert [(f.i, f.j) for f in py] == [(2, 0), (2, 0), (2, 0)]
    sfm = tum.associate(str(tmp_path), "sfm")
    assert [(f.i, f.j) for f in sfm] == [(2, 0)]
    # SfM pose: lower_bound on fmod(ts, 1e5) -- the first ground-truth row at or after ts
    traj = tum.read_traj(os.path.join(str(tmp_path), "groundtruth.txt"))
    k = int(np.nonzero(traj[:, 0] >= sfm[0].ts)[0][0])
    assert np.array_equal(sfm[0].pose, traj[k, 1:])
    # Python pose: lerp + slerp between the bracketing rows (main.py:127-140)
    ts = py[0].ts
    k = int(np.nonzero(traj[:, 0] >= ts)[0][0])
    t = (ts - traj[k - 1, 0]) / (traj[k, 0] - traj[k - 1, 0])
    exp = np.concatenate([(traj[k, 1:4] - traj[k - 1, 1:4]) * t + traj[k - 1, 1:4],
                          P.slerp(traj[k - 1, -4:], traj[k, -4:], t)])
    assert 0 < t < 1 and np.array_equal(py[0].pose, exp)


def test_associate_sfm_window_and_cap(tmp_path):
    depth = [f"{1311868163.9 + 0.05 * k:.4f}" for k in range(130)]  # 68163.90 .. 68170.35
    _write_dir(str(tmp_path), depth, depth, _gt(800))
    sfm = tum.associate(str(tmp_path), "sfm")
    assert len(sfm) == 100  # kernel.cpp:73-74: cnt > 100 breaks
    assert all(68164.0 <= f.ts <= 68170.0 for f in sfm)
    assert [f.i for f in sfm] == list(range(sfm[0].i, sfm[0].i + 100)) and all(f.i == f.j for f in sfm)


def test_interpolate_pose_edges():
    traj = np.array([[1.0, 0, 0, 0, 0, 0, 0, 1], [2.0, 1, 2, 3, 0, 0, 0.3826834, 0.9238795]])
    p = P.interpolate_pose(traj, 1.5)
    assert np.allclose(p[:3], [0.5, 1.0, 1.5])
    assert np.allclose(p[3:], P.slerp(traj[0, 4:], traj[1, 4:], 0.5))
    p1 = P.interpolate_pose(traj, 1.0)  # first row: pairs with row -1 (t == 1)
    assert np.allclose(p1, traj[0, 1:])
    with pytest.raises(AssertionError):
        P.interpolate_pose(traj, 0.5)  # before the first row: t > 1 fails main.py:134
    with pytest.raises(ValueError):
        P.interpolate_pose(traj, 2.5)


def test_mean_depth():
    rng = np.random.default_rng(11)
    d = rng.integers(0, 20000, (48, 64)).astype(np.uint16)
    d[rng.random(d.shape) < 0.3] = 0
    s = 0.0
    n = 0
    for v in d.reshape(-1):  # utils.cu:82-89, in pixel order
        if v:
            s += int(v) / 5000.0
            n += 1
    assert tum.mean_depth_m(d) == float(np.float32(s / n))
    assert tum.mean_depth_raw(d) == float(np.mean(d[d > 0]))
    assert math.isnan(tum.mean_depth_m(np.zeros((4, 4), np.uint16)))


def test_synthetic_tum_lines_roundtrip_poses():
    """The bench stream's groundtruth lines read back through read_traj + parse_pos give the
    stream's own extrinsics (the host pose path the bench exercises)."""
    st = SyntheticStream(seed=1)
    lines = st.tum_lines(8)
    assert lines[0].startswith("#")
    rows = [ln.split() for ln in lines[1:]]
    traj = np.array([[float(r[0][5:])] + [float(x) for x in r[1:]] for r in rows])
    for k in range(8):
        assert abs(traj[k, 0] - math.fmod(st.stamp(k), 1e5)) < 1e-4
        assert np.allclose(P.parse_pos(traj[k, 1:]), st.frame(k).w2c, atol=1e-8)


def test_associate_python_matches_executed_reference(tmp_path):
    """tum.associate(mode="python") against the reference's own main.py:63-140 loop, executed
    on the same file lists and groundtruth by tests/golden/gen_label_tum.py: identical (i, j)
    pairs (repeats and skips included) and identical interpolated extrinsics."""
    from conftest import GOLDEN

    g = np.load(os.path.join(GOLDEN, "tum_assoc_golden.npz"), allow_pickle=False)
    for case in ("jitter", "half_rate_rgb"):
        root = tmp_path / case
        _write_dir(str(root), [str(s) for s in g[f"{case}_depth"]], [str(s) for s in g[f"{case}_rgb"]],
                   [str(s) for s in g["gt_lines"]], shape=(2, 2))
        py = tum.associate(str(root), "python")
        assert [(f.i, f.j) for f in py] == [tuple(int(x) for x in p) for p in g[f"{case}_pairs"]], case
        assert len(py) > 5
        for f, ext in zip(py, g[f"{case}_extrinsic"]):
            assert np.array_equal(P.parse_pos(f.pose), ext), case
