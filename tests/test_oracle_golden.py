"""Pin the oracles against golden vectors produced by the reference's own code
(tests/golden/gen_golden.py executed src/TSDF_Python/tsdf.py:32-52 and :78-120).

* The NumPy restatement (oracle.numpy_integrate) must reproduce the reference block
  bit for bit (same float64 arithmetic, same storage dtypes).
* The f32 C restatement (the bit-level reference of the HIP kernels) must agree with the
  float64 reference within the north star's 1e-4 on SDF, exactly on weight and colour,
  on every voxel whose f32 and f64 pixel choice agree; the voxels where they differ are
  bounded by a mismatch budget (4.5e-5 of voxels measured at 256^3).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

K = np.eye(4, dtype=np.float32)
K[(0, 1, 0, 1), (0, 1, 2, 2)] = (520.9, 521.0, 325.1, 249.7)


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="module")
def frames():
    f = _load("frames_tum_fr2.npz")
    return {"a": (f["depth_a"], f["rgb_a"]), "b": (f["depth_b"], f["rgb_b"])}


CASES = {"d64": ["a", "a", "b"], "d128": ["a"]}


def _dense(g, k, n):
    idx = g[f"f{k}_idx"]
    return idx, g[f"f{k}_sdf"], g[f"f{k}_wt"], g[f"f{k}_color"]


@pytest.mark.parametrize("case", ["d64", "d128"])
def test_numpy_restatement_matches_reference_block(case, frames, oracle):
    g = _load(f"integrate_{case}.npz")
    D = int(g["vol_dim"])
    n = int(g["f0_nflat"])  # tex_dim^2: the reference visits only these flat indices
    mu = float(g["place_mu"])
    sdf = np.full(n, mu, np.float64)  # NEP 50: ones(f32) * np.float64 -> float64 (tsdf.py:48)
    wt = np.zeros(n, np.int32)
    col = np.zeros((n, 3), np.int32)
    for k, fr in enumerate(CASES[case]):
        depth, rgb = frames[fr]
        oracle.numpy_integrate(sdf, wt, col, D, g["place_vol_start"], g["place_voxel"], mu, K, g[f"f{k}_E"], depth, rgb,
                               n_flat=n)
        idx, r_sdf, r_wt, r_col = _dense(g, k, n)
        assert np.array_equal(np.nonzero(wt)[0], idx)
        assert np.array_equal(sdf[idx], r_sdf)
        assert np.array_equal(wt[idx], r_wt)
        assert np.array_equal(col[idx], r_col)
    if case == "d128":
        assert n == 1448 * 1448 and D ** 3 - n == 448  # tsdf.py:22 truncation, SURVEY §0.4


def test_placement_python_mode_matches_reference(frames):
    from semtsdf.tsdf import bounding_rect_nonzero

    g = _load("integrate_d64.npz")
    depth, _ = frames["a"]
    mean = np.mean(depth[depth > 0])
    kinv = np.linalg.inv(K)
    rect = bounding_rect_nonzero(depth.astype(np.uint8))
    tl = np.dot(kinv[:3, :3], [rect[0], rect[1], 1]) * (mean / 5000)
    br = np.dot(kinv[:3, :3], [rect[0] + rect[2], rect[1] + rect[3], 1]) * (mean / 5000)
    half = np.sqrt(np.dot(tl[:2] - br[:2], tl[:2] - br[:2])) / 2
    c = (tl + br) / 2
    assert np.array_equal(c - half, g["place_vol_start"])
    assert np.array_equal(c + half, g["place_vol_end"])
    assert np.array_equal((2 * half) / 63 * np.ones(3), g["place_voxel"]) or np.allclose(
        ((c + half) - (c - half)) / 63, g["place_voxel"], rtol=0, atol=0)
    assert float(g["place_mu"]) == 5 * g["place_voxel"][0]


def test_pose_math_matches_reference():
    from semtsdf import pose as P

    g = _load("pose_golden.npz")
    for i, p in enumerate(g["poses"]):
        assert np.allclose(P.transform44(p), g["transform44"][i], rtol=0, atol=1e-12)
        assert np.allclose(P.parse_pos(p), g["parse_pos"][i], rtol=0, atol=1e-12)
        assert np.allclose(P.parse_pos(p), g["transform44"][i], rtol=0, atol=1e-12)
    q = g["poses"][:, 3:]
    ref = g["slerp"]
    for j, t in enumerate((0.0, 0.25, 0.5, 1.0)):
        assert np.allclose(P.slerp(q[0], q[1], t), ref[j], rtol=0, atol=1e-14)
    assert np.allclose(P.slerp(q[0], -q[2], 0.3), ref[4], rtol=0, atol=1e-14)


def test_transform44_degenerate_branch_matches_reference():
    from semtsdf import pose as P

    g = _load("pose_golden.npz")
    assert np.array_equal(P.transform44(g["degenerate_pose"]), g["transform44_degenerate"])


def c1_frames():
    """The C1 golden's frames: the seeded synthetic stream (seed 0), regenerated and checked
    against the checksums stored by gen_golden.py."""
    from semtsdf.synth import SyntheticStream

    g = _load("integrate_c1_d128.npz")
    st = SyntheticStream(seed=0)
    frames = [st.frame(k) for k in range(int(g["n_frames"]))]
    sums = [int(f.depth.astype(np.int64).sum()) ^ (int(f.rgb.astype(np.int64).sum()) << 1) for f in frames]
    assert sums == [int(x) for x in g["frame_sums"]], "synthetic stream drifted from the golden's frames"
    return g, frames


def test_numpy_restatement_matches_reference_c1():
    """C1 (128^3, 20 frames): the NumPy restatement reproduces the executed reference block."""
    import oracle as O

    g, frames = c1_frames()
    D, n = int(g["vol_dim"]), int(g["n_flat"])
    mu = float(g["place_mu"])
    sdf = np.full(n, mu, np.float64)
    wt = np.zeros(n, np.int32)
    col = np.zeros((n, 3), np.int32)
    for k, fr in enumerate(frames):
        O.numpy_integrate(sdf, wt, col, D, g["place_vol_start"], g["place_voxel"], mu, K, g["E"][k], fr.depth, fr.rgb,
                          n_flat=n)
    idx = g["idx"].astype(np.int64)
    assert np.array_equal(np.nonzero(wt)[0], idx)
    assert np.array_equal(sdf[idx].astype(np.float32), g["sdf"])
    assert np.array_equal(wt[idx], g["wt"]) and np.array_equal(col[idx], g["color"])


def agreeing_voxels(oracle, D, n_flat, vol_start, voxel, mu, Es, frames, Es32=None):
    """Voxels whose f32 pixel choice (the build's contract) equals the float64 reference
    block's in every frame -- the only place the two integrates can differ beyond rounding --
    and the voxels that the NumPy block's truncation toward zero accepted at pixel column or
    row 0 (u or v in (-1, 0)) while the reference's CUDA floor (__float2int_rd, tsdf.cu:43-44),
    which the contract follows, rejects them: a defined difference, not a rounding one.
    Es: the reference's float64 relative poses; Es32: the f32 poses the build used (default
    Es rounded to f32)."""
    og = oracle.OGeom([D] * 3, vol_start, voxel, mu)
    agree = np.ones(D ** 3, bool)
    edge = np.zeros(D ** 3, bool)
    for i, (E, (depth, rgb)) in enumerate(zip(Es, frames)):
        H, W = depth.shape
        a = oracle.project(og, K, (E if Es32 is None else Es32[i]).astype(np.float32), W, H)
        b = np.full(D ** 3, -2, np.int64)
        b[:n_flat] = oracle.numpy_pixels(D, vol_start, voxel, K, E, W, H, n_flat)
        agree &= a == b
        edge |= (a == -1) & (b >= 0) & (((b % W) == 0) | ((b // W) == 0))
    return agree, edge


def check_against_golden(sdf, wt, col, D, n_flat, mu, idx, r_sdf, r_wt, r_col, agree, edge, n_frames):
    """The parity rule against the float64 reference: on voxels whose pixel choice agreed in
    every frame, |dsdf| <= 1e-4 and weight and colour exact; the truncation-edge voxels are
    excluded (see agreeing_voxels); the other pixel-border voxels whose state differs are
    bounded by a mismatch budget of 1e-4 of the visited voxels per integrated frame."""
    n = D ** 3
    ref_wt = np.zeros(n, np.int64)
    ref_wt[idx] = r_wt
    ref_sdf = np.full(n, mu)
    ref_sdf[idx] = r_sdf
    ref_col = np.zeros((n, 3), np.int64)
    ref_col[idx] = r_col
    vis = np.zeros(n, bool)
    vis[:n_flat] = True  # the reference visits only tex_dim^2 flat indices (tsdf.py:22)
    ok = agree & vis
    border = ~agree & ~edge & vis
    differs = (np.abs(sdf - ref_sdf) > 1e-4) | (wt != ref_wt) | (col.reshape(-1, 3) != ref_col).any(axis=1)
    assert (border & differs).sum() <= 1e-4 * n_frames * n_flat, (border & differs).sum()
    assert np.abs(sdf[ok] - ref_sdf[ok]).max() <= 1e-4
    assert np.array_equal(wt[ok], ref_wt[ok])
    assert np.array_equal(col.reshape(-1, 3)[ok], ref_col[ok])
    return ok


def test_c_oracle_vs_reference_c1_exact_on_agreeing_pixels(oracle):
    g, frames = c1_frames()
    D, n_flat = int(g["vol_dim"]), int(g["n_flat"])
    mu = float(g["place_mu"])
    og = oracle.OGeom([D] * 3, g["place_vol_start"], g["place_voxel"], mu)
    st = oracle.OState([D] * 3, np.float32(mu), semantic=False, color_i32=True)
    for k, fr in enumerate(frames):
        oracle.integrate(og, st, K, g["E"][k].astype(np.float32), fr.depth, fr.rgb, flags=0x4)
    agree, edge = agreeing_voxels(oracle, D, n_flat, g["place_vol_start"], g["place_voxel"], mu, g["E"],
                                  [(f.depth, f.rgb) for f in frames])
    ok = check_against_golden(st.sdf, st.wt, st.color, D, n_flat, mu, g["idx"].astype(np.int64), g["sdf"], g["wt"],
                              g["color"], agree, edge, len(frames))
    assert (st.wt[ok] > 0).sum() > 100_000


def test_c_oracle_vs_reference_d64_exact_colour(frames, oracle):
    """The d64 golden (3 real frames) under the same rule: colour exact wherever the pixel
    choice agreed in every frame so far (this replaces a 0.999 colour-agreement bound)."""
    g = _load("integrate_d64.npz")
    D = 64
    mu = float(g["place_mu"])
    og = oracle.OGeom([D] * 3, g["place_vol_start"], g["place_voxel"], mu)
    st = oracle.OState([D] * 3, np.float32(mu), semantic=False, color_i32=True)
    seq = [frames[c] for c in CASES["d64"]]
    for k, (depth, rgb) in enumerate(seq):
        oracle.integrate(og, st, K, g[f"f{k}_E"].astype(np.float32), depth, rgb, flags=0x4)
        agree, edge = agreeing_voxels(oracle, D, D ** 3, g["place_vol_start"], g["place_voxel"], mu,
                                      [g[f"f{j}_E"] for j in range(k + 1)], seq[: k + 1])
        check_against_golden(st.sdf, st.wt, st.color, D, D ** 3, mu, g[f"f{k}_idx"], g[f"f{k}_sdf"], g[f"f{k}_wt"],
                             g[f"f{k}_color"], agree, edge, k + 1)


@pytest.mark.parametrize("fname", ["a", "b"])
@pytest.mark.parametrize("D", [64, 128, 256])
def test_library_placement_matches_reference_and_oracle(frames, oracle, fname, D):
    """semtsdf_place_from_frame (a host function of the C ABI; no GPU call): Python mode
    against the executed reference init_vars (tsdf.py:32-52), rounded once to the f32
    parameter block; SfM mode (tsdf.cu:173-199) against the C restatement."""
    import semtsdf
    from semtsdf import _lib as L

    g = _load("placement_golden.npz")
    depth, _ = frames[fname]
    p = semtsdf.default_params(D, (520.9, 521.0, 325.1, 249.7), 640, 480)
    p.Kinv[:] = [float(x) for x in g[f"{fname}{D}_intrinsic_inv"].astype(np.float32).reshape(-1)]
    semtsdf.place_from_frame(p, depth, float(g[f"{fname}{D}_mean_depth"]), L.PLACE_PYTHON)
    for key in ("vol_start", "vol_end", "voxel"):
        assert np.array_equal(np.array(getattr(p, key)[:], np.float32), g[f"{fname}{D}_{key}"].astype(np.float32)), key
    assert np.float32(p.mu) == np.float32(g[f"{fname}{D}_mu"])
    kinv = np.array(p.Kinv[:], np.float32)
    for mode, mean in ((L.PLACE_PYTHON, float(g[f"{fname}{D}_mean_depth"])),
                       (L.PLACE_SFM, float(np.float32(g[f"{fname}{D}_mean_depth"] / 5000.0)))):
        q = semtsdf.default_params(D, (520.9, 521.0, 325.1, 249.7), 640, 480)
        q.Kinv[:] = [float(x) for x in kinv]
        semtsdf.place_from_frame(q, depth, mean, mode)
        o = oracle.place(depth, kinv, [D] * 3, mean, mode)
        for key in ("vol_start", "vol_end", "voxel"):
            assert np.array_equal(np.array(getattr(q, key)[:], np.float32), o[key]), (mode, key)
        assert np.float32(q.mu) == np.float32(o["mu"])


def hist_golden_check(D, hist, wt, oracle):
    """The label path against the reference's own first-frame class count (tsdf.py:122-130,
    executed by tests/golden/gen_label_tum.py after the integrate block on a real frame with
    synthetic non-overlapping instance masks).  `hist` [D^3, 32] is a semantic, UNGATED state
    after that one frame (label k + 1 where mask channel k is set, 0 elsewhere).  On the touched
    voxels whose f32 pixel choice equals the float64 block's: bin k + 1 == the reference count
    of channel k for every channel, and bin 0 (background, tsdf.cu:61) counts the rest.
    Returns the number of compared voxels."""
    g = _load("hist_golden.npz")
    n_cls = int(g["n_cls"])
    vs, vx, mu = g[f"d{D}_vol_start"], g[f"d{D}_voxel"], float(g[f"d{D}_mu"])
    n_flat = int(g[f"d{D}_nflat"])
    idx, cnt = g[f"d{D}_idx"], g[f"d{D}_cls_cnt"].astype(np.uint32)
    f = _load("frames_tum_fr2.npz")
    agree, edge = agreeing_voxels(oracle, D, n_flat, vs, vx, mu, [g[f"d{D}_E"]], [(f["depth_a"], f["rgb_a"])])
    hist = hist.reshape(-1, 32)
    sel = agree[idx]
    assert sel.mean() > 0.999  # only pixel-border voxels differ in their pixel
    v = idx[sel]
    assert np.array_equal(wt[v] > 0, np.ones(v.size, bool))
    assert np.array_equal(hist[v, 1:n_cls + 1], cnt[sel])
    assert np.array_equal(hist[v, 0], 1 - cnt[sel].sum(axis=1))
    assert not hist[v, n_cls + 1:].any()
    assert int(cnt[sel].sum()) > 1000  # the instances are actually seen
    return int(v.size)


@pytest.mark.parametrize("D", [64, 128])
def test_c_oracle_histogram_matches_reference_class_count(D, oracle):
    g = _load("hist_golden.npz")
    f = _load("frames_tum_fr2.npz")
    og = oracle.OGeom([D] * 3, g[f"d{D}_vol_start"], g[f"d{D}_voxel"], float(g[f"d{D}_mu"]))
    st = oracle.OState([D] * 3, np.float32(g[f"d{D}_mu"]), semantic=True)
    oracle.integrate(og, st, K, g[f"d{D}_E"].astype(np.float32), f["depth_a"], f["rgb_a"], mask=g["labels"],
                     flags=0x1)
    assert hist_golden_check(D, st.hist, st.wt, oracle) > 10_000
