"""Known-answer and property tests of the C oracle (SURVEY.md §4 test plan), CPU only."""
import numpy as np
import pytest

from semtsdf.synth import SyntheticStream

KI = (520.9, 521.0, 325.1, 249.7)


def _K():
    K = np.eye(4, dtype=np.float32)
    K[(0, 1, 0, 1), (0, 1, 2, 2)] = KI
    return K


def _Kinv():
    fx, fy, cx, cy = KI
    Ki = np.eye(4, dtype=np.float32)
    Ki[0, 0], Ki[0, 2], Ki[1, 1], Ki[1, 2] = 1 / fx, -cx / fx, 1 / fy, -cy / fy
    return Ki


def plane_frame(z0=2.0, W=640, H=480, label=3, rgb=(10, 200, 40)):
    depth = np.full((H, W), int(round(z0 * 5000)), np.uint16)
    col = np.zeros((H, W, 3), np.uint8)
    col[:] = rgb
    mask = np.full((H, W), label, np.uint8)
    return depth, col, mask


def test_fronto_parallel_plane_known_answer(oracle):
    """sdf = clamp(z0 - z, <= mu)/mu for voxels in front of / near the plane, untouched
    (sdf = mu, weight 0) behind it by more than mu; after n identical frames weight = n,
    sdf unchanged, colour = pixel colour, hist[label] = n on gated voxels."""
    D = 32
    z0 = 2.0
    start = np.array([-0.4, -0.3, 1.8], np.float32)
    voxel = np.array([0.4 / 31 * 2, 0.3 / 31 * 2, 0.4 / 31], np.float32)
    mu = np.float32(5 * voxel[2])
    g = oracle.OGeom([D] * 3, start, voxel, mu)
    st = oracle.OState([D] * 3, mu, semantic=True)
    depth, col, mask = plane_frame(z0)
    E = np.eye(4, dtype=np.float32)
    for n in range(1, 4):
        oracle.integrate(g, st, _K(), E, depth, col, mask, flags=0x3)
        z = (start[2] + np.arange(D, dtype=np.float32) * voxel[2]).astype(np.float32)
        diff = np.float32(z0) - z
        sdf = st.sdf.reshape(D, D, D)
        wt = st.wt.reshape(D, D, D)
        hist = st.hist.reshape(D, D, D, 32)
        colr = st.color.reshape(D, D, D, 3)
        cx = D // 2  # a column in the middle of the image
        for zi in range(D):
            if diff[zi] <= -mu:
                assert wt[cx, cx, zi] == 0 and sdf[cx, cx, zi] == mu
            else:
                f = min(diff[zi], mu) / mu
                assert wt[cx, cx, zi] == n
                assert abs(sdf[cx, cx, zi] - f) < 1e-6
                if f < 0.99:
                    assert hist[cx, cx, zi, 3] == n and hist[cx, cx, zi].sum() == n
                    assert tuple(colr[cx, cx, zi]) == (10, 200, 40)
                else:
                    assert hist[cx, cx, zi].sum() == 0


def test_depth_zero_and_off_image_untouched(oracle):
    D = 16
    g = oracle.OGeom([D] * 3, [-5, -5, 1.0], [0.05, 0.05, 0.05], 0.25)
    st = oracle.OState([D] * 3, np.float32(0.25), semantic=True)
    depth, col, mask = plane_frame(1.5)
    depth[:] = 0
    oracle.integrate(g, st, _K(), np.eye(4, dtype=np.float32), depth, col, mask, flags=0x3)
    assert (st.wt == 0).all() and (st.sdf == np.float32(0.25)).all() and st.hist.sum() == 0


def test_label_overflow_counted_not_written(oracle):
    D = 8
    g = oracle.OGeom([D] * 3, [-0.1, -0.1, 1.9], [0.03, 0.03, 0.03], 0.15)
    st = oracle.OState([D] * 3, np.float32(0.15), semantic=True)
    depth, col, mask = plane_frame(2.0, label=40)
    cnt = oracle.integrate(g, st, _K(), np.eye(4, dtype=np.float32), depth, col, mask, flags=0x3)
    assert cnt[2] > 0 and st.hist.sum() == 0


def test_vote_mode_semantics(oracle):
    """TSDF_Python/tsdf.cu:48-57: first label sticks, same label counts up, other down."""
    D = 8
    g = oracle.OGeom([D] * 3, [-0.1, -0.1, 1.9], [0.03, 0.03, 0.03], 0.15)
    st = oracle.OState([D] * 3, np.float32(0.15), color_i32=True, vote=True)
    depth, col, _ = plane_frame(2.0)
    for lab in (5, 5, 7, 7, 7, 7):
        cls = np.full(depth.shape, lab, np.int32)
        oracle.integrate(g, st, _K(), np.eye(4, dtype=np.float32), depth, col, cls=cls, flags=0x4 | 0x8)
    t = st.wt > 0
    # 5 (cnt 1), 5 (2), 7 (1), 7 (0), 7 -> reset to 7 (1), 7 (2)
    assert (st.cls[t] == 7).all() and (st.cls_cnt[t] == 2).all()


def test_association_f32_and_f64_decisions_agree(oracle):
    """The device path accumulates in fixed point/f64; the reference in f32 pixel order.
    On the synthetic stream both give the same relabelled masks."""
    st = SyntheticStream(seed=0)
    D = 48
    f0 = st.frame(0)
    pl = oracle.place(f0.depth, _Kinv(), [D] * 3, np.mean(f0.depth[f0.depth > 0]) / 5000.0, 0)
    g = oracle.OGeom([D] * 3, pl["vol_start"], pl["voxel"], pl["mu"], pl["vol_end"])
    ost = oracle.OState([D] * 3, np.float32(pl["mu"]), semantic=True)
    num = 0
    for k in range(1, 4):
        fr = st.frame(k)
        E = (fr.w2c @ f0.c2w).astype(np.float32)
        m = fr.mask.copy()
        if k == 1:
            num = int(m.max()) + 1
        else:
            probs, box = oracle.march_probs(g, _Kinv(), E, 640, 480, ost.sdf, ost.hist)
            m32, n32, _, p32, _ = oracle.filter_overlaps(probs, box, m, k - 1, num, 0.05, precision=0)
            m64, n64, _, p64, _ = oracle.filter_overlaps(probs, box, m, k - 1, num, 0.05, precision=1)
            assert np.array_equal(m32, m64) and n32 == n64 and np.array_equal(p32, p64)
            m, num = m64, n64
            # labels were permuted per frame: association must map back to consistent ids
            for sph in range(1, 7):
                ids = np.unique(m[fr.gt_ids == sph])
                assert ids.size <= 1
        oracle.integrate(g, ost, _K(), E, fr.depth, fr.rgb, m, flags=0x3)
    assert num <= 8


def test_placement_modes(oracle):
    d = np.zeros((480, 640), np.uint16)
    d[100:200, 50:300] = 10000
    d[150, 400] = 256  # multiple of 256: invisible to the wrapping u8 cast (tsdf.py:35)
    sfm = oracle.place(d, _Kinv(), [64] * 3, 2.0, 0)
    py = oracle.place(d, _Kinv(), [64] * 3, 2.0 * 5000, 1)
    assert sfm["vol_end"][0] > py["vol_end"][0]  # the extra pixel widens the SfM rect only
    assert np.isclose(sfm["mu"], 5 * sfm["voxel"][0])


def test_synthetic_stream_properties():
    st = SyntheticStream(seed=1)
    f = st.frame(0)
    assert f.depth.dtype == np.uint16 and f.rgb.shape == (480, 640, 3) and f.mask.dtype == np.uint8
    valid = f.depth > 0
    assert 0.96 < valid.mean() < 0.99  # 2 % dropout
    z = f.depth[valid] / 5000.0
    assert z.max() <= 3.0 + 1e-3 and z.min() > 0.5
    assert f.mask.max() <= 6 and set(np.unique(f.mask)) - {0} == set(range(1, f.mask.max() + 1))
    f2 = SyntheticStream(seed=1).frame(0)
    assert np.array_equal(f.depth, f2.depth) and np.array_equal(f.mask, f2.mask)


def test_reciprocal_division_is_correctly_rounded(oracle):
    """k_integrate divides by mu and by w+1 through RN reciprocals (div_by_rcp, Markstein);
    it must equal the IEEE quotient of the reference (tsdf.cu:52,56) for |a| >= 2^-60."""
    rng = np.random.default_rng(5)
    # diff / mu: diff in [-mu, mu], mu = 5 voxel for voxels of 0.5 mm .. 10 cm
    for mu in np.float32([0.0025, 0.0234375, 0.03125, 0.5]).tolist() + rng.uniform(0.002, 0.5, 12).astype(
            np.float32).tolist():
        mu = np.float32(mu)
        a = np.concatenate([rng.uniform(-mu, mu, 200000).astype(np.float32),
                            np.float32(mu) * np.float32([1, -1, 0.5, -0.5, 0.999999, 1e-6, -1e-12]),
                            (rng.standard_normal(20000) * np.float32(2.0) ** rng.integers(-60, 0, 20000)).astype(
                                np.float32)])
        a = np.clip(a, -mu, mu)
        assert oracle.div_rcp_mismatches(a, float(mu)) == 0, mu
    # (sdf * w + f) / (w + 1): |numerator| <= w + 1, w + 1 <= 4096 (the LDS table)
    for den in list(range(1, 70)) + rng.integers(70, 4097, 60).tolist():
        a = rng.uniform(-den, den, 20000).astype(np.float32)
        assert oracle.div_rcp_mismatches(a, float(den)) == 0, den


def test_colour_mean_reciprocal_floor_is_exact():
    """k_integrate's u8 colour running mean (avg_u8): floor(RN(num * RN(1/d) + 2^-12)) equals
    the reference's integer quotient (c*w + x) / (w + 1) (tsdf.cu:57-60) for every c, x in
    0..255 and every d = w + 1 <= 1024 (the reciprocal table), exhaustively (67M cases).
    The product num * r is exact in float64, so adding 2^-12 and rounding once to float32
    is exactly the kernel's fma."""
    o = np.arange(256, dtype=np.int64)[:, None]
    x = np.arange(256, dtype=np.int64)[None, :]
    for den in range(1, 1025):
        num = (o * (den - 1) + x).ravel()
        r = np.float64(np.float32(1.0) / np.float32(den))
        v = (num.astype(np.float64) * r + 2.0 ** -12).astype(np.float32)
        assert np.array_equal(np.floor(v).astype(np.int64), num // den), den
