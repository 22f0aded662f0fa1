"""GPU parity: the HIP path (through the C ABI) against the C oracle and the golden
vectors of the reference's NumPy integrate.  Bit-exact for integer state and sdf bits,
1e-4 + mismatch budget against the float64 reference block."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

KI = (520.9, 521.0, 325.1, 249.7)


@pytest.fixture(scope="module")
def S():
    import semtsdf
    from semtsdf import _lib as L

    semtsdf.load()
    return semtsdf, L


@pytest.fixture(scope="module")
def stream():
    from semtsdf.synth import SyntheticStream

    st = SyntheticStream(seed=0)
    return st, [st.frame(k) for k in range(6)]


def make(S, oracle, dims, frame0, flags, cull=True):
    semtsdf, L = S
    p = semtsdf.default_params(64, KI, 640, 480)
    p.dim[0], p.dim[1], p.dim[2] = dims
    semtsdf.place_from_frame(p, frame0.depth, float(np.mean(frame0.depth[frame0.depth > 0])) / 5000.0, L.PLACE_SFM)
    p.flags = flags | (0 if cull else L.F_NO_CULL)
    vol = semtsdf.Volume(p, 0)
    g = oracle.OGeom.from_params(p)
    ost = oracle.OState(list(dims), p.mu, semantic=bool(flags & 1), color_i32=bool(flags & 4), vote=bool(flags & 8))
    return p, vol, g, ost


def assert_same(vol, ost, hist=False, cls=False):
    out = vol.download(hist=hist, cls=cls)
    assert np.array_equal(out["sdf"].view(np.uint32), ost.sdf.view(np.uint32)), "sdf bits"
    assert np.array_equal(out["wt"], ost.wt), "weight"
    assert np.array_equal(out["color"], ost.color), "colour"
    if hist:
        assert np.array_equal(out["hist"], ost.hist), "histogram"
    if cls:
        assert np.array_equal(out["cls"], ost.cls) and np.array_equal(out["cls_cnt"], ost.cls_cnt), "vote"


@pytest.mark.parametrize("flags", [0x3, 0x4, 0x7, 0x1, 0x2])
@pytest.mark.parametrize("cull", [True, False])
def test_integrate_bit_exact(S, oracle, stream, flags, cull):
    st, frames = stream
    dims = (64, 64, 64)
    p, vol, g, ost = make(S, oracle, dims, frames[0], flags, cull)
    for k in range(1, 4):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        m = fr.gt_ids if flags & 1 else None
        vol.integrate(fr.depth, fr.rgb, m, E)
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, m, flags=flags)
    assert_same(vol, ost, hist=bool(flags & 1))
    vol.close()


def test_integrate_ragged_dims_and_real_frames(S, oracle):
    """Dims that are not multiples of the 8x8x32 brick, real TUM frames."""
    f = np.load(os.path.join(GOLDEN, "frames_tum_fr2.npz"))
    semtsdf, L = S

    class Fr:
        pass

    f0 = Fr()
    f0.depth = f["depth_a"]
    p, vol, g, ost = make(S, oracle, (37, 70, 45), f0, 0x3)
    rng = np.random.default_rng(3)
    for k, (d, c) in enumerate(((f["depth_a"], f["rgb_a"]), (f["depth_b"], f["rgb_b"]))):
        E = np.eye(4, dtype=np.float32)
        E[:3, 3] = (0.01 * k, -0.02 * k, 0.0)
        m = rng.integers(0, 6, d.shape).astype(np.uint8)
        vol.integrate(d, c, m, E)
        oracle.integrate(g, ost, list(p.K), E, d, c, m, flags=0x3)
    assert_same(vol, ost, hist=True)
    vol.close()


def test_vote_mode_and_dropin(S, oracle, stream):
    from semtsdf import tsdf_cuda

    st, frames = stream
    semtsdf, L = S
    D = 40
    f0 = frames[0]
    pl = oracle.place(f0.depth, np.array(semtsdf.default_params(D, KI, 640, 480).Kinv[:], np.float32), [D] * 3,
                      np.mean(f0.depth[f0.depth > 0]) / 5000.0, 0)
    n = D ** 3
    sdf = np.full(n, np.float32(pl["mu"]), np.float32)
    wt = np.zeros(n, np.int32)
    col = np.zeros(n * 3, np.int32)
    cls = np.zeros(n, np.int32)
    cnt = np.zeros(n, np.int32)
    K = np.eye(4, dtype=np.float32)
    K[(0, 1, 0, 1), (0, 1, 2, 2)] = KI
    g = oracle.OGeom([D] * 3, pl["vol_start"], [pl["voxel"][0]] * 3, pl["mu"])
    ost = oracle.OState([D] * 3, np.float32(pl["mu"]), color_i32=True, vote=True)
    for k in range(1, 4):
        fr = frames[k]
        E = (fr.w2c @ f0.c2w).astype(np.float32)
        c_in = fr.gt_ids.astype(np.int32)
        tsdf_cuda.tsdf_update(sdf, col, wt, cls, cnt, D, pl["vol_start"], float(pl["voxel"][0]), float(pl["mu"]), K,
                              fr.depth, fr.rgb, c_in, E, 640, 480)
        oracle.integrate(g, ost, K, E, fr.depth, fr.rgb, cls=c_in, flags=0xC)
    assert np.array_equal(sdf.view(np.uint32), ost.sdf.view(np.uint32))
    assert np.array_equal(wt, ost.wt) and np.array_equal(col, ost.color)
    assert np.array_equal(cls, ost.cls) and np.array_equal(cnt, ost.cls_cnt)


def test_association_probs_and_relabel(S, oracle, stream):
    st, frames = stream
    semtsdf, L = S
    p, vol, g, ost = make(S, oracle, (64, 64, 64), frames[0], 0x3)
    num = 0
    for k in range(1, 6):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        m_gpu = np.ascontiguousarray(fr.mask.copy())
        if k >= 2:
            probs_g, box_g = vol.assoc_probs(E)
            probs_o, box_o = oracle.march_probs(g, list(p.Kinv), E, 640, 480, ost.sdf, ost.hist, p.box_thresh)
            assert np.array_equal(probs_g.reshape(-1).view(np.uint32), probs_o.view(np.uint32))
            assert np.array_equal(box_g.reshape(-1), box_o)
        stats = vol.parse_frame(fr.depth, fr.rgb, m_gpu, E)
        m_ref = fr.mask.copy()
        if k == 1:
            num = int(m_ref.max()) + 1
        else:
            m_ref, num, _, prev, _ = oracle.filter_overlaps(probs_o, box_o, m_ref, k - 1, num, p.prior_mrcnn_err_rate,
                                                            precision=0)
            assert np.array_equal(np.array(stats.assigned_prev[:]), prev)
            assert stats.num_objs == num
        assert np.array_equal(m_gpu, m_ref), f"frame {k}"
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, m_ref, flags=0x3)
        stt = vol.state()
        assert stt.n_obs == k and stt.num_objs == num
    assert_same(vol, ost, hist=True)
    vol.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_render_matches_oracle(S, oracle, stream, mode):
    st, frames = stream
    semtsdf, L = S
    p, vol, g, ost = make(S, oracle, (64, 64, 64), frames[0], 0x3)
    for k in range(1, 4):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        vol.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, fr.gt_ids, flags=0x3)
    dist = float(np.mean(frames[0].depth[frames[0].depth > 0]) / 5000.0)
    for angle in (0.0, 0.2):
        s2w, c = semtsdf.orbit_camera(list(p.Kinv), angle, dist)
        s2w_o, c_o = oracle.orbit_camera(list(p.Kinv), angle, dist)
        assert np.array_equal(s2w, s2w_o) and np.array_equal(c, c_o)
        img, t = vol.raycast(s2w, c, mode, want_t=True)
        ref, t_ref = oracle.render(g, s2w, c, 640, 480, mode, ost.sdf, ost.hist, ost.color)
        diff = (img != ref).any(axis=-1)
        assert not diff.any(), (angle, int(diff.sum()))
        assert (t >= 0).mean() > 0.2  # the scene is actually hit
        assert np.array_equal(t.view(np.uint32), t_ref.view(np.uint32))
    vol.close()


def test_render_and_association_256_match_oracle(S, oracle, stream):
    """At 256^3 (32 bricks per axis: octant distance boxes up to the cap, LDS-staged map
    passes, dirty-brick refresh between frames) the hit distances and labels of a render and
    the association probabilities equal the oracle's."""
    st, frames = stream
    semtsdf, L = S
    p, vol, g, ost = make(S, oracle, (256, 256, 256), frames[0], 0x3)
    dist = float(np.mean(frames[0].depth[frames[0].depth > 0]) / 5000.0)
    for k in range(1, 4):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        vol.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, fr.gt_ids, flags=0x3)
        if k < 3:  # a render between frames: the next refresh is a dirty-brick update
            vol.raycast(*semtsdf.orbit_camera(list(p.Kinv), 0.1, dist), L.RENDER_LABEL)
    s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.3, dist)
    img, t = vol.raycast(s2w, c, L.RENDER_LABEL, want_t=True)
    ref, t_ref = oracle.render(g, s2w, c, 640, 480, L.RENDER_LABEL, ost.sdf, ost.hist, ost.color)
    assert (t >= 0).mean() > 0.2
    assert np.array_equal(t.view(np.uint32), t_ref.view(np.uint32))
    assert np.array_equal(img, ref), int((img != ref).any(axis=-1).sum())
    E = (frames[4].w2c @ frames[0].c2w).astype(np.float32)
    vol.set_state(3, 6)
    probs_g, box_g = vol.assoc_probs(E)
    probs_o, box_o = oracle.march_probs(g, list(p.Kinv), E, 640, 480, ost.sdf, ost.hist, p.box_thresh)
    assert np.array_equal(probs_g.reshape(-1).view(np.uint32), probs_o.view(np.uint32))
    vol.close()


def test_integrate_general_intrinsics(S, oracle, stream):
    """A K with skew and a non-unit last row (not the pinhole fast path): the general
    screen map s = M p + m with a separate camera depth row, bit-exact."""
    st, frames = stream
    semtsdf, L = S
    dims = (48, 40, 56)
    p, vol, g, ost = make(S, oracle, dims, frames[0], 0x3)
    vol.close()
    p.K[1] = 2.5     # skew
    p.K[10] = 1.001  # K[2][2]
    vol = semtsdf.Volume(p, 0)
    for k in range(1, 4):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        vol.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, fr.gt_ids, flags=0x3)
    assert (ost.wt > 0).sum() > 1000
    assert_same(vol, ost, hist=True)
    vol.close()


def test_uploaded_volume_raycasts_and_associates(S, oracle, stream):
    """A volume state integrated by the oracle alone and uploaded through the ABI: the
    histogram bin mask and the empty-space maps are rebuilt by the upload, so label render
    and association probabilities match the oracle on it."""
    st, frames = stream
    semtsdf, L = S
    p, vol, g, ost = make(S, oracle, (64, 64, 64), frames[0], 0x3)
    for k in range(1, 4):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, fr.gt_ids, flags=0x3)
    vol.upload(sdf=ost.sdf, wt=ost.wt, color=ost.color, hist=ost.hist)
    vol.set_state(3, int(frames[1].gt_ids.max()) + 1)
    back = vol.download(hist=True)
    assert np.array_equal(back["hist"], ost.hist)
    dist = float(np.mean(frames[0].depth[frames[0].depth > 0]) / 5000.0)
    s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.1, dist)
    img, t = vol.raycast(s2w, c, L.RENDER_LABEL, want_t=True)
    ref, t_ref = oracle.render(g, s2w, c, 640, 480, 0, ost.sdf, ost.hist, ost.color)
    assert np.array_equal(img, ref), int((img != ref).any(axis=-1).sum())
    assert np.array_equal(t.view(np.uint32), t_ref.view(np.uint32))
    fr = frames[4]
    E = (fr.w2c @ frames[0].c2w).astype(np.float32)
    probs_g, box_g = vol.assoc_probs(E)
    probs_o, box_o = oracle.march_probs(g, list(p.Kinv), E, 640, 480, ost.sdf, ost.hist, p.box_thresh)
    assert (probs_o > 0).sum() > 1000  # the scene is actually hit and labelled
    assert np.array_equal(probs_g.reshape(-1).view(np.uint32), probs_o.view(np.uint32))
    assert np.array_equal(box_g.reshape(-1), box_o)
    vol.close()


def test_gpu_vs_numpy_reference_golden(S, oracle):
    """GPU integrate (TSDF+colour mode, NumPy rule: i32 colour, ungated) against the executed
    reference block (d64: 3 real frames): |dsdf| <= 1e-4, weight and colour exact on every
    voxel whose pixel choice agreed with the float64 block in every frame so far, differing
    pixel-border voxels within the 1e-4 budget (tests/test_oracle_golden.py)."""
    from test_oracle_golden import agreeing_voxels, check_against_golden

    semtsdf, L = S
    g = np.load(os.path.join(GOLDEN, "integrate_d64.npz"))
    f = np.load(os.path.join(GOLDEN, "frames_tum_fr2.npz"))
    frames = [(f["depth_a"], f["rgb_a"]), (f["depth_a"], f["rgb_a"]), (f["depth_b"], f["rgb_b"])]
    D = 64
    p = semtsdf.default_params(D, KI, 640, 480)
    for i in range(3):
        p.vol_start[i] = g["place_vol_start"][i]
        p.vol_end[i] = g["place_vol_end"][i]
        p.voxel[i] = g["place_voxel"][i]
    p.mu = float(g["place_mu"])
    p.flags = L.F_COLOR_I32
    vol = semtsdf.Volume(p, 0)
    mu = float(g["place_mu"])
    for k, (d, c) in enumerate(frames):
        vol.integrate(d, c, None, g[f"f{k}_E"].astype(np.float32))
        out = vol.download()
        agree, edge = agreeing_voxels(oracle, D, D ** 3, g["place_vol_start"], g["place_voxel"], mu,
                                      [g[f"f{j}_E"] for j in range(k + 1)], frames[: k + 1])
        check_against_golden(out["sdf"], out["wt"], out["color"], D, D ** 3, mu, g[f"f{k}_idx"], g[f"f{k}_sdf"],
                             g[f"f{k}_wt"], g[f"f{k}_color"], agree, edge, k + 1)
    vol.close()


def test_gpu_d128_golden(S, oracle):
    """The d128 golden (one real frame at 128^3, whose flat layout the reference truncates to
    1448^2 voxels) through the HIP path, same rule."""
    from test_oracle_golden import agreeing_voxels, check_against_golden

    semtsdf, L = S
    g = np.load(os.path.join(GOLDEN, "integrate_d128.npz"))
    f = np.load(os.path.join(GOLDEN, "frames_tum_fr2.npz"))
    D = 128
    n_flat = int(g["f0_nflat"])
    p = semtsdf.default_params(D, KI, 640, 480)
    for i in range(3):
        p.vol_start[i] = g["place_vol_start"][i]
        p.vol_end[i] = g["place_vol_end"][i]
        p.voxel[i] = g["place_voxel"][i]
    p.mu = float(g["place_mu"])
    p.flags = L.F_COLOR_I32
    vol = semtsdf.Volume(p, 0)
    vol.integrate(f["depth_a"], f["rgb_a"], None, g["f0_E"].astype(np.float32))
    out = vol.download()
    agree, edge = agreeing_voxels(oracle, D, n_flat, g["place_vol_start"], g["place_voxel"], float(g["place_mu"]),
                                  [g["f0_E"]], [(f["depth_a"], f["rgb_a"])])
    ok = check_against_golden(out["sdf"], out["wt"], out["color"], D, n_flat, float(g["place_mu"]), g["f0_idx"],
                              g["f0_sdf"], g["f0_wt"], g["f0_color"], agree, edge, 1)
    assert (out["wt"][ok] > 0).sum() > 100_000
    vol.close()


def test_gpu_c1_golden_through_host_class(S, oracle):
    """C1 (BASELINE configs[0]: NumPy integrate, 128^3, 20 frames, no masks) on the HIP path,
    driven by the host TSDF class exactly as TSDF_Python/main.py drives tsdf.py: Python
    placement (init_vars, checked against the executed reference), frame 0 integrated with
    the identity-like relative pose, poses from TUM lines via the host pose path.  Final
    state against the executed reference block's, by the golden rule."""
    from semtsdf import FusionConfig, TSDF
    from semtsdf import pose as P
    from test_oracle_golden import agreeing_voxels, c1_frames, check_against_golden

    g, frames = c1_frames()
    D, n_flat = int(g["vol_dim"]), int(g["n_flat"])
    from semtsdf.synth import SyntheticStream

    st = SyntheticStream(seed=0)
    B = g["world_offset"]
    lines = [P.c2w_to_tum(st.stamp(k), B @ st.c2w(k)) for k in range(len(frames))]
    traj = np.array([[float(ln.split()[0][5:])] + [float(x) for x in ln.split()[1:]] for ln in lines])
    cfg = FusionConfig(vol_dim=D, placement="python", integrate_first_frame=True, semantic=False, gate_color=False,
                       color_i32=True)
    t = TSDF(KI, D, cfg)
    for k, fr in enumerate(frames):
        t.parse_frame(fr.depth, fr.rgb, P.parse_pos(traj[k, 1:]), np.mean(fr.depth[fr.depth > 0]))
        if k == 0:  # init_vars (tsdf.py:32-52) restated on the host: identical float64 results
            assert np.array_equal(t.vol_start, g["place_vol_start"]) and np.array_equal(t.voxel, g["place_voxel"])
            assert t.mu == float(g["place_mu"])
    assert t.N == len(frames)
    out = t.vol.download()
    mu = float(g["place_mu"])
    ext = [P.parse_pos(traj[k, 1:]) for k in range(len(frames))]
    E_host = [P.relative_pose(e, np.linalg.inv(ext[0])) for e in ext]  # what parse_frame passed down
    assert max(np.abs(E_host[k] - g["E"][k].astype(np.float32)).max() for k in range(len(frames))) < 1e-7
    agree, edge = agreeing_voxels(oracle, D, n_flat, g["place_vol_start"], g["place_voxel"], mu, g["E"],
                                  [(f.depth, f.rgb) for f in frames], Es32=E_host)
    ok = check_against_golden(out["sdf"], out["wt"], out["color"], D, n_flat, mu, g["idx"].astype(np.int64),
                              g["sdf"], g["wt"], g["color"], agree, edge, len(frames))
    assert (out["wt"][ok] > 0).sum() > 100_000
    t.close()


def test_host_tsdf_class_and_checkpoint(S, oracle, stream, tmp_path):
    from semtsdf import TSDF, FusionConfig

    st, frames = stream
    t = TSDF(KI, 48, FusionConfig(vol_dim=48))
    for k in range(0, 4):
        fr = frames[k]
        mean_m = float(np.mean(fr.depth[fr.depth > 0]) / 5000.0)
        m = fr.mask.copy()
        t.parse_frame(fr.depth, fr.rgb, fr.w2c, mean_m, m)
    assert t.N == 3 and t.n_obs == 3  # SfM: frame 0 places only
    path = str(tmp_path / "vol.npz")
    t.save(path)
    t2 = TSDF.load(path, FusionConfig(vol_dim=48))
    a = t.vol.download(hist=True)
    b = t2.vol.download(hist=True)
    for key in a:
        assert np.array_equal(a[key], b[key]), key
    assert t2.n_obs == t.n_obs and t2.num_objs == t.num_objs
    img = t.render(0.1)
    assert img.shape == (480, 640, 3)
    t.close()
    t2.close()


def test_checkpoint_restores_full_params(S, stream, tmp_path):
    """A checkpoint of a volume with non-default knobs and Python placement reloads with the
    identical parameter block, and the reloaded volume associates, integrates and renders
    exactly like the one that was saved."""
    from semtsdf import FusionConfig, TSDF

    st, frames = stream
    cfg = FusionConfig(vol_dim=40, placement="python", prior_mrcnn_err_rate=0.07, box_thresh=0.25, gate=0.95,
                       duplicate_thresh=0.4)
    t = TSDF(KI, 40, cfg)
    for k in range(0, 4):
        fr = frames[k]
        t.parse_frame(fr.depth, fr.rgb, fr.w2c, float(np.mean(fr.depth[fr.depth > 0])), fr.mask.copy())
    path = str(tmp_path / "vol.npz")
    t.save(path)
    t2 = TSDF.load(path)
    assert bytes(t.vol.get_params()) == bytes(t2.vol.get_params())
    assert t2.vol.get_params().prior_mrcnn_err_rate == np.float32(0.07) and t2.config.placement == "python"
    assert np.array_equal(t2.intrinsic_inv, t.intrinsic_inv)
    fr = frames[4]
    m1, m2 = fr.mask.copy(), fr.mask.copy()
    s1 = t.parse_frame(fr.depth, fr.rgb, fr.w2c, 1.0, m1)
    s2 = t2.parse_frame(fr.depth, fr.rgb, fr.w2c, 1.0, m2)
    assert np.array_equal(m1, m2) and bytes(s1) == bytes(s2)
    a, b = t.vol.download(hist=True), t2.vol.download(hist=True)
    for key in a:
        assert np.array_equal(a[key], b[key]), key
    assert np.array_equal(t.render(0.2), t2.render(0.2))
    t.close()
    t2.close()


def test_dropin_tail_planes_and_reuse(S, oracle, stream):
    """tsdf_cuda.tsdf_update drop-in: with vol_dim % 8 != 0 the reference's (vol_dim/8)^3
    blocks never reach the last planes (TSDF_Python/tsdf.cu:90), so they stay unchanged;
    a second geometry on the cached handle (new voxel and miu) is re-validated and used."""
    from semtsdf import tsdf_cuda

    st, frames = stream
    D, d8 = 42, 40
    K = np.eye(4, dtype=np.float32)
    K[(0, 1, 0, 1), (0, 1, 2, 2)] = KI
    rng = np.random.default_rng(9)
    n = D ** 3
    for geo in range(2):
        pl = oracle.place(frames[0].depth, np.linalg.inv(K).astype(np.float32), [D] * 3,
                          np.mean(frames[0].depth[frames[0].depth > 0]) / 5000.0 * (1.0 + 0.2 * geo), 0)
        vs, vx, mu = pl["vol_start"], float(pl["voxel"][0]), float(pl["mu"])
        sdf = np.full(n, np.float32(mu), np.float32)
        wt = np.zeros(n, np.int32)
        col = np.zeros(n * 3, np.int32)
        cls = np.zeros(n, np.int32)
        cnt = np.zeros(n, np.int32)
        g = oracle.OGeom([D] * 3, vs, [vx] * 3, mu)
        ost = oracle.OState([D] * 3, np.float32(mu), color_i32=True, vote=True)
        inside = np.zeros((D, D, D), bool)
        inside[:d8, :d8, :d8] = True
        inside = inside.reshape(-1)
        for k in range(1, 4):
            fr = frames[k]
            E = (fr.w2c @ frames[0].c2w).astype(np.float32)
            c_in = fr.gt_ids.astype(np.int32)
            before = [a.copy() for a in (sdf, wt, col, cls, cnt)]
            tsdf_cuda.tsdf_update(sdf, col, wt, cls, cnt, D, vs, vx, mu, K, fr.depth, fr.rgb, c_in, E, 640, 480)
            oracle.integrate(g, ost, K, E, fr.depth, fr.rgb, cls=c_in, flags=0xC)
            for a, b in ((sdf, before[0]), (wt, before[1]), (cls, before[3]), (cnt, before[4])):
                assert np.array_equal(a[~inside].view(np.uint32), b[~inside].view(np.uint32))
            assert np.array_equal(col.reshape(-1, 3)[~inside], before[2].reshape(-1, 3)[~inside])
            assert np.array_equal(sdf[inside].view(np.uint32), ost.sdf[inside].view(np.uint32))
            assert np.array_equal(wt[inside], ost.wt[inside]) and np.array_equal(cls[inside], ost.cls[inside])
            assert np.array_equal(col.reshape(-1, 3)[inside], ost.color.reshape(-1, 3)[inside])
        assert (wt[inside] > 0).sum() > 1000 and (ost.wt[~inside] > 0).sum() > 0  # the tail would be touched


def test_error_paths(S, stream):
    semtsdf, L = S
    st, frames = stream
    p = semtsdf.default_params(16, KI, 640, 480)
    with pytest.raises(semtsdf.SemTSDFError):
        semtsdf.Volume(p, 0)  # not placed: voxel == 0
    semtsdf.place_from_frame(p, frames[0].depth, 2.5, L.PLACE_SFM)
    vol = semtsdf.Volume(p, 0)
    with pytest.raises(semtsdf.SemTSDFError) as e:
        vol.associate(np.ascontiguousarray(frames[1].mask.copy()), np.eye(4, dtype=np.float32))
    assert e.value.code == L.ERR_STATE  # n_obs == 0 (tsdf.cu:426)
    bad = frames[1].mask.copy()
    bad[0, 0] = 40
    # id policy 0: the frame is applied (its observation counted), then ERR_LABEL is reported
    with pytest.raises(semtsdf.SemTSDFError) as e:
        vol.integrate(frames[1].depth, frames[1].rgb, bad, np.eye(4, dtype=np.float32))
    assert e.value.code == L.ERR_LABEL and vol.state().n_obs == 1
    vol.close()
    # SEMTSDF_F_ID_SATURATE: no association mints such an id, so the label is refused, nothing applied
    p.flags |= L.F_ID_SATURATE
    vol = semtsdf.Volume(p, 0)
    with pytest.raises(semtsdf.SemTSDFError) as e:
        vol.integrate(frames[1].depth, frames[1].rgb, bad, np.eye(4, dtype=np.float32))
    assert e.value.code == L.ERR_LABEL and vol.state().n_obs == 0
    vol.close()


@pytest.mark.parametrize("nshards,chunk", [(2, 8), (3, 5), (4, 16), (3, 2), (8, 15)])
def test_sharded_handles_equal_single_volume(S, oracle, stream, nshards, chunk):
    """Z-slab shards on one device: the gathered owned planes equal the
    single-handle volume bit for bit, halo planes equal their owners, and each shard
    equals the C oracle run on the same local plane map."""
    from semtsdf.shard import ShardLayout

    st, frames = stream
    semtsdf, L = S
    dims = (40, 36, 48)
    p, vol, g, ost = make(S, oracle, dims, frames[0], 0x3)
    shards = []
    for sidx in range(nshards):
        q = semtsdf.default_params(64, KI, 640, 480)
        for fld in ("dim", "vol_start", "vol_end", "voxel", "K", "Kinv"):
            getattr(q, fld)[:] = getattr(p, fld)[:]
        q.mu, q.flags = p.mu, p.flags
        q.z_nshards, q.z_shard, q.z_chunk = nshards, sidx, chunk
        shards.append(semtsdf.Volume(q, 0))
    lay = ShardLayout(dims[2], nshards, chunk)
    for k in range(1, 4):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        vol.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
        for sh in shards:
            sh.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
    full = vol.download(hist=True)
    locs = [sh.download(hist=True) for sh in shards]
    for key, extra in (("sdf", ()), ("wt", ()), ("color", (3,)), ("hist", (32,))):
        parts = [lc[key].reshape((dims[0], dims[1], -1) + extra) for lc in locs]
        got = lay.gather(parts, dims[0], dims[1])
        ref = full[key].reshape((dims[0], dims[1], dims[2]) + extra)
        assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), key
        assert lay.check_halo(parts), key
    # one shard against the oracle with the same local plane map
    zmap = lay.local_to_global(1)
    ost1 = oracle.OState(list(dims), p.mu, semantic=True, lz=zmap.size)
    for k in range(1, 4):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        oracle.integrate(g, ost1, list(p.K), E, fr.depth, fr.rgb, fr.gt_ids, flags=0x3, zmap=zmap)
    assert np.array_equal(locs[1]["sdf"].view(np.uint32), ost1.sdf.view(np.uint32))
    assert np.array_equal(locs[1]["hist"], ost1.hist)
    for sh in shards:
        sh.close()
    vol.close()


def _shard_handles(S, p, nshards, chunk):
    semtsdf, L = S
    shards = []
    for sidx in range(nshards):
        q = semtsdf.default_params(64, KI, 640, 480)
        for fld in ("dim", "vol_start", "vol_end", "voxel", "K", "Kinv"):
            getattr(q, fld)[:] = getattr(p, fld)[:]
        q.mu, q.flags = p.mu, p.flags
        q.z_nshards, q.z_shard, q.z_chunk = nshards, sidx, chunk
        shards.append(semtsdf.Volume(q, 0))
    return shards


@pytest.mark.parametrize("nshards,chunk,dimz,exchange", [(2, 8, 64, "allgather"), (3, 5, 64, "min"),
                                                         (4, 16, 64, "allgather"), (1, 64, 64, "min"),
                                                         (8, 63, 512, "min"), (4, 15, 128, "min")])
def test_sharded_pipeline_equals_single_volume(S, oracle, stream, nshards, chunk, dimz, exchange):
    """The Z-sharded association + integrate + raycast protocol (k_shard_*, host
    LocalShardGroup) reproduces the single-volume pipeline bit for bit: relabelled masks,
    decisions, the gathered volume, rendered images and hit distances; with the exchange
    between steps as an all-gather or as an int64 minimum (the all-reduce MIN of the
    distributed group); (8, 63) is the bench's chunking of a 512-plane z axis over 8 shards."""
    from semtsdf.shard import LocalShardGroup, ShardLayout
    from semtsdf.volume import DeviceBuffer

    st, frames = stream
    semtsdf, L = S
    dims = (48, 40, dimz)
    p, vol, g, ost = make(S, oracle, dims, frames[0], 0x3)
    shards = _shard_handles(S, p, nshards, chunk)
    grp = LocalShardGroup(shards, exchange=exchange)
    npx = 640 * 480
    dbuf, rbuf = DeviceBuffer(npx * 2), DeviceBuffer(npx * 3)
    mbufs = [DeviceBuffer(npx) for _ in shards]
    for k in range(1, 6):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        m_single = np.ascontiguousarray(fr.mask.copy())
        stats = vol.parse_frame(fr.depth, fr.rgb, m_single, E)
        dbuf.upload(fr.depth, grp.stream)
        rbuf.upload(fr.rgb, grp.stream)
        for mb in mbufs:
            mb.upload(fr.mask, grp.stream)
        if k >= 2:
            sstats = grp.associate_dev([mb.ptr for mb in mbufs], E, want_stats=True)
            for ss in sstats:
                assert list(ss.assigned_prev) == list(stats.assigned_prev)
                assert ss.num_objs == stats.num_objs and bytes(ss.lut) == bytes(stats.lut)
        for sh, mb in zip(shards, mbufs):
            sh.integrate_dev(dbuf.ptr, rbuf.ptr, mb.ptr, E, grp.stream)
        for mb in mbufs:
            got = np.zeros(npx, np.uint8)
            mb.download(got, grp.stream)
            shards[0].sync()
            assert np.array_equal(got, m_single.reshape(-1)), f"frame {k}"
        for sh in shards:
            assert sh.state().num_objs == vol.state().num_objs and sh.state().n_obs == k
    lay = ShardLayout(dims[2], nshards, chunk)
    full = vol.download(hist=True)
    parts = [sh.download(hist=True)["hist"].reshape(dims[0], dims[1], -1, 32) for sh in shards]
    assert np.array_equal(lay.gather(parts, dims[0], dims[1]), full["hist"].reshape(dims + (32,)))
    dist = float(np.mean(frames[0].depth[frames[0].depth > 0]) / 5000.0)
    for mode in (L.RENDER_LABEL, L.RENDER_COLOR):
        for angle in (0.0, 0.3):
            s2w, c = semtsdf.orbit_camera(list(p.Kinv), angle, dist)
            img, t = vol.raycast(s2w, c, mode, want_t=True)
            simg, stt = grp.raycast(s2w, c, mode, want_t=True)
            assert (t >= 0).mean() > 0.2
            assert np.array_equal(stt.view(np.uint32), t.view(np.uint32)), (mode, angle)
            assert np.array_equal(simg, img), (mode, angle)
    for sh in shards:
        sh.close()
    vol.close()


@pytest.mark.parametrize("dims", [(37, 29, 45), (16, 8, 32), (9, 17, 70)])
@pytest.mark.parametrize("flags", [0x1, 0x4, 0xC])
def test_tiled_layout_roundtrip(S, stream, dims, flags):
    """upload -> download reproduces every array bit for bit through the tiled device layout
    (y not a multiple of 8, z not a multiple of 32: padding rows/planes must stay invisible),
    and integrating on top keeps untouched voxels unchanged."""
    semtsdf, L = S
    st, frames = stream
    p = semtsdf.default_params(64, KI, 640, 480)
    p.dim[0], p.dim[1], p.dim[2] = dims
    semtsdf.place_from_frame(p, frames[0].depth, float(np.mean(frames[0].depth[frames[0].depth > 0])) / 5000.0,
                             L.PLACE_SFM)
    p.flags = flags
    vol = semtsdf.Volume(p, 0)
    n = int(np.prod(dims))
    rng = np.random.default_rng(sum(dims) + flags)
    ci32 = bool(flags & L.F_COLOR_I32)
    up = {
        "sdf": rng.uniform(-1, 1, n).astype(np.float32),
        "wt": rng.integers(0, 2000, n, dtype=np.int32),
        "color": (rng.integers(-5000, 5000, n * 3, dtype=np.int32) if ci32
                  else rng.integers(0, 256, n * 3, dtype=np.uint8)),
    }
    sem = bool(flags & L.F_SEMANTIC)
    vote = bool(flags & L.F_VOTE)
    if sem:
        h = np.zeros((n, L.MAX_OBJECTS), np.uint32)
        idx = rng.integers(0, n, n // 3)
        h[idx, rng.integers(0, L.MAX_OBJECTS, idx.size)] = rng.integers(1, 9, idx.size, dtype=np.uint32)
        up["hist"] = h.reshape(-1)
    if vote:
        up["cls"] = rng.integers(0, 80, n, dtype=np.int32)
        up["cls_cnt"] = rng.integers(0, 7, n, dtype=np.int32)
    vol.upload(**up)
    out = vol.download(hist=sem, cls=vote)
    for k, v in up.items():
        got = out[k]
        if k == "sdf":
            assert np.array_equal(got.view(np.uint32), v.view(np.uint32)), k
        else:
            assert np.array_equal(got.reshape(-1), v.reshape(-1)), k
    vol.close()


def test_full_size_512_semantic_integrate(S, oracle, stream):
    """C3 at its full size (512^3, semantic, culling on, 3 frames of the bench's synthetic
    stream): every array bit-identical to the exhaustive C oracle.  The oracle runs over
    disjoint x-slabs in threads (ctypes releases the GIL; slabs share no voxel)."""
    from concurrent.futures import ThreadPoolExecutor

    st, frames = stream
    p, vol, g, ost = make(S, oracle, (512, 512, 512), frames[0], 0x3)
    slabs = [(x, x + 32) for x in range(0, 512, 32)]
    touched = 0
    with ThreadPoolExecutor(8) as ex:
        for k in range(1, 4):
            fr = frames[k]
            E = (fr.w2c @ frames[0].c2w).astype(np.float32)
            vol.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
            counts = list(ex.map(lambda r: oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, fr.gt_ids,
                                                            flags=0x3, x_range=r), slabs))
            touched += sum(int(c[0]) for c in counts)
    assert touched > 10_000_000  # the surface band and free space in front of it are exercised
    assert_same(vol, ost, hist=True)
    vol.close()


def test_steady_lines_repeated_frames_and_weight_limit(S, oracle, stream):
    """Steady sdf lines (all 1.0f, weights < 2^23) skip their sdf traffic: repeated frames
    make most free-space lines steady; an uploaded state of sdf 1.0 with weights around 2^23
    and 2^24 checks the weight bound of the flag and that uploads clear the flags."""
    st, frames = stream
    p, vol, g, ost = make(S, oracle, (64, 64, 64), frames[0], 0x3)
    for k in (1, 1, 1, 2, 2, 1, 3, 3, 1):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        vol.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, fr.gt_ids, flags=0x3)
    assert (ost.sdf == 1.0).mean() > 0.05  # free space converged to exactly 1.0
    assert_same(vol, ost, hist=True)
    rng = np.random.default_rng(5)
    n = ost.sdf.size
    base = np.where(rng.random(n) < 0.5, (1 << 23) - 3, (1 << 24) - 3).astype(np.int64)
    ost.sdf[:] = np.float32(1.0)
    ost.wt[:] = (base + rng.integers(0, 6, n)).astype(np.int32)
    vol.upload(sdf=ost.sdf, wt=ost.wt)
    for k in (1, 1, 2, 1, 1, 3):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        vol.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, fr.gt_ids, flags=0x3)
    assert_same(vol, ost, hist=True)
    vol.close()


def test_full_free_units_hole_free_frames(S, oracle, stream):
    """Full free units (cull class 3: every voxel in the image with a nonzero depth pixel and
    f == 1, integrated without projection): frames whose depth holes are filled make them
    common; every array stays bit-identical to the exhaustive oracle."""
    from concurrent.futures import ThreadPoolExecutor

    st, frames = stream
    filled = []
    for fr in frames[:4]:
        d = fr.depth.copy()
        d[d == 0] = np.uint16(d[d > 0].max())  # holes become far samples
        filled.append(d)
    p, vol, g, ost = make(S, oracle, (256, 256, 256), frames[0], 0x3)
    vol.set_instrumentation(events=False, count=True)
    slabs = [(x, x + 32) for x in range(0, 256, 32)]
    with ThreadPoolExecutor(8) as ex:
        for k in range(1, 4):
            fr = frames[k]
            E = (fr.w2c @ frames[0].c2w).astype(np.float32)
            vol.integrate(filled[k], fr.rgb, fr.gt_ids, E)
            list(ex.map(lambda r: oracle.integrate(g, ost, list(p.K), E, filled[k], fr.rgb, fr.gt_ids, flags=0x3,
                                                   x_range=r), slabs))
    tm = vol.timing()
    assert tm.full_units > 1000 and tm.free_units >= tm.full_units
    assert_same(vol, ost, hist=True)
    vol.close()


def test_render_stream_beside_association_equals_serial(S, stream):
    """A live view on its own stream beside the next frame's association (both only read the
    volume; the brick-map update is ordered across streams by the library, the integrate waits
    for the view through parse_frame_dev_after) gives the same views, labels and volume as the
    serial order."""
    import torch

    semtsdf, L = S
    st, frames = stream
    dev = torch.device("cuda", 0)
    npx = 640 * 480
    d_in = [torch.from_numpy(fr.depth.reshape(-1).view(np.int16)).to(dev) for fr in frames]
    r_in = [torch.from_numpy(fr.rgb.reshape(-1)).to(dev) for fr in frames]
    m_in = [torch.from_numpy(np.ascontiguousarray(fr.mask).reshape(-1)).to(dev) for fr in frames]
    torch.cuda.synchronize()

    def run(overlap):
        p = semtsdf.default_params(96, KI, 640, 480)
        semtsdf.place_from_frame(p, frames[0].depth, float(np.mean(frames[0].depth[frames[0].depth > 0])) / 5000.0,
                                 L.PLACE_SFM)
        p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
        vol = semtsdf.Volume(p, 0)
        vs = torch.cuda.ExternalStream(vol.stream, device=dev)
        rs = torch.cuda.Stream(device=dev) if overlap else vs
        done, integrated = torch.cuda.Event(), torch.cuda.Event()
        masks = [m.clone() for m in m_in]
        torch.cuda.synchronize()
        views = []
        for k in range(1, len(frames)):
            fr = frames[k]
            E = (fr.w2c @ frames[0].c2w).astype(np.float32)
            vol.parse_frame_dev(d_in[k].data_ptr(), r_in[k].data_ptr(), masks[k].data_ptr(), E,
                                integrate_after_event=done.cuda_event if (overlap and k > 1) else None)
            if overlap:
                integrated.record(vs)
                rs.wait_event(integrated)
            out = torch.zeros(npx * 3, dtype=torch.uint8, device=dev)
            s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.05 * k, 1.5)
            vol.raycast_dev(s2w, c, L.RENDER_LABEL, out.data_ptr(), stream=rs.cuda_stream)
            if overlap:
                done.record(rs)
            views.append(out)
        vol.sync()
        torch.cuda.synchronize()
        state = vol.download(hist=True)
        res = [v.cpu() for v in views], [m.cpu() for m in masks]
        vol.close()
        return res, state

    (va, ma), sa = run(False)
    (vb, mb), sb = run(True)
    assert any(int(v.count_nonzero()) > 0 for v in va)
    for x, y in zip(va + ma, vb + mb):
        assert torch.equal(x, y)
    for key in ("sdf", "wt", "color", "hist"):
        assert np.array_equal(sa[key], sb[key]), key


@pytest.mark.parametrize("D", [96, 160])
def test_parse_frame_view_fused_equals_serial(S, stream, D):
    """semtsdf_parse_frame_view_dev (the live view of the state before the frame rendered in
    the same launch as the frame's association march) gives the same views (images and hit
    distances, label and colour modes), relabelled masks and volume as raycast_dev followed by
    parse_frame_dev, and as the host-pointer parse_frame (whose prepass runs after the
    decision and relabels in place, where the device paths run the prepass beside the march
    and relabel the mask and the pixel records after it); the first frame (no association)
    renders the view alone."""
    import torch

    semtsdf, L = S
    st, frames = stream
    dev = torch.device("cuda", 0)
    npx = 640 * 480
    d_in = [torch.from_numpy(fr.depth.reshape(-1).view(np.int16)).to(dev) for fr in frames]
    r_in = [torch.from_numpy(fr.rgb.reshape(-1)).to(dev) for fr in frames]
    m_in = [torch.from_numpy(np.ascontiguousarray(fr.mask).reshape(-1)).to(dev) for fr in frames]
    torch.cuda.synchronize()

    def run(fused):
        p = semtsdf.default_params(D, KI, 640, 480)
        semtsdf.place_from_frame(p, frames[0].depth, float(np.mean(frames[0].depth[frames[0].depth > 0])) / 5000.0,
                                 L.PLACE_SFM)
        p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
        vol = semtsdf.Volume(p, 0)
        if fused == "fold":  # the frame's mask statistics and depth pyramid in the march launch
            vol.set_instrumentation(events=False, frame_fold=True)
        masks = [m.clone() for m in m_in]
        torch.cuda.synchronize()
        views = []
        for k in range(len(frames)):
            fr = frames[k]
            E = (fr.w2c @ frames[0].c2w).astype(np.float32)
            out = torch.zeros(npx * 3, dtype=torch.uint8, device=dev)
            tt = torch.zeros(npx, dtype=torch.float32, device=dev)
            s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.05 * k, 1.5)
            mode = L.RENDER_COLOR if k % 3 == 2 else L.RENDER_LABEL
            if fused == "host":
                vol.raycast_dev(s2w, c, mode, out.data_ptr(), tt.data_ptr())
                vol.sync()
                m = np.ascontiguousarray(frames[k].mask.copy())
                vol.parse_frame(fr.depth, fr.rgb, m, E)
                masks[k].copy_(torch.from_numpy(m.reshape(-1)))
            elif fused:
                vol.parse_frame_view_dev(d_in[k].data_ptr(), r_in[k].data_ptr(), masks[k].data_ptr(), E, s2w, c, mode,
                                         out.data_ptr(), tt.data_ptr())
            else:
                vol.raycast_dev(s2w, c, mode, out.data_ptr(), tt.data_ptr())
                vol.parse_frame_dev(d_in[k].data_ptr(), r_in[k].data_ptr(), masks[k].data_ptr(), E)
            views += [out, tt]
        vol.sync()
        torch.cuda.synchronize()
        state = vol.download(hist=True)
        res = [v.cpu() for v in views], [m.cpu() for m in masks]
        vol.close()
        return res, state

    (va, ma), sa = run(False)
    assert sum(int(v.count_nonzero()) for v in va[::2]) > 0
    for variant in (True, "fold", "host"):
        (vb, mb), sb = run(variant)
        for x, y in zip(va + ma, vb + mb):
            assert torch.equal(x, y), variant
        for key in ("sdf", "wt", "color", "hist"):
            assert np.array_equal(sa[key], sb[key]), (variant, key)


def test_parse_frame_ragged_image_device_equals_host_and_oracle(S, oracle, stream):
    """A 637 x 479 image (pixel count not a multiple of 4, rows not 4-aligned): the device
    parse path (prepass beside the march, the relabel of mask and pixel records after the
    decision, k_relabel_records' per-pixel path) equals the host-pointer parse_frame and the
    C oracle (masks, object counts, every array)."""
    import torch

    semtsdf, L = S
    st, frames = stream
    Wr, Hr = 637, 479
    dev = torch.device("cuda", 0)
    crop = [(np.ascontiguousarray(fr.depth[:Hr, :Wr]), np.ascontiguousarray(fr.rgb[:Hr, :Wr]),
             np.ascontiguousarray(fr.mask[:Hr, :Wr])) for fr in frames]

    def make_vol():
        p = semtsdf.default_params(64, KI, Wr, Hr)
        semtsdf.place_from_frame(p, crop[0][0], float(np.mean(crop[0][0][crop[0][0] > 0])) / 5000.0, L.PLACE_SFM)
        p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
        return p, semtsdf.Volume(p, 0)

    p, vh = make_vol()
    _, vd = make_vol()
    g = oracle.OGeom.from_params(p)
    ost = oracle.OState([64] * 3, p.mu, semantic=True)
    num = 0
    for k in range(1, len(frames)):
        d, c, m = crop[k]
        E = (frames[k].w2c @ frames[0].c2w).astype(np.float32)
        mh = m.copy()
        vh.parse_frame(d, c, mh, E)
        dd = torch.from_numpy(d.reshape(-1).view(np.int16)).to(dev)
        cd = torch.from_numpy(c.reshape(-1)).to(dev)
        md = torch.from_numpy(m.reshape(-1).copy()).to(dev)
        torch.cuda.synchronize()
        vd.parse_frame_dev(dd.data_ptr(), cd.data_ptr(), md.data_ptr(), E)
        vd.sync()
        m_ref = m.copy()
        if k == 1:
            num = int(m_ref.max()) + 1
        else:
            probs, box = oracle.march_probs(g, list(p.Kinv), E, Wr, Hr, ost.sdf, ost.hist, p.box_thresh)
            m_ref, num, _, _, _ = oracle.filter_overlaps(probs, box, m_ref, k - 1, num, p.prior_mrcnn_err_rate, 0)
        oracle.integrate(g, ost, list(p.K), E, d, c, m_ref, flags=0x3)
        assert np.array_equal(mh, m_ref), f"host mask, frame {k}"
        assert np.array_equal(md.cpu().numpy().reshape(Hr, Wr), m_ref), f"device mask, frame {k}"
        assert vh.state().num_objs == num and vd.state().num_objs == num
    assert_same(vh, ost, hist=True)
    assert_same(vd, ost, hist=True)
    vh.close()
    vd.close()


@pytest.mark.parametrize("D", [64, 128])
def test_gpu_histogram_matches_reference_class_count(S, oracle, D):
    """The HIP label path pinned to the reference's own code: a semantic, ungated volume
    (flags SEMANTIC only, so every touched voxel counts its label) after the first real frame
    equals the class count of src/TSDF_Python/tsdf.py:122-130 executed after the integrate
    block (tests/golden/hist_golden.npz) on every touched voxel whose pixel choice agrees."""
    from test_oracle_golden import hist_golden_check

    semtsdf, L = S
    g = np.load(os.path.join(GOLDEN, "hist_golden.npz"))
    f = np.load(os.path.join(GOLDEN, "frames_tum_fr2.npz"))
    p = semtsdf.default_params(D, KI, 640, 480)
    for i in range(3):
        p.vol_start[i] = g[f"d{D}_vol_start"][i]
        p.vol_end[i] = g[f"d{D}_vol_start"][i] + (D - 1) * g[f"d{D}_voxel"][i]
        p.voxel[i] = g[f"d{D}_voxel"][i]
    p.mu = float(g[f"d{D}_mu"])
    p.flags = L.F_SEMANTIC
    vol = semtsdf.Volume(p, 0)
    vol.integrate(f["depth_a"], f["rgb_a"], np.ascontiguousarray(g["labels"]), g[f"d{D}_E"].astype(np.float32))
    out = vol.download(hist=True)
    assert hist_golden_check(D, out["hist"], out["wt"], oracle) > 10_000
    vol.close()


def test_headless_orbit_views_deterministic(S, oracle, stream, tmp_path):
    """f4: the reference's endless orbit loop (kernel.cpp:101-107, viewer.cu:137-179) headless:
    TSDF.orbit writes the views as PNG files; the sequence is deterministic (two runs give
    identical files), view k is the raycast at angle 0.01 (k + 1), the first view equals the
    oracle's render, and the checkpoint CLI (python -m semtsdf.orbit) writes the same files."""
    from PIL import Image

    from semtsdf import TSDF, FusionConfig
    from semtsdf.orbit import main as orbit_main

    semtsdf, L = S
    st, frames = stream
    t = TSDF(KI, 64, FusionConfig(vol_dim=64))
    for k in range(0, 4):
        fr = frames[k]
        t.parse_frame(fr.depth, fr.rgb, fr.w2c, float(np.mean(fr.depth[fr.depth > 0]) / 5000.0), fr.mask.copy())
    a = t.orbit(5, str(tmp_path / "a"))
    b = t.orbit(5, str(tmp_path / "b"))
    assert [os.path.basename(x) for x in a] == [f"view_{k:05d}.png" for k in range(5)]
    for x, y in zip(a, b):
        assert open(x, "rb").read() == open(y, "rb").read()
    imgs = t.orbit(5)
    for k, (x, img) in enumerate(zip(a, imgs)):
        assert np.array_equal(np.array(Image.open(x))[:, :, ::-1], img)
        assert np.array_equal(img, t.render(0.01 * (k + 1)))
    assert any(int(img.any(axis=-1).sum()) > 1000 for img in imgs)
    p = t.vol.get_params()
    out = t.vol.download(hist=True)
    g = oracle.OGeom.from_params(p)
    s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01, t.mean_depth)
    ref, _ = oracle.render(g, s2w, c, 640, 480, 0, out["sdf"], out["hist"], out["color"])
    assert np.array_equal(imgs[0], ref)
    ck = str(tmp_path / "vol.npz")
    t.save(ck)
    t.close()
    orbit_main([ck, str(tmp_path / "cli"), "--views", "5"])
    for k, x in enumerate(a):
        assert open(x, "rb").read() == open(str(tmp_path / "cli" / f"view_{k:05d}.png"), "rb").read()


def assoc_margins(table, n_labels, thr):
    """Per current label (rows 1..n_labels-1 of the candidate table): the gap between its best
    and second-best candidate, and between its best and the acceptance threshold 3 eps."""
    gaps, thr_gaps = [], []
    for i in range(1, n_labels):
        row = np.sort(table[i, 1:])[::-1]
        if row[0] <= 0.0:
            continue
        if row[0] > thr:  # an accepted candidate: the runner-up must not overtake it
            gaps.append(float(row[0] - row[1]))
        thr_gaps.append(float(abs(row[0] - thr)))
    return gaps, thr_gaps


def test_association_30_frames_f32_pixel_order_rule(S, oracle):
    """a6 over a long stream: 30 frames at 128^3.  Every frame the GPU's decisions (2^-28
    fixed-point sums) equal the reference's own rule, f32 logf sums in pixel order and expf of
    the f32 mean (tsdf.cu:312-349, oracle precision 0), on the same volume state, and so do the
    relabelled masks and object counts.  The smallest best-vs-second and best-vs-3 eps margins
    of the stream are reported (the distance by which f32 rounding would have to move a
    decision)."""
    import json
    from concurrent.futures import ThreadPoolExecutor

    from semtsdf.synth import SyntheticStream

    semtsdf, L = S
    st = SyntheticStream(seed=2, noise=True)
    frames = [st.frame(k) for k in range(31)]
    p, vol, g, ost = make(S, oracle, (128, 128, 128), frames[0], 0x3)
    eps = float(p.prior_mrcnn_err_rate)
    bands = [(y, min(y + 60, 480)) for y in range(0, 480, 60)]
    gaps, thr_gaps, decided = [], [], 0
    num = 0
    for k in range(1, 31):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        m_gpu = np.ascontiguousarray(fr.mask.copy())
        stats = vol.parse_frame(fr.depth, fr.rgb, m_gpu, E)
        m_ref = fr.mask.copy()
        if k == 1:
            num = int(m_ref.max()) + 1
        else:
            probs = np.zeros(640 * 480 * 32, np.float32)
            box = np.zeros(640 * 480 * 32, np.uint8)
            Ki = np.ascontiguousarray(np.array(list(p.Kinv), np.float32))
            E16 = np.ascontiguousarray(E.reshape(16))

            def band(r):
                oracle.lib().oracle_march_probs(oracle._p(g.dims), oracle._p(g.geo), oracle._p(oracle.k9(Ki)),
                                                oracle._p(E16), 640, 480, oracle._p(ost.sdf), oracle._p(ost.hist),
                                                float(p.box_thresh), oracle._p(probs), oracle._p(box), r[0], r[1])

            with ThreadPoolExecutor(8) as ex:
                list(ex.map(band, bands))
            table = np.zeros((32, 32), np.float64)
            m_ref, num, mx, prev, _ = oracle.filter_overlaps(probs, box, m_ref, k - 1, num, eps, precision=0,
                                                             table=table)
            assert np.array_equal(np.array(stats.assigned_prev[:]), prev), k
            assert stats.num_objs == num, k
            a, b = assoc_margins(table, mx, 3.0 * eps)
            gaps += a
            thr_gaps += b
            decided += int((prev >= 0).sum())
        assert np.array_equal(m_gpu, m_ref), f"frame {k}"
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, m_ref, flags=0x3)
    assert decided > 50  # most instances are matched to earlier ids
    rep = {"frames": 30, "dim": 128, "matched_decisions": decided, "candidate_rows": len(gaps),
           "min_best_vs_second": min(gaps), "min_best_vs_3eps": min(thr_gaps),
           "rule": "f32 logf sums in pixel order, expf of the f32 mean (tsdf.cu:312-349)"}
    print("association margins", json.dumps(rep))
    out = os.environ.get("SEMTSDF_REPORT_DIR")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "assoc_margins.json"), "w") as f:
            json.dump(rep, f)
    assert min(gaps) > 1e-6 and min(thr_gaps) > 1e-6
    vol.close()


def test_full_size_256_c2_mode(S, oracle, stream):
    """C2 at its full size: 256^3 TSDF + colour with the NumPy rule (int32 colour, ungated,
    flags 0x4), 4 frames of the synthetic stream, culling on: sdf bits, weights and colours
    identical to the exhaustive C oracle (x-slabs in threads)."""
    from concurrent.futures import ThreadPoolExecutor

    st, frames = stream
    p, vol, g, ost = make(S, oracle, (256, 256, 256), frames[0], 0x4)
    slabs = [(x, x + 32) for x in range(0, 256, 32)]
    touched = 0
    with ThreadPoolExecutor(8) as ex:
        for k in range(1, 5):
            fr = frames[k]
            E = (fr.w2c @ frames[0].c2w).astype(np.float32)
            vol.integrate(fr.depth, fr.rgb, None, E)
            counts = list(ex.map(lambda r: oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, None, flags=0x4,
                                                            x_range=r), slabs))
            touched += sum(int(c[0]) for c in counts)
    assert touched > 1_000_000
    assert_same(vol, ost)
    vol.close()


def test_color_i32_storage_widening(S, oracle, stream):
    """COLOR_I32 volumes (the NumPy rule's int32 colours) store bytes while every colour fits
    [0, 255] and switch to int32 storage when an upload brings other values (negative, > 255)
    or when a weight could reach 2^23 (where the reference's int32 mean wraps).  Integrating
    across both switches stays bit-identical to the oracle's int32 arithmetic."""
    st, frames = stream
    semtsdf, L = S
    dims = (64, 64, 64)
    for case in ("values", "weights"):
        p, vol, g, ost = make(S, oracle, dims, frames[0], 0x4)
        for k in (1, 2):
            fr = frames[k]
            E = (fr.w2c @ frames[0].c2w).astype(np.float32)
            vol.integrate(fr.depth, fr.rgb, None, E)
            oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, None, flags=0x4)
        assert_same(vol, ost)
        narrow_bytes = vol.state().device_bytes
        rng = np.random.default_rng(17)
        if case == "values":  # out-of-byte colours on a few voxels
            c = ost.color.reshape(-1, 3)
            idx = rng.choice(c.shape[0], 5000, replace=False)
            c[idx] = rng.integers(-3000, 3000, (idx.size, 3), dtype=np.int32)
            vol.upload(color=ost.color)
        else:  # weights just below the wrap bound
            ost.wt[:] = np.where(ost.wt > 0, (1 << 23) - 2 + rng.integers(0, 2, ost.wt.size), 0).astype(np.int32)
            vol.upload(wt=ost.wt)
        for k in (3, 4, 5):
            fr = frames[k]
            E = (fr.w2c @ frames[0].c2w).astype(np.float32)
            vol.integrate(fr.depth, fr.rgb, None, E)
            oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, None, flags=0x4)
        assert vol.state().device_bytes > narrow_bytes, case  # int32 storage now
        assert_same(vol, ost)
        assert (ost.color < 0).any() or (ost.wt >= (1 << 23)).any(), case
        vol.close()


def test_async_prepass_integrate_matches_oracle(S, oracle, stream):
    """semtsdf_integrate_dev_async: the frame prepass of frame k+1 on the volume's prep stream
    overlaps the integrate of frame k (two prepass buffer sets used in turn).  Resident frames
    issued back to back, mixed with synchronous integrate_dev calls and a host-pointer
    integrate, give every array bit-identical to the oracle."""
    from semtsdf.volume import DeviceBuffer

    st, frames = stream
    semtsdf, L = S
    p, vol, g, ost = make(S, oracle, (96, 96, 96), frames[0], 0x3)
    npx = 640 * 480
    F = len(frames) - 1
    d, r, m = DeviceBuffer(F * npx * 2), DeviceBuffer(F * npx * 3), DeviceBuffer(F * npx)
    for i, fr in enumerate(frames[1:]):
        d.upload(fr.depth, None, i * npx * 2)
        r.upload(fr.rgb, None, i * npx * 3)
        m.upload(fr.gt_ids, None, i * npx)
    order = [0, 1, 2, 3, 4, 0, 1, 2, 3, 4, 2, 2, 3]
    mode = ["async", "async", "async", "sync", "async", "async", "host", "async", "async", "sync", "async", "async",
            "async"]
    for i, md in zip(order, mode):
        fr = frames[1 + i]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        if md == "async":
            vol.integrate_dev_async(d.ptr + i * npx * 2, r.ptr + i * npx * 3, m.ptr + i * npx, E)
        elif md == "sync":
            vol.integrate_dev(d.ptr + i * npx * 2, r.ptr + i * npx * 3, m.ptr + i * npx, E)
        else:
            vol.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
        oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, fr.gt_ids, flags=0x3)
    vol.sync()
    assert_same(vol, ost, hist=True)
    for b in (d, r, m):
        b.free()
    vol.close()


def test_async_prepass_sharded_equals_sync(S, oracle, stream):
    """The bench's C4 step on a Z-slab shard (semtsdf_integrate_dev_async, the prepass beside
    the previous integrate) leaves every local array bit-identical to the synchronous
    integrate of the same shard."""
    from semtsdf.volume import DeviceBuffer

    st, frames = stream
    semtsdf, L = S
    dims = (72, 64, 96)
    p, vol, g, ost = make(S, oracle, dims, frames[0], 0x3)
    vol.close()
    npx = 640 * 480
    F = len(frames) - 1
    d, r, m = DeviceBuffer(F * npx * 2), DeviceBuffer(F * npx * 3), DeviceBuffer(F * npx)
    for i, fr in enumerate(frames[1:]):
        d.upload(fr.depth, None, i * npx * 2)
        r.upload(fr.rgb, None, i * npx * 3)
        m.upload(fr.gt_ids, None, i * npx)
    for sidx in range(2):
        q = semtsdf.default_params(64, KI, 640, 480)
        for fld in ("dim", "vol_start", "vol_end", "voxel", "K", "Kinv"):
            getattr(q, fld)[:] = getattr(p, fld)[:]
        q.mu, q.flags = p.mu, p.flags
        q.z_nshards, q.z_shard, q.z_chunk = 2, sidx, 15
        va, vb = semtsdf.Volume(q, 0), semtsdf.Volume(q, 0)
        for i in [0, 1, 2, 3, 4, 0, 1, 2]:
            E = (frames[1 + i].w2c @ frames[0].c2w).astype(np.float32)
            va.integrate_dev_async(d.ptr + i * npx * 2, r.ptr + i * npx * 3, m.ptr + i * npx, E)
            vb.integrate_dev(d.ptr + i * npx * 2, r.ptr + i * npx * 3, m.ptr + i * npx, E)
        va.sync()
        vb.sync()
        xa, xb = va.download(hist=True), vb.download(hist=True)
        assert np.count_nonzero(xb["wt"]) > 0
        for key in ("sdf", "wt", "color", "hist"):
            assert np.array_equal(xa[key].view(np.uint8), xb[key].view(np.uint8)), (sidx, key)
        va.close()
        vb.close()
    for b in (d, r, m):
        b.free()


def test_kernel_copy_from_pinned_and_refusal_of_pageable(S):
    """semtsdf_memcpy kind 4 (the copy kernel the live loop uploads frames with) copies from
    pinned host memory bit for bit, and refuses pageable host memory (a kernel reading it would
    fault) with an error instead of launching."""
    import ctypes as C

    import torch

    semtsdf, L = S
    lib = L.load()
    n = 640 * 480 * 6
    h = torch.randint(0, 256, (n,), dtype=torch.uint8).pin_memory()
    d = torch.zeros(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    L.check(lib.semtsdf_memcpy(C.c_void_p(d.data_ptr()), C.c_void_p(h.data_ptr()), n, 4, None))
    torch.cuda.synchronize()
    assert torch.equal(d.cpu(), h)
    pageable = np.zeros(n + 16, np.uint8)
    off = (-pageable.ctypes.data) % 16
    rc = lib.semtsdf_memcpy(C.c_void_p(d.data_ptr()), C.c_void_p(pageable.ctypes.data + off), n, 4, None)
    assert rc != 0 and b"device-accessible" in lib.semtsdf_last_error()
