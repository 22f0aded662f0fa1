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
                                                            precision=1)
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
        agree = (img == ref).all(axis=-1).mean()
        assert agree >= 0.995, agree
        assert (t >= 0).mean() > 0.2  # the scene is actually hit
        assert np.array_equal(t.view(np.uint32), t_ref.view(np.uint32))
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
    assert (img == ref).all(axis=-1).mean() >= 0.995
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
    """GPU integrate (TSDF+colour mode, NumPy rule: i32 colour, ungated) against the
    executed reference block: |dsdf| <= 1e-4 on all but <= 1e-4 of the voxels."""
    semtsdf, L = S
    g = np.load(os.path.join(GOLDEN, "integrate_d64.npz"))
    f = np.load(os.path.join(GOLDEN, "frames_tum_fr2.npz"))
    frames = [(f["depth_a"], f["rgb_a"]), (f["depth_a"], f["rgb_a"]), (f["depth_b"], f["rgb_b"])]
    D = 64
    n = D ** 3
    p = semtsdf.default_params(D, KI, 640, 480)
    K = np.eye(4, dtype=np.float32)
    K[(0, 1, 0, 1), (0, 1, 2, 2)] = KI
    for i in range(3):
        p.vol_start[i] = g["place_vol_start"][i]
        p.vol_end[i] = g["place_vol_end"][i]
        p.voxel[i] = g["place_voxel"][i]
    p.mu = float(g["place_mu"])
    p.flags = L.F_COLOR_I32
    vol = semtsdf.Volume(p, 0)
    for k, (d, c) in enumerate(frames):
        vol.integrate(d, c, None, g[f"f{k}_E"].astype(np.float32))
        out = vol.download()
        idx = g[f"f{k}_idx"]
        ref_sdf = np.full(n, float(g["place_mu"]))
        ref_sdf[idx] = g[f"f{k}_sdf"]
        ref_wt = np.zeros(n, np.int32)
        ref_wt[idx] = g[f"f{k}_wt"]
        ref_col = np.zeros((n, 3), np.int32)
        ref_col[idx] = g[f"f{k}_color"]
        off = np.abs(out["sdf"] - ref_sdf) > 1e-4
        assert off.mean() <= 1e-4, off.mean()
        assert (out["wt"] != ref_wt).mean() <= 1e-4
        ok = ~off & (out["wt"] == ref_wt)
        assert (out["color"].reshape(-1, 3)[ok] == ref_col[ok]).all(axis=1).mean() >= 0.999
    vol.close()


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


def test_error_paths(S, stream):
    semtsdf, L = S
    st, frames = stream
    p = semtsdf.default_params(16, KI, 640, 480)
    with pytest.raises(semtsdf.SemTSDFError):
        semtsdf.Volume(p, 0)  # not placed: voxel == 0
    semtsdf.place_from_frame(p, frames[0].depth, 2.5, L.PLACE_SFM)
    vol = semtsdf.Volume(p, 0)
    bad = frames[1].mask.copy()
    bad[0, 0] = 40
    with pytest.raises(semtsdf.SemTSDFError) as e:
        vol.integrate(frames[1].depth, frames[1].rgb, bad, np.eye(4, dtype=np.float32))
    assert e.value.code == L.ERR_LABEL
    with pytest.raises(semtsdf.SemTSDFError) as e:
        vol.associate(np.ascontiguousarray(frames[1].mask.copy()), np.eye(4, dtype=np.float32))
    assert e.value.code == L.ERR_STATE  # n_obs == 0 (tsdf.cu:426)
    vol.close()


@pytest.mark.parametrize("nshards,chunk", [(2, 8), (3, 5), (4, 16)])
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


@pytest.mark.parametrize("nshards,chunk", [(2, 8), (3, 5), (4, 16), (1, 64)])
def test_sharded_pipeline_equals_single_volume(S, oracle, stream, nshards, chunk):
    """The Z-sharded association + integrate + raycast protocol (k_shard_*, host
    LocalShardGroup) reproduces the single-volume pipeline bit for bit: relabelled masks,
    decisions, the gathered volume, rendered images and hit distances."""
    from semtsdf.shard import LocalShardGroup, ShardLayout
    from semtsdf.volume import DeviceBuffer

    st, frames = stream
    semtsdf, L = S
    dims = (48, 40, 64)
    p, vol, g, ost = make(S, oracle, dims, frames[0], 0x3)
    shards = _shard_handles(S, p, nshards, chunk)
    grp = LocalShardGroup(shards)
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
            L.check(L.load().semtsdf_shard_note_integrated(sh.handle, L.ptr(mb.ptr), L.ptr(grp.stream)))
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
