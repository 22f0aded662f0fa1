"""GPU: the empty-space octant maps the marches skip with.  The LDS line passes
(k_brick_oct_lds: the dilation folded into the three axis passes) give exactly the maps of the
global-memory passes (k_brick_dilate + k_brick_oct_axis x3), and both equal a NumPy restatement
of the map's definition from the downloaded sdf: brick b is skippable when every voxel of the
bricks b + {0,1}^3 (inside the volume) holds sdf >= voxel/2 (1 + 2^-16); byte o of b's word is
the L-inf distance, capped, to the nearest non-skippable brick of octant o (bit a of o set:
negative along axis a), i.e. min over 0 <= k < cap per axis of max(k, d0(b + s k e))."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KI = (520.9, 521.0, 325.1, 249.7)
CAP = 16  # kBrickDistCap (SEMTSDF_BRICK_DIST_CAP)


@pytest.fixture(scope="module")
def S():
    import semtsdf
    from semtsdf import _lib as L

    semtsdf.load()
    return semtsdf, L


@pytest.fixture(scope="module")
def stream():
    from semtsdf.synth import SyntheticStream

    st = SyntheticStream(seed=3)
    return st, [st.frame(k) for k in range(5)]


def numpy_maps(sdf_xyz: np.ndarray, voxel: float) -> np.ndarray:
    """Octant words from the definition (dims need not be multiples of 8: partial edge bricks)."""
    thr = np.float32(voxel) / np.float32(2.0) * np.float32(1.0 + 2.0 ** -16)
    X, Y, Z = sdf_xyz.shape
    nb = [(X + 7) // 8, (Y + 7) // 8, (Z + 7) // 8]
    pad = np.full((nb[0] * 8, nb[1] * 8, nb[2] * 8), np.inf, np.float32)
    pad[:X, :Y, :Z] = sdf_xyz
    plain = pad.reshape(nb[0], 8, nb[1], 8, nb[2], 8).min(axis=(1, 3, 5))
    bmin = plain.copy()
    for dx in (0, 1):
        for dy in (0, 1):
            for dz in (0, 1):
                sh = np.full_like(plain, np.inf)
                sh[: nb[0] - dx, : nb[1] - dy, : nb[2] - dz] = plain[dx:, dy:, dz:]
                bmin = np.minimum(bmin, sh)
    d0 = np.where(bmin >= thr, CAP, 0).astype(np.int32)
    words = np.zeros(d0.shape, np.uint64)
    for o in range(8):
        d = d0.copy()
        for a in range(3):
            s = -1 if (o >> a) & 1 else 1
            out = d.copy()  # k = 0
            n = d.shape[a]
            for k in range(1, CAP):
                if k >= n:
                    break
                sh = np.full_like(d, 1 << 20)
                src = [slice(None)] * 3
                dst = [slice(None)] * 3
                if s > 0:
                    src[a], dst[a] = slice(k, n), slice(0, n - k)
                else:
                    src[a], dst[a] = slice(0, n - k), slice(k, n)
                sh[tuple(dst)] = d[tuple(src)]
                out = np.minimum(out, np.maximum(k, sh))
            d = out
        words |= d.astype(np.uint64) << np.uint64(8 * o)
    return words.reshape(-1)


@pytest.mark.parametrize("dims", [(96, 96, 96), (120, 88, 136), (64, 160, 40)])
def test_lds_map_passes_equal_global_passes_and_definition(S, stream, dims):
    semtsdf, L = S
    st, frames = stream
    vols = []
    for other in (False, True):
        p = semtsdf.default_params(64, KI, 640, 480)
        p.dim[0], p.dim[1], p.dim[2] = dims
        semtsdf.place_from_frame(p, frames[0].depth, float(np.mean(frames[0].depth[frames[0].depth > 0])) / 5000.0,
                                 L.PLACE_SFM)
        p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
        v = semtsdf.Volume(p, 0)
        v.set_instrumentation(events=False, other_map_passes=other)
        vols.append(v)
    voxel = float(p.voxel[0])
    skippable = []
    for k, fr in enumerate(frames):
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        for v in vols:
            v.integrate(fr.depth, fr.rgb, np.ascontiguousarray(fr.mask), E)
        wa, wb = vols[0].map_words(), vols[1].map_words()
        assert wa is not None and wb is not None
        assert np.array_equal(wa, wb), (dims, k, int(np.count_nonzero(wa != wb)))
        if k in (0, len(frames) - 1):
            s = vols[0].download(wt=False, color=False)["sdf"].reshape(dims)
            ref = numpy_maps(s, voxel)
            assert np.array_equal(wa, ref), (dims, k, int(np.count_nonzero(wa != ref)))
        skippable.append(float(np.mean((wa & np.uint64(0xFF)) > 0)))
    for v in vols:
        v.close()
    # the maps are not trivial: some bricks skippable, some not
    assert 0.0 < skippable[-1] < 1.0, skippable

