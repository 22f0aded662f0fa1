"""Oracle parity at the benchmarked configurations (SURVEY.md §8 a4-a8 at C3/C4 sizes).

* The observation count of the split calls (ABI 12): frames integrated through
  semtsdf_integrate_dev(_async) -- the bench's integrate-only step -- advance n_obs like every
  integrated frame of the reference (src/SfM_CUDA/tsdf.cu:218-220, first-frame object count
  :463-468), so a following semtsdf_parse_frame_dev associates against the state the reference
  would hold: masks, object counts and every array equal the C oracle run through the same
  frames with filter_overlaps at precision 0 (the reference's f32 pixel-order rule).
* C3 as the bench times its live pipeline: 512^3 semantic volume, 640x480 frames of the bench's
  own stream (seed 1, noise on, poses through the TUM text path), every frame through
  semtsdf_parse_frame_view_dev (k_march_fused: the live view of the state before the frame in
  the launch of the frame's association march).  Against the threaded oracle frame by frame:
  the relabelled masks and object counts (oracle_march_probs in row bands, filter_overlaps
  precision 0), the lagged view's image and hit-distance bits (oracle_render in row bands,
  viewer.cu:17-86), and at the end every array of the volume (x-slabs).
* C4's volume: one association frame of the 1024^3 single volume (tsdf.cu:72-135,304-416)
  against the oracle's 1024^3 state (its histogram pages are only touched near surfaces).
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KI = (520.9, 521.0, 325.1, 249.7)
W, H = 640, 480
NPX = W * H
NT = 16  # oracle threads (the GPU box's CPU share)


@pytest.fixture(scope="module")
def S():
    import semtsdf
    from semtsdf import _lib as L

    semtsdf.load()
    return semtsdf, L


def bench_stream(n):
    """Frames 0..n-1 of the bench's stream and their relative poses through the TUM text path
    (read_traj -> parse_pos -> relative to frame 0, tsdf.cu:217), as bench.run_pipeline."""
    import tempfile

    from semtsdf import pose as P
    from semtsdf import tum
    from semtsdf.synth import SyntheticStream

    st = SyntheticStream(seed=1, noise=True)
    frames = [st.frame(k) for k in range(n)]
    with tempfile.TemporaryDirectory() as d:
        gt = os.path.join(d, "groundtruth.txt")
        with open(gt, "w") as f:
            f.write("\n".join(st.tum_lines(n)) + "\n")
        traj = tum.read_traj(gt)
    ext0_inv = np.linalg.inv(P.parse_pos(traj[0, 1:]))
    Es = [np.ascontiguousarray(P.relative_pose(P.parse_pos(traj[k, 1:]), ext0_inv), np.float32) for k in range(n)]
    return frames, Es


def placed(S, D, f0):
    semtsdf, L = S
    p = semtsdf.default_params(D, KI, W, H)
    semtsdf.place_from_frame(p, f0.depth, float(np.mean(f0.depth[f0.depth > 0])) / 5000.0, L.PLACE_SFM)
    p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
    return p


def bands(n, parts):
    step = (n + parts - 1) // parts
    return [(a, min(a + step, n)) for a in range(0, n, step)]


def oracle_integrate(oracle, ex, g, ost, p, E, fr, mask):
    D = int(g.dims[0])
    return sum(int(c[0]) for c in ex.map(
        lambda r: oracle.integrate(g, ost, list(p.K), E, fr.depth, fr.rgb, mask, flags=0x3, x_range=r),
        bands(D, 2 * NT)))


def oracle_march(oracle, ex, g, p, E, ost):
    probs = np.zeros(NPX * 32, np.float32)
    box = np.zeros(NPX * 32, np.uint8)
    Ki = np.ascontiguousarray(np.array(list(p.Kinv), np.float32))
    E16 = np.ascontiguousarray(np.asarray(E, np.float32).reshape(16))

    def band(r):
        oracle.lib().oracle_march_probs(oracle._p(g.dims), oracle._p(g.geo), oracle._p(oracle.k9(Ki)), oracle._p(E16),
                                        W, H, oracle._p(ost.sdf), oracle._p(ost.hist), float(p.box_thresh),
                                        oracle._p(probs), oracle._p(box), r[0], r[1])

    list(ex.map(band, bands(H, 4 * NT)))
    return probs, box


def oracle_view(oracle, ex, g, s2w, c, mode, ost):
    out = np.zeros(NPX * 3, np.uint8)
    t = np.zeros(NPX, np.float32)
    s16 = np.ascontiguousarray(np.asarray(s2w, np.float32).reshape(16))
    c3 = np.ascontiguousarray(np.asarray(c, np.float32).reshape(3))

    def band(r):
        oracle.lib().oracle_render(oracle._p(g.dims), oracle._p(g.geo), oracle._p(s16), oracle._p(c3), W, H, int(mode),
                                   0, oracle._p(ost.sdf), oracle._p(ost.hist), oracle._p(ost.color), oracle._p(out),
                                   oracle._p(t), r[0], r[1])

    list(ex.map(band, bands(H, 4 * NT)))
    return out.reshape(H, W, 3), t.reshape(H, W)


def assert_slabs_equal(vol, ost, D, step=64):
    """Every array of the volume against the oracle state, downloaded step x-planes at a time."""
    per = D * D
    for x0 in range(0, D, step):
        x1 = min(x0 + step, D)
        got = vol.download_slab(x0, x1, hist=True)
        sl = slice(x0 * per, x1 * per)
        assert np.array_equal(got["sdf"].reshape(-1).view(np.uint32), ost.sdf[sl].view(np.uint32)), ("sdf", x0)
        assert np.array_equal(got["wt"].reshape(-1), ost.wt[sl]), ("wt", x0)
        assert np.array_equal(got["color"].reshape(-1), ost.color[3 * x0 * per:3 * x1 * per]), ("color", x0)
        assert np.array_equal(got["hist"].reshape(-1), ost.hist[32 * x0 * per:32 * x1 * per]), ("hist", x0)


def test_integrate_dev_then_parse_frame_dev_equals_oracle(S, oracle):
    """The bench's C4 semantic leg in small: frames integrated through integrate_dev_async /
    integrate_dev with globally consistent ids (the integrate-only step), then frames with
    per-frame permuted labels through parse_frame_dev.  n_obs counts every integrated frame, the
    first one sets num_objs, and the associations equal the oracle's precision-0 rule on the
    same state; no association term exceeds log(p / n_obs) = 0 (every probability <= n_obs, as in
    the reference), so none of them is forced onto the exact path by the certificate's range."""
    from semtsdf.volume import DeviceBuffer

    semtsdf, L = S
    frames, Es = bench_stream(9)
    D = 128
    p = placed(S, D, frames[0])
    vol = semtsdf.Volume(p, 0)
    g = oracle.OGeom.from_params(p)
    ost = oracle.OState([D] * 3, p.mu, semantic=True)
    bufs = []
    for fr in frames:
        b = (DeviceBuffer(NPX * 2), DeviceBuffer(NPX * 3), DeviceBuffer(NPX))
        b[0].upload(fr.depth, vol.stream)
        b[1].upload(fr.rgb, vol.stream)
        bufs.append(b)
    vol.sync()
    num = n_obs = 0
    with ThreadPoolExecutor(NT) as ex:
        for k in range(1, 5):  # integrate-only frames (ids consistent across frames)
            d, r, m = bufs[k]
            m.upload(frames[k].gt_ids, vol.stream)
            if k % 2:
                vol.integrate_dev_async(d.ptr, r.ptr, m.ptr, Es[k])
            else:
                vol.integrate_dev(d.ptr, r.ptr, m.ptr, Es[k])
            if n_obs == 0:
                num = int(frames[k].gt_ids.max()) + 1
            oracle_integrate(oracle, ex, g, ost, p, Es[k], frames[k], frames[k].gt_ids)
            n_obs += 1
            st = vol.state()
            assert (st.n_obs, st.num_objs) == (n_obs, num), k
        vol.reset_timing()
        for k in range(5, 9):  # semantic frames: association of per-frame labels, relabel, integrate
            d, r, m = bufs[k]
            m.upload(frames[k].mask, vol.stream)
            vol.parse_frame_dev(d.ptr, r.ptr, m.ptr, Es[k])
            got = np.zeros(NPX, np.uint8)
            m.download(got, vol.stream)
            vol.sync()
            probs, box = oracle_march(oracle, ex, g, p, Es[k], ost)
            m_ref, num, _, _, _ = oracle.filter_overlaps(probs, box, frames[k].mask, n_obs, num,
                                                         p.prior_mrcnn_err_rate, precision=0)
            assert np.array_equal(got, m_ref.reshape(-1)), f"frame {k}"
            assert probs.max() <= n_obs  # a reachable state: no count above the observations
            oracle_integrate(oracle, ex, g, ost, p, Es[k], frames[k], m_ref)
            n_obs += 1
            st = vol.state()
            assert (st.n_obs, st.num_objs) == (n_obs, num), k
    tm = vol.timing()
    assert tm.n_assoc == 4 and tm.assoc_pos_max == 0.0
    assert_slabs_equal(vol, ost, D)
    for b in bufs:
        for x in b:
            x.free()
    vol.close()


def test_bench_c3_fused_pipeline_512_equals_oracle(S, oracle):
    """The bench's live C3 frame at its own configuration: 512^3 semantic volume, 640x480
    frames of the bench stream, semtsdf_parse_frame_view_dev per frame with the label view at
    the bench's orbit angle 0.01 (k - 1), four frames (three associations).  Frame by frame
    against the threaded oracle: relabelled mask, object count, the view of the state before the
    frame (image and hit-distance bits); at the end every array."""
    from semtsdf.volume import DeviceBuffer

    semtsdf, L = S
    nfr = 5
    frames, Es = bench_stream(nfr)
    D = 512
    p = placed(S, D, frames[0])
    vol = semtsdf.Volume(p, 0)
    g = oracle.OGeom.from_params(p)
    ost = oracle.OState([D] * 3, p.mu, semantic=True)
    mean_m = float(np.mean(frames[0].depth[frames[0].depth > 0]) / 5000.0)
    d_b, r_b, m_b = DeviceBuffer(NPX * 2), DeviceBuffer(NPX * 3), DeviceBuffer(NPX)
    out_b, t_b = DeviceBuffer(NPX * 3), DeviceBuffer(NPX * 4)
    num = 0
    hits = 0
    with ThreadPoolExecutor(NT) as ex:
        for k in range(1, nfr):
            fr = frames[k]
            d_b.upload(fr.depth, vol.stream)
            r_b.upload(fr.rgb, vol.stream)
            m_b.upload(fr.mask, vol.stream)
            s2w, c = semtsdf.orbit_camera(list(p.Kinv), 0.01 * (k - 1), mean_m)
            vol.parse_frame_view_dev(d_b.ptr, r_b.ptr, m_b.ptr, Es[k], s2w, c, L.RENDER_LABEL, out_b.ptr, t_b.ptr)
            got_m = np.zeros(NPX, np.uint8)
            img = np.zeros(NPX * 3, np.uint8)
            tt = np.zeros(NPX, np.float32)
            m_b.download(got_m, vol.stream)
            out_b.download(img, vol.stream)
            t_b.download(tt, vol.stream)
            vol.sync()
            ref, t_ref = oracle_view(oracle, ex, g, s2w, c, L.RENDER_LABEL, ost)  # the state before frame k
            assert np.array_equal(tt.view(np.uint32), t_ref.reshape(-1).view(np.uint32)), f"view t, frame {k}"
            assert np.array_equal(img, ref.reshape(-1)), f"view image, frame {k}"
            hits += int((t_ref >= 0).sum())
            if k == 1:
                m_ref, num = fr.mask.copy(), int(fr.mask.max()) + 1
            else:
                probs, box = oracle_march(oracle, ex, g, p, Es[k], ost)
                m_ref, num, _, _, _ = oracle.filter_overlaps(probs, box, fr.mask, k - 1, num, p.prior_mrcnn_err_rate,
                                                             precision=0)
            assert np.array_equal(got_m, m_ref.reshape(-1)), f"mask, frame {k}"
            assert vol.state().num_objs == num and vol.state().n_obs == k
            oracle_integrate(oracle, ex, g, ost, p, Es[k], fr, m_ref)
    assert hits > 0.2 * NPX * (nfr - 2)  # the views after the first frame see the scene
    assert_slabs_equal(vol, ost, D)
    for b in (d_b, r_b, m_b, out_b, t_b):
        b.free()
    vol.close()


def test_c4_1024_single_volume_association_equals_oracle(S, oracle):
    """One association frame of C4's 1024^3 single volume: two frames integrated, then frame 3
    through parse_frame_dev; its probabilities (semtsdf_assoc_probs, the back_proj_kernel output),
    relabelled mask and object count equal the oracle's on its 1024^3 state."""
    from semtsdf.volume import DeviceBuffer

    semtsdf, L = S
    frames, Es = bench_stream(4)
    D = 1024
    p = placed(S, D, frames[0])
    vol = semtsdf.Volume(p, 0)
    g = oracle.OGeom.from_params(p)
    ost = oracle.OState([D] * 3, p.mu, semantic=True)
    d_b, r_b, m_b = DeviceBuffer(NPX * 2), DeviceBuffer(NPX * 3), DeviceBuffer(NPX)
    with ThreadPoolExecutor(NT) as ex:
        for k in (1, 2):
            fr = frames[k]
            d_b.upload(fr.depth, vol.stream)
            r_b.upload(fr.rgb, vol.stream)
            m_b.upload(fr.mask, vol.stream)
            vol.parse_frame_dev(d_b.ptr, r_b.ptr, m_b.ptr, Es[k])
            vol.sync()
            if k == 1:
                m_ref, num = fr.mask.copy(), int(fr.mask.max()) + 1
            else:
                probs, box = oracle_march(oracle, ex, g, p, Es[k], ost)
                m_ref, num, _, _, _ = oracle.filter_overlaps(probs, box, fr.mask, 1, num, p.prior_mrcnn_err_rate,
                                                             precision=0)
            oracle_integrate(oracle, ex, g, ost, p, Es[k], fr, m_ref)
        fr = frames[3]
        probs, box = oracle_march(oracle, ex, g, p, Es[3], ost)
    probs_g, box_g = vol.assoc_probs(Es[3])
    assert np.array_equal(probs_g.reshape(-1).view(np.uint32), probs.view(np.uint32))
    assert np.array_equal(box_g.reshape(-1), box)
    assert (probs.reshape(NPX, 32)[:, 1:] > 0).any(axis=1).sum() > 10_000  # the frame sees labelled surfaces
    m_ref, num, _, prev, _ = oracle.filter_overlaps(probs, box, fr.mask, 2, num, p.prior_mrcnn_err_rate, precision=0)
    d_b.upload(fr.depth, vol.stream)
    r_b.upload(fr.rgb, vol.stream)
    m_b.upload(fr.mask, vol.stream)
    vol.parse_frame_dev(d_b.ptr, r_b.ptr, m_b.ptr, Es[3])
    got = np.zeros(NPX, np.uint8)
    m_b.download(got, vol.stream)
    vol.sync()
    assert np.array_equal(got, m_ref.reshape(-1))
    assert vol.state().num_objs == num and vol.state().n_obs == 3
    assert (prev[1:] >= 0).sum() >= 2  # instances matched to earlier ids, not all new
    for b in (d_b, r_b, m_b):
        b.free()
    vol.close()
