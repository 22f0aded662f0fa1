"""Surface export: the PLY writer on the CPU; the device export against the
downloaded volume on the GPU."""
import os
import tempfile

import numpy as np
import pytest

KI = (520.9, 521.0, 325.1, 249.7)


def test_ply_round_trip():
    from semtsdf.export import PALETTE, read_ply, write_ply

    rng = np.random.default_rng(0)
    n = 1000
    xyz = rng.normal(size=(n, 3)).astype(np.float32)
    rgb = rng.integers(0, 256, (n, 3), dtype=np.uint8)
    lab = rng.integers(0, 32, n, dtype=np.uint8)
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "s.ply")
        write_ply(f, xyz, rgb, lab)
        r = read_ply(f)
        assert np.array_equal(r["xyz"].view(np.uint32), xyz.view(np.uint32))
        assert np.array_equal(r["rgb"], rgb) and np.array_equal(r["label"], lab)
        write_ply(f, xyz, rgb, lab, color_by_label=True)
        r = read_ply(f)
        want = np.where((lab > 0)[:, None], PALETTE[lab], rgb)
        assert np.array_equal(r["rgb"], want)
    with tempfile.TemporaryDirectory() as d:  # empty cloud
        f = os.path.join(d, "e.ply")
        write_ply(f, np.zeros((0, 3), np.float32), np.zeros((0, 3), np.uint8))
        assert read_ply(f)["xyz"].shape == (0, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("flags,nshards", [(0x3, 1), (0x4, 1), (0x3, 2)])
def test_export_surface_equals_downloaded_volume(flags, nshards):
    """Every voxel with weight >= 1 and |sdf| < 0.2 of the volume after three frames, in the
    reference's flat order, with its colour and histogram argmax -- as selected from the
    downloaded arrays (sharded: the shards' exports concatenated equal the single volume's
    in z-sorted order)."""
    import semtsdf
    from semtsdf import _lib as L
    from semtsdf.synth import SyntheticStream

    semtsdf.load()
    st = SyntheticStream(seed=0)
    frames = [st.frame(k) for k in range(4)]
    p = semtsdf.default_params(64, KI, 640, 480)
    p.dim[0], p.dim[1], p.dim[2] = 48, 40, 64
    semtsdf.place_from_frame(p, frames[0].depth, float(np.mean(frames[0].depth[frames[0].depth > 0])) / 5000.0,
                             L.PLACE_SFM)
    p.flags = flags
    vols = []
    for sidx in range(nshards):
        q = semtsdf.default_params(64, KI, 640, 480)
        for fld in ("dim", "vol_start", "vol_end", "voxel", "K", "Kinv"):
            getattr(q, fld)[:] = getattr(p, fld)[:]
        q.mu, q.flags = p.mu, p.flags
        q.z_nshards, q.z_shard, q.z_chunk = nshards, sidx, 8
        vols.append(semtsdf.Volume(q, 0))
    single = semtsdf.Volume(p, 0) if nshards > 1 else vols[0]
    for k in range(1, 4):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        for v in (vols + [single] if nshards > 1 else vols):
            v.integrate(fr.depth, fr.rgb, np.ascontiguousarray(fr.mask) if flags & 1 else None, E)
    out = single.download(hist=bool(flags & 1))
    D = (48, 40, 64)
    sdf, wt = out["sdf"].reshape(D), out["wt"].reshape(D)
    sel = (wt >= 1) & (np.abs(sdf) < 0.2)
    idx = np.argwhere(sel)
    col = out["color"].reshape(D + (3,))[sel]
    col = np.clip(col, 0, 255).astype(np.uint8)
    lab = np.zeros(idx.shape[0], np.uint8)
    if flags & 1:
        h = out["hist"].reshape(D + (32,))[sel]
        best = np.zeros(idx.shape[0], np.uint32)
        for kk in range(32):  # first maximum, counts > 0 only
            better = h[:, kk] > best
            lab[better] = kk
            best[better] = h[better, kk]
    parts = [semtsdf.export_surface(v) for v in vols]
    got_idx = np.concatenate([e["index"] for e in parts])
    order = np.lexsort((got_idx[:, 2], got_idx[:, 1], got_idx[:, 0]))
    assert idx.shape[0] > 1000
    assert np.array_equal(got_idx[order], idx.astype(np.uint32))
    cat = lambda key: np.concatenate([e[key] for e in parts])[order]
    assert np.array_equal(cat("sdf").view(np.uint32), sdf[sel].view(np.uint32))
    assert np.array_equal(cat("rgb"), col)
    assert np.array_equal(cat("label"), lab)
    start = np.array(list(p.vol_start), np.float32)
    voxel = np.array(list(p.voxel), np.float32)
    want = (idx.astype(np.float64) * voxel.astype(np.float64) + start.astype(np.float64)).astype(np.float32)
    assert np.array_equal(cat("xyz"), want)
    for v in vols:
        v.close()
    if nshards > 1:
        single.close()
