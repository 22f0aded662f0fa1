"""C4 rows on the GPU: the distributed Z-slab shard group and the full
1024^3 volume.

* DistShardGroup (semtsdf/shard.py; torch.distributed, RCCL on a multi-GPU node): two ranks
  spawned as separate processes on the one GPU of the test box, gloo carrying the
  collectives (RCCL refuses two ranks on one device).  Every rank runs the sharded
  per-frame pipeline (association protocol + all-reduce of the partial tables, integrate)
  and the sharded raycast; rank 0 also runs the single-volume pipeline.  Relabelled masks,
  association decisions, the gathered volume and the rendered images and hit distances
  must equal the single volume bit for bit, with either exchange (all-reduce MIN of the
  int64 records, or all-gather).
* A 1024^3 semantic volume (144 GiB of state on one GPU) integrated through the HIP path,
  x-slabs checked bit for bit against the C oracle run on those planes only.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KI = (520.9, 521.0, 325.1, 249.7)
DIMS = (48, 40, 64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _params(semtsdf, L, f0, shard=None, nshards=1, chunk=8):
    p = semtsdf.default_params(64, KI, 640, 480)
    p.dim[0], p.dim[1], p.dim[2] = DIMS
    semtsdf.place_from_frame(p, f0.depth, float(np.mean(f0.depth[f0.depth > 0])) / 5000.0, L.PLACE_SFM)
    p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
    if shard is not None:
        p.z_nshards, p.z_shard, p.z_chunk = nshards, shard, chunk
    return p


def _rank(rank, world, port, exchange, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import semtsdf
        from semtsdf import _lib as L
        from semtsdf.shard import DistShardGroup
        from semtsdf.synth import SyntheticStream

        semtsdf.load()
        st = SyntheticStream(seed=0)
        frames = [st.frame(k) for k in range(6)]
        q.put((rank, {force: _rank_pass(semtsdf, L, DistShardGroup, torch, frames, rank, world, exchange, force)
                      for force in (False, True)}))
    finally:
        dist.destroy_process_group()


def _rank_pass(semtsdf, L, DistShardGroup, torch, frames, rank, world, exchange, force):
    """One pass of a rank: force=True sends every association row of the shard group to the exact
    path, so every frame's decision runs DistShardGroup.associate_dev's NEED_PIXELS branch (the
    per-pixel data of every shard, an int32 all-reduce SUM, assoc_apply_exact)."""
    vol = semtsdf.Volume(_params(semtsdf, L, frames[0], rank, world), 0)
    vol.set_instrumentation(events=False, force_exact=force)
    grp = DistShardGroup(vol, exchange=exchange)
    single = semtsdf.Volume(_params(semtsdf, L, frames[0]), 0) if rank == 0 else None
    out = {"masks": [], "luts": [], "single_masks": [], "single_luts": [], "exact_rows": []}
    for k in range(1, 6):
        fr = frames[k]
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        d = torch.from_numpy(fr.depth.view(np.int16)).cuda()
        r = torch.from_numpy(fr.rgb).cuda()
        m = torch.from_numpy(fr.mask.copy()).cuda()
        torch.cuda.synchronize()  # inputs copied by torch's stream before the volume's stream reads them
        if vol.state().n_obs > 0:
            stt = grp.associate_dev(m.data_ptr(), E, want_stats=True)
            out["luts"].append(bytes(stt.lut))
            out["exact_rows"].append(int(stt.exact_rows))
        vol.integrate_dev(d.data_ptr(), r.data_ptr(), m.data_ptr(), E, grp._stream())
        torch.cuda.synchronize()
        out["masks"].append(m.cpu().numpy())
        if single is not None:
            ms = np.ascontiguousarray(fr.mask.copy())
            s1 = single.parse_frame(fr.depth, fr.rgb, ms, E)
            out["single_masks"].append(ms)
            if k >= 2:
                out["single_luts"].append(bytes(s1.lut))
    dist_c = float(np.mean(frames[0].depth[frames[0].depth > 0]) / 5000.0)
    out["images"], out["single_images"] = [], []
    p = vol.params
    for mode in (L.RENDER_LABEL, L.RENDER_COLOR):
        for angle in (0.0, 0.3):
            s2w, c = semtsdf.orbit_camera(list(p.Kinv), angle, dist_c)
            img, t = grp.raycast(s2w, c, mode, want_t=True)
            torch.cuda.synchronize()
            out["images"].append((img.cpu().numpy(), t.cpu().numpy()))
            if single is not None:
                out["single_images"].append(single.raycast(s2w, c, mode, want_t=True))
    torch.cuda.synchronize()
    out["local"] = vol.download(hist=True)
    out["state"] = (int(vol.state().n_obs), int(vol.state().num_objs))
    if single is not None:
        out["single"] = single.download(hist=True)
        out["single_state"] = (int(single.state().n_obs), int(single.state().num_objs))
        single.close()
    vol.close()
    return out


@pytest.mark.parametrize("exchange", ["min", "allgather"])
def test_dist_shard_group_two_ranks_equals_single_volume(exchange):
    """Two gloo ranks, each pass of them: the certified decision, then every row forced onto the
    exact path (the multi-process NEED_PIXELS exchange, shard.py DistShardGroup.associate_dev)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, exchange, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, out = q.get(timeout=240)
        res[rank] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0, f"rank exit code {p.exitcode}"
    for force in (False, True):
        _check_two_ranks({r: res[r][force] for r in (0, 1)}, force)


def _check_two_ranks(res, force):
    from semtsdf.shard import ShardLayout

    r0 = res[0]
    for rank in (0, 1):
        o = res[rank]
        if force:  # every decision took the exchanged exact path on every rank
            assert len(o["exact_rows"]) == 4 and all(x != 0 for x in o["exact_rows"]), o["exact_rows"]
        for k, (m, ms) in enumerate(zip(o["masks"], r0["single_masks"])):
            assert np.array_equal(m.reshape(-1), ms.reshape(-1)), (rank, k)
        assert o["luts"] == r0["single_luts"], rank
        assert o["state"] == r0["single_state"], rank
        for i, ((img, t), (simg, st)) in enumerate(zip(o["images"], r0["single_images"])):
            assert (st >= 0).mean() > 0.2
            dt = (t.view(np.uint32) != st.view(np.uint32))
            di = (img != simg).any(axis=-1)
            assert not dt.any() and not di.any(), (rank, i, int(dt.sum()), int(di.sum()), t[dt][:5], st[dt][:5])
    lay = ShardLayout(DIMS[2], 2, 8)
    for key, extra in (("sdf", ()), ("wt", ()), ("color", (3,)), ("hist", (32,))):
        parts = [res[r]["local"][key].reshape((DIMS[0], DIMS[1], -1) + extra) for r in (0, 1)]
        got = lay.gather(parts, DIMS[0], DIMS[1])
        ref = r0["single"][key].reshape(DIMS + extra)
        assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), key


def _rccl_rank(port, q):
    """One rank of a world-1 RCCL ("nccl") process group: the DistShardGroup paths that only
    run on RCCL (all_gather_into_tensor, the all-reduce MIN/SUM ordered on the volume's stream
    through the ExternalStream), with inputs produced and outputs consumed on a torch stream
    of the caller and no device-wide synchronisation in between (the group orders itself
    against the caller's stream)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        import semtsdf
        from semtsdf import _lib as L
        from semtsdf.shard import DistShardGroup
        from semtsdf.synth import SyntheticStream

        semtsdf.load()
        assert dist.get_backend() == "nccl"
        st = SyntheticStream(seed=0)
        frames = [st.frame(k) for k in range(6)]
        dist_c = float(np.mean(frames[0].depth[frames[0].depth > 0]) / 5000.0)
        res = {}
        user = torch.cuda.Stream()
        for exchange, force in (("min", False), ("allgather", False), ("min", True), ("allgather", True)):
            vol = semtsdf.Volume(_params(semtsdf, L, frames[0], 0, 1), 0)
            # force: every row on the exact path (the NEED_PIXELS branch: assoc_pixels, an int32
            # all-reduce SUM over RCCL, assoc_apply_exact)
            vol.set_instrumentation(events=False, force_exact=force)
            grp = DistShardGroup(vol, exchange=exchange)
            assert grp.nccl
            single = semtsdf.Volume(_params(semtsdf, L, frames[0]), 0)
            masks, smasks, imgs, simgs, xrows = [], [], [], [], []
            with torch.cuda.stream(user):
                for k in range(1, 6):
                    fr = frames[k]
                    E = (fr.w2c @ frames[0].c2w).astype(np.float32)
                    # produced by kernels on the caller's stream, read by the group's stream
                    d = torch.from_numpy(fr.depth.view(np.int16)).cuda().clone()
                    r = torch.from_numpy(fr.rgb).cuda().clone()
                    m = torch.from_numpy(fr.mask.copy()).cuda().add(0)
                    sst = grp.parse_frame_dev(d.data_ptr(), r.data_ptr(), m.data_ptr(), E, want_stats=True)
                    if sst is not None:
                        xrows.append(int(sst.exact_rows))
                    masks.append(m.cpu().numpy())  # consumed on the caller's stream
                    ms = np.ascontiguousarray(fr.mask.copy())
                    single.parse_frame(fr.depth, fr.rgb, ms, E)
                    smasks.append(ms)
                p = vol.params
                for mode in (L.RENDER_LABEL, L.RENDER_COLOR):
                    for angle in (0.0, 0.3):
                        s2w, c = semtsdf.orbit_camera(list(p.Kinv), angle, dist_c)
                        img, t = grp.raycast(s2w, c, mode, want_t=True)
                        imgs.append((img.cpu().numpy(), t.cpu().numpy()))
                        simgs.append(single.raycast(s2w, c, mode, want_t=True))
            torch.cuda.synchronize()
            res[(exchange, force)] = dict(masks=masks, smasks=smasks, imgs=imgs, simgs=simgs, xrows=xrows,
                                 state=(int(vol.state().n_obs), int(vol.state().num_objs)),
                                 sstate=(int(single.state().n_obs), int(single.state().num_objs)),
                                 vol=vol.download(hist=True), single=single.download(hist=True))
            vol.close()
            single.close()
        q.put(("ok", res))
    except Exception as e:  # report to the parent instead of hanging its queue
        import traceback

        q.put(("error", traceback.format_exc() + repr(e)))
    finally:
        dist.destroy_process_group()


def test_dist_shard_group_rccl_world1_equals_single_volume():
    """DistShardGroup on the RCCL backend (world size 1: RCCL refuses two ranks on the one
    GPU of the test box): the sharded association + integrate + composite raycast, with both
    exchanges (all-reduce MIN, all_gather_into_tensor), equal the single volume bit for bit --
    with the certified decision and with every row forced onto the exchanged exact path."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_rccl_rank, args=(_free_port(), q))
    proc.start()
    kind, res = q.get(timeout=240)
    proc.join(timeout=60)
    assert kind == "ok", res
    assert proc.exitcode == 0
    for (exchange, force), o in res.items():
        if force:
            assert len(o["xrows"]) == 4 and all(x != 0 for x in o["xrows"]), o["xrows"]
        for k, (m, ms) in enumerate(zip(o["masks"], o["smasks"])):
            assert np.array_equal(m.reshape(-1), ms.reshape(-1)), (exchange, k)
        assert o["state"] == o["sstate"], exchange
        for i, ((img, t), (simg, st)) in enumerate(zip(o["imgs"], o["simgs"])):
            assert (st >= 0).mean() > 0.2
            assert np.array_equal(t.view(np.uint32), st.view(np.uint32)), (exchange, i)
            assert np.array_equal(img, simg), (exchange, i)
        for key in ("sdf", "wt", "color", "hist"):
            assert np.array_equal(o["vol"][key].view(np.uint8), o["single"][key].view(np.uint8)), (exchange, key)


def test_full_size_1024_semantic_slabs(oracle):
    """C4's volume size on one GPU: 1024^3 semantic (sdf, weight, colour, 32-bin histogram =
    144 GiB), 3 frames of the synthetic stream with culling on; x-slabs through the middle
    and the edges of the frustum equal the C oracle's run on the same planes bit for bit."""
    import semtsdf
    from semtsdf import _lib as L
    from semtsdf.synth import SyntheticStream

    st = SyntheticStream(seed=0)
    frames = [st.frame(k) for k in range(4)]
    p = semtsdf.default_params(1024, KI, 640, 480)
    semtsdf.place_from_frame(p, frames[0].depth, float(np.mean(frames[0].depth[frames[0].depth > 0])) / 5000.0,
                             L.PLACE_SFM)
    p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
    vol = semtsdf.Volume(p, 0)
    assert vol.state().device_bytes > 140 * 2 ** 30
    Es = []
    for fr in frames[1:]:
        E = (fr.w2c @ frames[0].c2w).astype(np.float32)
        Es.append(E)
        vol.integrate(fr.depth, fr.rgb, fr.gt_ids, E)
    g = oracle.OGeom.from_params(p)
    K = list(p.K)
    touched = 0
    for x0 in (96, 508, 900):
        x1 = x0 + 8
        ost = oracle.OState([8, 1024, 1024], p.mu, semantic=True)
        for fr, E in zip(frames[1:], Es):
            touched += int(oracle.integrate_slab(g, ost, K, E, fr.depth, fr.rgb, (x0, x1), mask=fr.gt_ids)[0])
        got = vol.download_slab(x0, x1, hist=True)
        assert np.array_equal(got["sdf"].view(np.uint32), ost.sdf.view(np.uint32)), x0
        assert np.array_equal(got["wt"], ost.wt) and np.array_equal(got["color"], ost.color), x0
        assert np.array_equal(got["hist"], ost.hist), x0
    assert touched > 1_000_000
    vol.close()


def test_c4_full_size_sharded_equals_unsharded():
    """C4 as the north star states it, on one GPU: the 1024^3 semantic volume whole (phase 1,
    144 GiB) and as 8 Z-slab shards of 47-plane chunks (phase 2, LocalShardGroup, the bench's
    chunking; 8 x 18.7 GiB), one after the other.  Three frames through the full per-frame
    pipeline (association raycast + relabel + integrate; sharded: the ray protocol, the
    all-reduce of the partial tables), then label and colour composites at two angles.
    Relabelled masks, object counts, images, hit-distance bits and three x-slabs of every
    array (gathered from the shards' owned planes) are identical."""
    import semtsdf
    from semtsdf import _lib as L
    from semtsdf.shard import LocalShardGroup, ShardLayout
    from semtsdf.synth import SyntheticStream
    from semtsdf.volume import DeviceBuffer

    D, NS, CH = 1024, 8, 47
    st = SyntheticStream(seed=0)
    frames = [st.frame(k) for k in range(4)]
    mean_m = float(np.mean(frames[0].depth[frames[0].depth > 0]) / 5000.0)

    def params(shard=None):
        p = semtsdf.default_params(D, KI, 640, 480)
        semtsdf.place_from_frame(p, frames[0].depth, mean_m, L.PLACE_SFM)
        p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
        if shard is not None:
            p.z_nshards, p.z_shard, p.z_chunk = NS, shard, CH
        return p

    Es = [(fr.w2c @ frames[0].c2w).astype(np.float32) for fr in frames]
    views = [(mode, angle) for mode in (L.RENDER_LABEL, L.RENDER_COLOR) for angle in (0.0, 0.3)]
    xs = (96, 508, 900)
    # phase 1: unsharded
    vol = semtsdf.Volume(params(), 0)
    assert vol.state().device_bytes > 140 * 2 ** 30
    masks1 = []
    for k in range(1, 4):
        m = np.ascontiguousarray(frames[k].mask.copy())
        vol.parse_frame(frames[k].depth, frames[k].rgb, m, Es[k])
        masks1.append(m)
    p1 = vol.params
    imgs1 = [vol.raycast(*semtsdf.orbit_camera(list(p1.Kinv), a, mean_m), mode, want_t=True) for mode, a in views]
    slabs1 = {x: vol.download_slab(x, x + 8, hist=True) for x in xs}
    state1 = (int(vol.state().n_obs), int(vol.state().num_objs))
    vol.close()
    del vol
    # phase 2: eight shards
    shards = [semtsdf.Volume(params(s), 0) for s in range(NS)]
    grp = LocalShardGroup(shards, exchange="min")
    npx = 640 * 480
    dbuf, rbuf = DeviceBuffer(npx * 2), DeviceBuffer(npx * 3)
    mbufs = [DeviceBuffer(npx) for _ in shards]
    for k in range(1, 4):
        dbuf.upload(frames[k].depth, grp.stream)
        rbuf.upload(frames[k].rgb, grp.stream)
        for mb in mbufs:
            mb.upload(frames[k].mask, grp.stream)
        grp.parse_frame_dev(dbuf.ptr, rbuf.ptr, [mb.ptr for mb in mbufs], Es[k])
        for mb in mbufs:
            got = np.zeros(npx, np.uint8)
            mb.download(got, grp.stream)
            shards[0].sync()
            assert np.array_equal(got, masks1[k - 1].reshape(-1)), f"mask of frame {k}"
    for sh in shards:
        assert (int(sh.state().n_obs), int(sh.state().num_objs)) == state1
    assert sum(sh.state().device_bytes for sh in shards) > 140 * 2 ** 30
    for (mode, a), (img, t) in zip(views, imgs1):
        simg, stt = grp.raycast(*semtsdf.orbit_camera(list(p1.Kinv), a, mean_m), mode, want_t=True)
        assert (t >= 0).mean() > 0.2
        assert np.array_equal(stt.view(np.uint32), t.view(np.uint32)), (mode, a)
        assert np.array_equal(simg, img), (mode, a)
    lay = ShardLayout(D, NS, CH)
    for x in xs:
        parts = [sh.download_slab(x, x + 8, hist=True) for sh in shards]
        for key, extra in (("sdf", ()), ("wt", ()), ("color", (3,)), ("hist", (32,))):
            loc = [pt[key].reshape((8, D, -1) + extra) for pt in parts]
            got = lay.gather(loc, 8, D)
            ref = slabs1[x][key].reshape((8, D, D) + extra)
            assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (x, key)
        assert (slabs1[x]["wt"] > 0).sum() > 100_000 or x != 508
    for b in [dbuf, rbuf] + mbufs:
        b.free()
    for sh in shards:
        sh.close()
