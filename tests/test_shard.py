"""Z-slab sharding: layout logic, and a world_size-2 gloo run in which each
rank integrates its shard with the C oracle and rank 0 reassembles the volume, which must
equal the single-volume result bit for bit (integrate is pointwise)."""
import os
import socket

import numpy as np
import pytest

from semtsdf.shard import ShardLayout

KI = (520.9, 521.0, 325.1, 249.7)


def _K():
    K = np.eye(4, dtype=np.float32)
    K[(0, 1, 0, 1), (0, 1, 2, 2)] = KI
    return K


def test_layout_covers_every_plane_once():
    for dimz, n, c in ((64, 2, 8), (64, 4, 16), (100, 3, 7), (512, 8, 32), (37, 1, 37)):
        lay = ShardLayout(dimz, n, c)
        owned = np.concatenate([lay.local_to_global(s)[lay.owned_local(s)] for s in range(n)])
        assert np.array_equal(np.sort(owned), np.arange(dimz))
        for s in range(n):
            g = lay.local_to_global(s)
            # monotone (brick/segment bounds stay conservative); a chunk's halo plane may be the
            # shard's own next chunk's first plane (boustrophedon rounds), integrated identically
            assert np.all(np.diff(g) >= 0)
            assert all(lay.owner(int(z)) == s for z in g[lay.owned_local(s)])


def _frames():
    from semtsdf.synth import SyntheticStream

    st = SyntheticStream(seed=3)
    return [st.frame(k) for k in range(3)]


def _rank_main(rank, world, port, out_q):
    import torch.distributed as dist

    import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        D = 32
        fr = _frames()
        pl = O.place(fr[0].depth, np.linalg.inv(_K()).astype(np.float32), [D] * 3,
                     np.mean(fr[0].depth[fr[0].depth > 0]) / 5000.0, 0)
        g = O.OGeom([D] * 3, pl["vol_start"], pl["voxel"], pl["mu"], pl["vol_end"])
        lay = ShardLayout(D, world, 4)
        zmap = lay.local_to_global(rank)
        st = O.OState([D, D, D], np.float32(pl["mu"]), semantic=True, lz=zmap.size)
        for f in fr[1:]:
            E = (f.w2c @ fr[0].c2w).astype(np.float32)
            O.integrate(g, st, _K(), E, f.depth, f.rgb, f.gt_ids, flags=0x3, zmap=zmap)
        import torch

        local = torch.from_numpy(st.sdf.view(np.int32).copy())
        sizes = [lay.local_planes(s) * D * D for s in range(world)]
        bufs = [torch.zeros(n, dtype=torch.int32) for n in sizes]
        if rank == 0:
            dist.gather(local, bufs, dst=0)
        else:
            dist.gather(local, None, dst=0)
        hist_local = torch.from_numpy(st.hist.view(np.int32).copy())
        hbufs = [torch.zeros(n * 32, dtype=torch.int32) for n in sizes]
        if rank == 0:
            dist.gather(hist_local, hbufs, dst=0)
        else:
            dist.gather(hist_local, None, dst=0)
        # sharded render protocol over gloo: every rank steps its shard, records are
        # all-gathered between steps; the composite must equal the single-volume render
        full_r = O.OState([D] * 3, np.float32(pl["mu"]), semantic=True)
        for f in fr[1:]:
            E = (f.w2c @ fr[0].c2w).astype(np.float32)
            O.integrate(g, full_r, _K(), E, f.depth, f.rgb, f.gt_ids, flags=0x3)
        img, t_img = _shard_render(O, g, full_r, pl, fr, lambda send: _gloo_allgather(dist, send, world), rank, world,
                                   lay.chunk)
        if rank == 0:
            ref, t_ref = _single_render(O, g, full_r, pl, fr)
            out_q.put(("render", bool(np.array_equal(img, ref)), bool(np.array_equal(t_img.view(np.uint32),
                                                                                        t_ref.view(np.uint32))),
                       float((t_ref >= 0).mean())))
        # bench protocol: max over ranks of a per-rank time
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            full = O.OState([D] * 3, np.float32(pl["mu"]), semantic=True)
            for f in fr[1:]:
                E = (f.w2c @ fr[0].c2w).astype(np.float32)
                O.integrate(g, full, _K(), E, f.depth, f.rgb, f.gt_ids, flags=0x3)
            locs = [b.numpy().view(np.float32).reshape(D, D, -1) for b in bufs]
            hl = [b.numpy().view(np.uint32).reshape(D, D, -1, 32) for b in hbufs]
            ok = np.array_equal(lay.gather(locs, D, D).view(np.uint32), full.sdf.reshape(D, D, D).view(np.uint32))
            ok_h = np.array_equal(lay.gather(hl, D, D), full.hist.reshape(D, D, D, 32))
            out_q.put((ok, ok_h, lay.check_halo(locs), float(t.item())))
    finally:
        dist.destroy_process_group()


W, H = 640, 480


def _camera(O, pl, fr):
    Kinv = np.linalg.inv(_K()).astype(np.float32)
    dist = float(np.mean(fr[0].depth[fr[0].depth > 0]) / 5000.0)
    return O.orbit_camera(Kinv.reshape(-1), 0.25, dist)


def _single_render(O, g, st, pl, fr, mode=0):
    s2w, c = _camera(O, pl, fr)
    return O.render(g, s2w, c, W, H, mode, st.sdf, st.hist, st.color)


def _gloo_allgather(dist, send, world):
    import torch

    t = torch.from_numpy(send)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.concatenate([p.numpy() for p in parts])


def _shard_render(O, g, st, pl, fr, allgather, shard, nshards, chunk, mode=0):
    """Drive the 4 protocol steps for one shard; allgather(send) -> gathered records."""
    s2w, c = _camera(O, pl, fr)
    npx = W * H
    state = np.zeros(6 * npx, np.int32)
    send = np.zeros(2 * npx, np.int32)
    gathered = np.zeros(2 * npx * nshards, np.int32)
    for step in range(4):
        O.shard_render_step(g, s2w, c, W, H, mode, st.sdf, st.hist, st.color, step, shard, nshards, chunk, gathered,
                            send, state)
        gathered = allgather(send.copy())
    out = np.zeros(npx * 3, np.uint8)
    t = np.zeros(npx, np.float32)
    O.shard_render_step(g, s2w, c, W, H, mode, st.sdf, st.hist, st.color, 4, shard, nshards, chunk, gathered, send,
                        state, out, t)
    return out.reshape(H, W, 3), t.reshape(H, W)


@pytest.mark.parametrize("nshards,chunk,mode", [(2, 4, 0), (3, 5, 1), (4, 2, 0), (1, 32, 1)])
def test_sharded_render_protocol_equals_single_volume(oracle, nshards, chunk, mode):
    """The split march (SURVEY.md §8e raycast composite) restated in the C oracle: virtual
    shards stepping in lockstep with an in-process all-gather reproduce the single-volume
    render bit for bit (image and hit distance)."""
    O = oracle
    D = 32
    fr = _frames()
    pl = O.place(fr[0].depth, np.linalg.inv(_K()).astype(np.float32), [D] * 3,
                 np.mean(fr[0].depth[fr[0].depth > 0]) / 5000.0, 0)
    g = O.OGeom([D] * 3, pl["vol_start"], pl["voxel"], pl["mu"], pl["vol_end"])
    st = O.OState([D] * 3, np.float32(pl["mu"]), semantic=True)
    for f in fr[1:]:
        E = (f.w2c @ fr[0].c2w).astype(np.float32)
        O.integrate(g, st, _K(), E, f.depth, f.rgb, f.gt_ids, flags=0x3)
    ref, t_ref = _single_render(O, g, st, pl, fr, mode)
    assert (t_ref >= 0).mean() > 0.2
    npx = W * H
    s2w, c = _camera(O, pl, fr)
    states = [np.zeros(6 * npx, np.int32) for _ in range(nshards)]
    sends = [np.zeros(2 * npx, np.int32) for _ in range(nshards)]
    gathered = np.zeros(2 * npx * nshards, np.int32)
    for step in range(4):
        for r in range(nshards):
            O.shard_render_step(g, s2w, c, W, H, mode, st.sdf, st.hist, st.color, step, r, nshards, chunk, gathered,
                                sends[r], states[r])
        gathered = np.concatenate(sends)
    for r in range(nshards):
        out = np.zeros(npx * 3, np.uint8)
        t = np.zeros(npx, np.float32)
        O.shard_render_step(g, s2w, c, W, H, mode, st.sdf, st.hist, st.color, 4, r, nshards, chunk, gathered,
                            sends[r], states[r], out, t)
        assert np.array_equal(out.reshape(H, W, 3), ref), r
        assert np.array_equal(t.view(np.uint32), t_ref.reshape(-1).view(np.uint32)), r


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_sharded_integrate_equals_single_volume():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0, f"rank exit code {p.exitcode}"
    res = {}
    for _ in range(2):
        item = q.get(timeout=10)
        res[item[0] if isinstance(item[0], str) else "integrate"] = item
    ok, ok_h, halo_ok, tmax = res["integrate"]
    assert ok and ok_h and halo_ok
    assert tmax == 2.0
    _, img_ok, t_ok, hit = res["render"]
    assert img_ok and t_ok and hit > 0.2
