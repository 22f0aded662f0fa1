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
            assert np.all(np.diff(g) > 0)  # monotone: brick/segment bounds stay conservative
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
    ok, ok_h, halo_ok, tmax = q.get(timeout=10)
    assert ok and ok_h and halo_ok
    assert tmax == 2.0
