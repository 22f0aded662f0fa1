"""Per-rank cost of the Z-sharded raycast composite on ONE GPU: the N shards of the C4
volume (1024^3 semantic, z_chunk 64) live side by side in HBM and are driven by a
LocalShardGroup (the exchange is an in-HBM int64 min instead of RCCL), so the shard
kernels' time / N approximates one rank's share.  Also times the single 1024^3 volume's
raycast for the speed-up baseline.  Usage: python tools/emu_composite.py [N] [views]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-maskrcnn_amd"))
import semtsdf  # noqa: E402
from semtsdf import _lib as L  # noqa: E402
from semtsdf.shard import LocalShardGroup  # noqa: E402
from semtsdf.synth import SyntheticStream  # noqa: E402
from semtsdf.volume import DeviceBuffer  # noqa: E402

KI = (520.9, 521.0, 325.1, 249.7)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
VIEWS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
D = int(os.environ.get("EMU_DIM", "1024"))
st = SyntheticStream(seed=1, noise=True)
f0 = st.frame(0)
frames = [st.frame(k) for k in range(1, 5)]
mean_m = float(np.mean(f0.depth[f0.depth > 0]) / 5000.0)


def params(world, rank):
    p = semtsdf.default_params(D, KI, 640, 480)
    semtsdf.place_from_frame(p, f0.depth, mean_m, L.PLACE_SFM)
    p.flags = L.F_SEMANTIC | L.F_GATE_COLOR
    if world > 1:
        p.z_nshards, p.z_shard, p.z_chunk = world, rank, 64
    return p


npx = 640 * 480
dbuf, rbuf, mbuf = DeviceBuffer(npx * 2), DeviceBuffer(npx * 3), DeviceBuffer(npx)
out = DeviceBuffer(npx * 3)


def feed(vols, stream):
    for fr in frames:
        dbuf.upload(fr.depth, stream)
        rbuf.upload(fr.rgb, stream)
        mbuf.upload(fr.gt_ids, stream)
        E = (fr.w2c @ f0.c2w).astype(np.float32)
        for v in vols:
            v.integrate_dev(dbuf.ptr, rbuf.ptr, mbuf.ptr, E, stream)


# single volume
vol = semtsdf.Volume(params(1, 0), 0)
feed([vol], vol.stream)
vol.sync()
for i in range(2):
    s2w, c = semtsdf.orbit_camera(list(vol.params.Kinv), 0.01 * i, mean_m)
    vol.raycast_dev(s2w, c, L.RENDER_LABEL, out.ptr)
vol.sync()
t0 = time.perf_counter()
for i in range(VIEWS):
    s2w, c = semtsdf.orbit_camera(list(vol.params.Kinv), 0.01 * i, mean_m)
    vol.raycast_dev(s2w, c, L.RENDER_LABEL, out.ptr)
vol.sync()
t_single = (time.perf_counter() - t0) / VIEWS
ref = np.zeros(npx * 3, np.uint8)
out.download(ref, vol.stream)
vol.sync()
vol.close()
print(f"single {D}^3 render: {t_single * 1e3:.3f} ms/view", flush=True)

vols = [semtsdf.Volume(params(N, r), 0) for r in range(N)]
grp = LocalShardGroup(vols, exchange="min")
feed(vols, grp.stream)
vols[0].sync()
for i in range(2):
    s2w, c = semtsdf.orbit_camera(list(vols[0].params.Kinv), 0.01 * i, mean_m)
    grp.raycast_dev(s2w, c, L.RENDER_LABEL, out.ptr)
vols[0].sync()
t0 = time.perf_counter()
for i in range(VIEWS):
    s2w, c = semtsdf.orbit_camera(list(vols[0].params.Kinv), 0.01 * i, mean_m)
    grp.raycast_dev(s2w, c, L.RENDER_LABEL, out.ptr)
vols[0].sync()
t_group = (time.perf_counter() - t0) / VIEWS
got = np.zeros(npx * 3, np.uint8)
out.download(got, grp.stream)
vols[0].sync()
print(f"{N} shards on one GPU: {t_group * 1e3:.3f} ms/view for all shards ({t_group * 1e3 / N:.3f} ms per shard); "
      f"last view identical to the single volume: {bool(np.array_equal(got, ref))}", flush=True)
